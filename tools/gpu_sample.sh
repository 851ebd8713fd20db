#!/bin/bash
# bf16 SAMPLE-mode rollouts: the bf16 head tests, the PPO GPU tests, then the
# bf16 PPO leg with the fused sample draw (default) and the logits path
# (VMP_BF16_SAMPLE=0), interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sample}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_actor_head_bf16.py tests/test_gpu_ppo.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for s in 1 0; do
    VMP_BF16_SAMPLE=$s timeout -k 10 300 python tools/bench_ppo.py --precision bf16 --updates 2 > $O/ppo_s${s}_$rep.log 2>&1
    rc=$?; echo "sample=$s rep$rep $(tail -1 $O/ppo_s${s}_$rep.log | cut -c1-400)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
