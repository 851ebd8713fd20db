#!/bin/bash
# Round 4: register thresholds in the heuristic (P <= 128) + atomic dirty
# marks: env tests, then the headline + period legs twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4r}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_env.py tests/test_gpu_act_obs.py tests/test_gpu_record.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/tests.log | head -8; exit $rc; }
ARGS="--no-cpu --no-ppo --ext-steps 0 --stress-steps 0 --steps 20 --warmup 5"
for i in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/bench$i.log 2>&1
  rc=$?; echo "bench$i rc=$rc"; tail -1 $O/bench$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['period']['mean_ms'], d['period']['ms_by_100_steps'], d['nominal_load']['kernel_ms'], d['fused_rollout']['value'])"; [ $rc -ne 0 ] && exit $rc
done
exit 0
