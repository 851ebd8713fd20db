#!/bin/bash
# Round 4: bf16 head backward with db's column sum on a side stream (default)
# vs inline (VMP_BF16_DB_STREAM=0): bf16 head + PPO GPU tests, then the bf16
# PPO update timing alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4db}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_actor_head_bf16.py tests/test_gpu_ppo.py > $O/test.log 2>&1
rc=$?; echo "test rc=$rc $(tail -1 $O/test.log)"; [ $rc -ne 0 ] && exit $rc
for s in 0 1 0 1; do
  VMP_BF16_DB_STREAM=$s timeout -k 10 300 python tools/bench_ppo.py --precision bf16 --envs 8192 --updates 2 --warmup 1 > $O/ppo_db$s.log 2>&1
  rc=$?; echo "db_stream=$s rc=$rc $(tail -1 $O/ppo_db$s.log | cut -c1-400)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
