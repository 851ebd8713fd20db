#!/bin/bash
# PPO training throughput (tools/bench_ppo.py) and its rocprofv3 kernel split.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ppo
timeout -k 10 300 python tools/bench_ppo.py --precision ${PREC:-f32} --envs ${ENVS:-8192} --updates 1 --warmup 1 > gpurun_out/ppo/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/ppo/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppo/kt -o run \
  -- python tools/bench_ppo.py --precision ${PREC:-f32} --envs ${ENVS:-8192} --updates 1 --warmup 0 > gpurun_out/ppo/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; head -25 gpurun_out/ppo/kt/run_kernel_stats.csv | cut -c1-200
exit $rc
