#!/bin/bash
# C5 block-kernel iteration: env parity (wave + block kernels, C5 steady state),
# then the C5 stress timing (512 and 1024 envs) and a rocprofv3 kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c5}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_act_obs.py -x -q --timeout 300 --timeout-method thread > $O/env_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 $O/env_tests.log; [ $rc -ne 0 ] && exit $rc
for n in 512 1024; do
  timeout -k 10 300 python tools/bench_stress.py --envs $n > $O/stress_$n.log 2>&1 || exit 1
  echo "stress $n: $(grep -v amdgpu.ids $O/stress_$n.log | tail -1 | cut -c1-600)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/bench_stress.py > $O/kt.log 2>&1 || exit 1
rm -f $O/kt/run_kernel_trace.csv
grep -h "k_env_big" $O/kt/*kernel_stats.csv | cut -c1-200
exit 0
