#!/bin/bash
# Round-end evidence: whole -m gpu suite, smoke(), the driver's bench command,
# then one rocprofv3 kernel-stats pass over the full bench (all legs, no CPU leg).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/final/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 gpurun_out/final/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
tail -1 gpurun_out/final/bench.log | head -c 700; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/kt -o run \
  -- python bench.py --no-cpu > gpurun_out/final/kt.log 2>&1
rc=$?; echo "kt_rc=$rc"
rm -f gpurun_out/final/kt/run_kernel_trace.csv
exit $rc
