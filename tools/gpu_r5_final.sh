#!/bin/bash
# Round-5 closing check: the whole -m gpu suite, smoke(), the headline
# rocprofv3 evidence (kernel trace + PMC passes of the headline window only,
# summarised into gpurun_out/final/traffic.json and used by this run's bench
# line), then the driver's default bench command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
STEPS=20 WARMUP=5 bash tools/gpu_profile.sh > $O/prof.log 2>&1
rc=$?; echo "prof_rc=$rc"; [ $rc -ne 0 ] && { tail $O/prof.log; exit $rc; }
python3 tools/pmc_summary.py gpurun_out/prof 32768 --write $O/traffic.json > /dev/null && cp $O/traffic.json profiles/traffic.json
find gpurun_out/prof/kt -name "*kernel_stats.csv" -exec cp {} $O/headline_kernel_stats.csv \;
rm -rf gpurun_out/prof/kt gpurun_out/prof/p1 gpurun_out/prof/p2 gpurun_out/prof/p3
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-300
exit 0
