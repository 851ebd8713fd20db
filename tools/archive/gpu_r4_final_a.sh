#!/bin/bash
# Round 4 evidence, part A: the whole -m gpu suite, smoke(), the driver's
# default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4final}; mkdir -p $O
timeout -k 10 850 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-600
