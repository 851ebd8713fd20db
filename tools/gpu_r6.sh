#!/bin/bash
# Round-6 GPU check: the named tests first (fail fast), then the whole -m gpu
# suite, smoke(), and the driver's default bench command.
# usage: bash tools/gpu_r6.sh OUTDIR [pytest node ids ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6}; shift; mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread "$@" > $O/first_tests.log 2>&1
  rc=$?; echo "first_rc=$rc"; tail -1 $O/first_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/first_tests.log | head -20; exit $rc; }
fi
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-400
exit 0
