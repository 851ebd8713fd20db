#!/bin/bash
# Round-3 iteration: the whole -m gpu suite, then the default bench line.
# Usage (gpurun): bash tools/gpu_r3.sh <outdir> [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r3}
mkdir -p $OUT
KARGS=()
[ -n "$2" ] && KARGS=(-k "$2")
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${KARGS[@]}" > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -c 3000 $OUT/bench.log; exit $rc
