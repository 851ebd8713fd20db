#!/bin/bash
# Fit-table rebuild skip: env parity on the new library, A/B against the
# base variant (bench legs, interleaved), then burst / quiet phase stamps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-fitskip}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/env_tests.log 2>&1
rc=$?; echo "env tests rc=$rc: $(tail -1 $O/env_tests.log)"; [ $rc -ne 0 ] && exit $rc
VARIANTS="base new" REPS=2 bash tools/gpu_ab.sh ${1:-fitskip}/ab; rc=$?; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_burst_stamps.sh ${1:-fitskip}/stamps
