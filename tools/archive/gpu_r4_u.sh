#!/bin/bash
# Round 4: DPP instead of LDS-pipe shuffles (next-finish min, pairwise leaf
# pairs): env / act / record tests, then same-box A/B vs libvmp_prev.so.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4u}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_env.py tests/test_gpu_record.py tests/test_gpu_exp.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/tests.log | head -8; exit $rc; }
bash tools/gpu_r4_s.sh ${1:-r4u}
