#!/bin/bash
# Round 4: the step-hint test across launch kinds, then the env test file.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_env.py > $O/env_tests.log 2>&1
rc=$?; echo "env tests rc=$rc"; tail -3 $O/env_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/env_tests.log | head -8; exit $rc; }
exit 0
