#!/bin/bash
# vmp_actor_mlp_f32: its parity tests, then tools/bench_actor_mlp.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-mlp}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_actor_mlp.py tests/test_gpu_ppo.py > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/bench_actor_mlp.py > $O/bench.log 2>&1
rc=$?; grep -v amdgpu $O/bench.log | tail -6; exit $rc
