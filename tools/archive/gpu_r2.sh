#!/bin/bash
# Round-2 iteration: full GPU parity suite, bench (all legs), C5 stamps.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -c 3000 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$NO_STAMPS" ]; then
  VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so \
    timeout -k 10 300 python tools/stamps_big.py 512 2000 bestfit > gpurun_out/c5_stamps.log 2>&1
  rc=$?; echo "stamps_rc=$rc"; grep -v amdgpu.ids gpurun_out/c5_stamps.log
fi
exit 0
