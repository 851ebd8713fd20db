#!/bin/bash
# C5 (P1000 / V10000, BestFit kl) iteration: block-kernel parity tests, the
# steady-state stress leg, and phase stamps of k_env_big (diagnostic build).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FF=${FF:-2000}
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q -k "block or large_v or c5" --timeout 300 --timeout-method thread > gpurun_out/c5_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/c5_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_stress.py --ff $FF > gpurun_out/c5_bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; grep -v amdgpu.ids gpurun_out/c5_bench.log; [ $rc -ne 0 ] && exit $rc
VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so \
  timeout -k 10 300 python tools/stamps_big.py 512 $FF bestfit > gpurun_out/c5_stamps.log 2>&1
rc=$?; echo "stamps_rc=$rc"; grep -v amdgpu.ids gpurun_out/c5_stamps.log
exit 0
