#!/bin/bash
# C5 (P1000 / V10000, BestFit kl) at steady state: phase stamps of k_env_big
# (diagnostic build) and the timed stress leg, both after FF fast-forward steps.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FF=${FF:-2000}
VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so \
  timeout -k 10 300 python tools/stamps_big.py 512 $FF bestfit > gpurun_out/c5_stamps.log 2>&1
rc=$?; echo "stamps_rc=$rc"; grep -v amdgpu.ids gpurun_out/c5_stamps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_stress.py --ff $FF > gpurun_out/c5_bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; grep -v amdgpu.ids gpurun_out/c5_bench.log; [ $rc -ne 0 ] && exit $rc
exit 0
