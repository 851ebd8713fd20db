#!/bin/bash
# Phase stamps (diagnostic build) of both env kernels at their bench configs.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LIB=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so
VMP_LIB_PATH=$LIB STAMP_TRAIN=1 timeout -k 10 300 python tools/stamps.py 32768 1000 > gpurun_out/stamps_main.log 2>&1
rc=$?; echo "stamps_main_rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps_main.log; [ $rc -ne 0 ] && exit $rc
exit 0
