#!/bin/bash
# Phase stamps (-DVMP_STAMPS build) of the headline kernel over the refill
# burst (steps 2001-2050 of phase-aligned envs) and the quiet phase after it
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-bstamps}; mkdir -p $O
LIB=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so
for ff in 2000 2500; do
  VMP_LIB_PATH=$LIB STAMP_TRAIN=1 timeout -k 10 300 python tools/stamps.py 32768 1000 $ff 50 > $O/stamps_$ff.log 2>&1
  rc=$?; echo "ff=$ff rc=$rc"; grep -v amdgpu.ids $O/stamps_$ff.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
