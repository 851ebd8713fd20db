#!/bin/bash
# Round 4: phase stamps (diagnostic build) of the headline kernel, phase-aligned
# quiet / burst windows and the headline's staggered window (per-group wave
# lifetimes); the dW GEMM layouts of the bf16 head backward.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4h}; mkdir -p $O
LIB=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so
VMP_LIB_PATH=$LIB STAMP_TRAIN=1 timeout -k 10 200 python tools/stamps.py 32768 1000 2500 50 > $O/stamps_quiet.log 2>&1
rc=$?; echo "quiet rc=$rc"; grep -v amdgpu.ids $O/stamps_quiet.log | tail -32; [ $rc -ne 0 ] && exit $rc
VMP_LIB_PATH=$LIB STAMP_TRAIN=1 timeout -k 10 200 python tools/stamps.py 32768 1000 2000 50 > $O/stamps_burst.log 2>&1
rc=$?; echo "burst rc=$rc"; grep -v amdgpu.ids $O/stamps_burst.log | tail -32; [ $rc -ne 0 ] && exit $rc
VMP_LIB_PATH=$LIB STAMP_TRAIN=1 STAMP_GROUPS=10 timeout -k 10 200 python tools/stamps.py 32768 1000 3400 50 > $O/stamps_stagger.log 2>&1
rc=$?; echo "stagger rc=$rc"; grep -v amdgpu.ids $O/stamps_stagger.log | tail -40; [ $rc -ne 0 ] && exit $rc
GEMM_AB=1 timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/gemm_ab.log 2>&1
rc=$?; echo "gemm_ab rc=$rc"; tail -1 $O/gemm_ab.log; exit $rc
