#!/bin/bash
# Round 4: the deep-pipeline bf16 head kernels (BK 32, NS stages) - parity
# tests per variant, then fused-kernel timing, two-stage (VMP_HG16_DEEP=0) vs deep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4n}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
for v in ${VARS:-hgd4 hgd5}; do
  VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_actor_head_bf16.py > $O/test_$v.log 2>&1
  rc=$?; echo "test $v rc=$rc $(tail -1 $O/test_$v.log)"; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/test_$v.log | head -5; exit $rc; }
done
for v in ${VARS:-hgd4 hgd5}; do
  for d in 0 1; do
    VMP_HG16_DEEP=$d FWD_ONLY=1 VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/head_${v}_d$d.log 2>&1
    rc=$?; echo "$v deep=$d rc=$rc $(tail -1 $O/head_${v}_d$d.log)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
