#!/bin/bash
# Round 4: (1) the period leg over env ages 2 501-3 500 phase-aligned (1 000
# launches) vs the same ages staggered as the headline (10 groups 100 steps
# apart, 100 launches: every age once), to price the phase mixing itself;
# (2) hipBLASLt layouts of the bf16 head backward's dh / dW GEMMs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4g}; mkdir -p $O
timeout -k 10 300 python bench.py --period-only --period-ff 2500 --period-steps 1000 --period-dump $O/aligned_ms.npy > $O/period_aligned.log 2>&1
rc=$?; echo "aligned rc=$rc"; tail -1 $O/period_aligned.log | cut -c1-1200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --period-only --period-groups 10 --period-ff 3400 --period-steps 100 --period-dump $O/stagger_ms.npy > $O/period_stagger.log 2>&1
rc=$?; echo "stagger rc=$rc"; tail -1 $O/period_stagger.log | cut -c1-1200; [ $rc -ne 0 ] && exit $rc
GEMM_AB=1 timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/gemm_ab.log 2>&1
rc=$?; echo "gemm_ab rc=$rc"; tail -1 $O/gemm_ab.log; [ $rc -ne 0 ] && exit $rc
VD=$PWD/vm-placement-migration-gym_amd/build/variants
VARS=${VARIANTS:-hgpre hgp4 hgp4n hgp2n}
for v in default $VARS default; do
  L=""; [ $v != default ] && L=$VD/libvmp_$v.so
  FWD_ONLY=1 VMP_LIB_PATH=$L timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/head_$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; tail -1 $O/head_$v.log; [ $rc -ne 0 ] && exit $rc
done
for v in $VARS; do
  VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_actor_head_bf16.py > $O/test_$v.log 2>&1
  rc=$?; echo "test $v rc=$rc"; tail -1 $O/test_$v.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
