#!/bin/bash
# Ping-pong bf16 head kernel: parity against the two-stage kernel, then the
# FWD_ONLY head bench with each kernel. Usage: bash tools/gpu_pp.sh TAG
set -o pipefail
O=gpurun_out/${1:-pp}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_actor_head_bf16.py -k "ping_pong or fused_matches" > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for pp in ${PPS:-0 2 3 0 2 3}; do
  VMP_HG16_PP=$pp FWD_ONLY=1 timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/hg_pp$pp.log 2>&1
  rc=$?; echo "pp=$pp $(tail -1 $O/hg_pp$pp.log)"; [ $rc -eq 0 ] || exit $rc
done
# the matrix loop alone (build/variants/libvmp_hggo.so: -DVMP_HG16_GEMM_ONLY, outputs wrong)
if [ -f vm-placement-migration-gym_amd/build/variants/libvmp_hggo.so ] && [ -n "$GO" ]; then
  for pp in 0 2 3; do
    VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_hggo.so VMP_HG16_PP=$pp FWD_ONLY=1 \
      timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/hggo_pp$pp.log 2>&1
    rc=$?; echo "gemm-only pp=$pp $(tail -1 $O/hggo_pp$pp.log)"; [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
