#!/bin/bash
# Round 4: XCD-team mapping of the bf16 head kernels (VMP_HG16_TEAM: 0 = one
# column tile per block index, as before) - parity tests, then fused-kernel
# timing per team size.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4m}; mkdir -p $O
L=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_${V:-hgteam}.so
VMP_LIB_PATH=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_actor_head_bf16.py > $O/test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -1 $O/test.log; [ $rc -ne 0 ] && exit $rc
for t in 0 4 2 8 0 4; do
  VMP_HG16_TEAM=$t FWD_ONLY=1 VMP_LIB_PATH=$L timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/head_t$t.log 2>&1
  rc=$?; echo "team $t rc=$rc $(tail -1 $O/head_t$t.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
