#!/bin/bash
# Round 4: bf16 head backward mask test with the last dlogits tile as 4-B pair stores (even A) vs default.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4ja}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
VMP_LIB_PATH=$VD/libvmp_hgls.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_actor_head_bf16.py > $O/test.log 2>&1
rc=$?; echo "test rc=$rc $(tail -1 $O/test.log)"; [ $rc -ne 0 ] && exit $rc
for v in default hgls default hgls; do
  L=""; [ $v != default ] && L=$VD/libvmp_$v.so
  FWD_ONLY=1 VMP_LIB_PATH=$L timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/head_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 $O/head_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
