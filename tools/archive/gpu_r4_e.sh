#!/bin/bash
# Round 4: bf16 head kernel variants A/B (fwd + bwd kernels alone), two rounds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4e; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
for round in 1 2; do
for v in default $VARIANTS; do
  if [ $v = default ]; then L=""; else L=$VD/libvmp_$v.so; fi
  FWD_ONLY=1 VMP_LIB_PATH=$L timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/head_$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; tail -3 $O/head_$v.log; exit $rc; }
  tail -1 $O/head_$v.log
done
done
