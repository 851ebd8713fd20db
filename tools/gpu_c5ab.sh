#!/bin/bash
# C5 A/B: bench_stress per library (default + C5_VARIANTS from build/variants)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/vm-placement-migration-gym_amd/build/variants
for v in default $C5_VARIANTS; do
  if [ $v = default ]; then unset VMP_LIB_PATH; else export VMP_LIB_PATH=$V/libvmp_$v.so; fi
  timeout -k 10 300 python tools/bench_stress.py --ff 2000 > gpurun_out/c5ab_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/c5ab_$v.log; exit $rc; }
  grep -v amdgpu.ids gpurun_out/c5ab_$v.log | tail -1 | cut -c1-330
done
