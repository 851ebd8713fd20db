#!/bin/bash
# launch-gap diagnostic for each library variant in $GAP_VARIANTS (+ default)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/vm-placement-migration-gym_amd/build/variants
for v in default ${GAP_VARIANTS:-}; do
  if [ $v = default ]; then unset VMP_LIB_PATH; else export VMP_LIB_PATH=$V/libvmp_$v.so; fi
  timeout -k 10 200 python tools/launch_gap.py > gpurun_out/gap_$v.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/gap_$v.log | tail -4; [ $rc -ne 0 ] && exit $rc
done
exit 0
