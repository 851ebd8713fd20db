#!/bin/bash
# Build libvmp.so variants for A/B measurement:
#   tools/build_variants.sh name "-DFLAG ..." [name "flags"] ...
# Output: vm-placement-migration-gym_amd/build/variants/libvmp_<name>.so
# (the Makefile's flags plus the extra ones).
cd "$(dirname "$0")/../vm-placement-migration-gym_amd" || exit 1
mkdir -p build/variants
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -DVMP_NT_STORE"
SRC="csrc/vmp_kernels.hip csrc/vmp_policy.hip csrc/vmp_headgemm.hip csrc/vmp_record.hip csrc/vmp_capi.cpp"
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc $FL $2 -shared -o build/variants/libvmp_$1.so $SRC &
  shift 2
done
wait
