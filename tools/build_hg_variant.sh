#!/bin/bash
# build_hg_variant.sh NAME [hipcc -D flags...]: libvmp.so with the bf16 head
# (vmp_headgemm_bf16.hip) compiled under extra flags, linked with the other
# objects of the normal build -> build/variants/libvmp_NAME.so
set -e
cd "$(dirname "$0")/../vm-placement-migration-gym_amd"
N=$1; shift
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -DVMP_NT_STORE"
mkdir -p build/variants
/opt/rocm/bin/hipcc $FLAGS "$@" -c -o build/variants/$N.hg.o csrc/vmp_headgemm_bf16.hip
/opt/rocm/bin/hipcc $FLAGS -shared -o build/variants/libvmp_$N.so build/obj/vmp_kernels.hip.o \
  build/obj/vmp_policy.hip.o build/obj/vmp_headgemm.hip.o build/variants/$N.hg.o \
  build/obj/vmp_record.hip.o build/obj/vmp_capi.cpp.o
rm -f build/variants/$N.hg.o
