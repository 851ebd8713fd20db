#!/bin/bash
# build_variant.sh NAME [hipcc -D flags...]: libvmp.so with vmp_kernels.hip
# compiled under extra flags (A/B timing variants), linked with the other
# objects of the normal build -> build/variants/libvmp_NAME.so
set -e
cd "$(dirname "$0")/../vm-placement-migration-gym_amd"
N=$1; shift
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -DVMP_NT_STORE"
mkdir -p build/variants
# the sources that share vmp_layout.h with the kernels are compiled with the
# variant (a layout change must reach the host side and the recorder too)
/opt/rocm/bin/hipcc $FLAGS "$@" -c -o build/variants/$N.o csrc/vmp_kernels.hip
/opt/rocm/bin/hipcc $FLAGS "$@" -c -o build/variants/$N.capi.o csrc/vmp_capi.cpp
/opt/rocm/bin/hipcc $FLAGS "$@" -c -o build/variants/$N.rec.o csrc/vmp_record.hip
/opt/rocm/bin/hipcc $FLAGS -shared -o build/variants/libvmp_$N.so build/variants/$N.o \
  build/obj/vmp_policy.hip.o build/obj/vmp_headgemm.hip.o build/obj/vmp_headgemm_bf16.hip.o \
  build/variants/$N.rec.o build/variants/$N.capi.o
rm -f build/variants/$N.o build/variants/$N.capi.o build/variants/$N.rec.o
