#!/bin/bash
# fused actor head: NW variants and a GEMM-only timing build
cd "$GRAFT_REPO_ROOT" || exit 1
for nw in 4 8 16; do
  echo "NW=$nw"; VMP_HG_NW=$nw timeout -k 10 200 python tools/bench_actor_head.py 2>&1 | grep -v amdgpu.ids | cut -c1-200 || exit 1
done
echo "GEMM only (default NW)"
VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_hgonly.so timeout -k 10 200 python tools/bench_actor_head.py 2>&1 | grep -v amdgpu.ids | cut -c1-200
