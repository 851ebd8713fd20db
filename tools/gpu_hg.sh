#!/bin/bash
# fused actor head: parity tests, then the head bench under measurement
# overrides (HG_ENVS: space-separated VAR=value sets, "-" = none) and variant
# builds (HG_VARIANTS, tools/build_variants.sh names) against the unfused path
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_actor_head.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hg_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/hg_tests.log; [ $rc -ne 0 ] && exit $rc
V=$PWD/vm-placement-migration-gym_amd/build/variants
for e in ${HG_ENVS:--}; do
  echo "default $e"; ( [ "$e" != "-" ] && export "$e"; timeout -k 10 200 python tools/bench_actor_head.py 2>&1 | grep -v amdgpu.ids | cut -c1-240 ) || exit 1
done
for v in ${HG_VARIANTS-hgonly}; do
  echo "$v"; VMP_LIB_PATH=$V/libvmp_$v.so timeout -k 10 200 python tools/bench_actor_head.py 2>&1 | grep -v amdgpu.ids | cut -c1-240 || exit 1
done
