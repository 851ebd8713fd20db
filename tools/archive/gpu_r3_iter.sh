#!/bin/bash
# Round-3 kernel iteration: env parity (wave + block kernels), phase stamps of
# the burst window, C5 stress timing and period timing per variant.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/it; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
timeout -k 10 500 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_act_obs.py -x -q --timeout 300 --timeout-method thread > $O/env_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 $O/env_tests.log; [ $rc -ne 0 ] && exit $rc
STAMP_TRAIN=1 VMP_LIB_PATH=$VD/libvmp_stamps.so timeout -k 10 200 python tools/stamps.py 32768 1000 ${SFF:-2000} 50 > $O/stamps.log 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps.log
for v in ${STRESS:-}; do
  VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 300 python tools/bench_stress.py > $O/stress_$v.log 2>&1 || exit 1
  echo "stress $v: $(grep -v amdgpu.ids $O/stress_$v.log | tail -1 | cut -c1-400)"
done
[ -n "$VARIANTS" ] && bash tools/gpu_variants_period.sh
exit 0
