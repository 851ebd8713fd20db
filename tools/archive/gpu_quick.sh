#!/bin/bash
# Quick GPU iteration: env parity suite, phase stamps, bench (no CPU leg), and
# the same bench on each library variant named in $VARIANTS
# (vm-placement-migration-gym_amd/build/variants/libvmp_<v>.so).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
summ() {
  python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1 value', round(d['value']/1e6,2), 'M  frac', round(d['roofline']['frac'],4), 'kern_ms', round(d['roofline']['kernel_ms'],4), 'fused', round(d['fused_rollout']['value']/1e6,1), d['parity']['reward_mae'], d['parity']['counters_equal'])"
}
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$NO_STAMPS" ]; then
  VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so timeout -k 10 300 python tools/stamps.py 8192 1000 > gpurun_out/stamps.log 2>&1
  rc=$?; echo "stamps_rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu --steps 100 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
summ default < gpurun_out/bench.log
for v in ${VARIANTS:-}; do
  VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_$v.so timeout -k 10 300 python bench.py --no-cpu --steps 100 > gpurun_out/bench_$v.log 2>&1
  rc=$?; echo "bench_$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
  summ $v < gpurun_out/bench_$v.log
done
exit 0
