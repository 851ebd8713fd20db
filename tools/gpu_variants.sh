#!/bin/bash
# GPU session: parity suite on the default build, then bench the default build
# and each register-budget variant (build/variants/libvmp_w<W>.so).
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 100 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
for W in ${VARIANTS:-2}; do
  VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_w$W.so timeout -k 10 300 python bench.py --no-cpu --steps 100 > gpurun_out/bench_w$W.log 2>&1
  rc=$?; echo "bench_w${W}_rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
