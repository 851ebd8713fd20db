#!/bin/bash
# GPU session: parity suite on the default build, then bench each register-budget variant.
mkdir -p gpurun_out
true
rc=$?
echo "tests_rc=$rc" | tee -a gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for W in 1 2 3; do
  VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_w$W.so timeout -k 10 300 python bench.py --no-cpu --steps 100 > gpurun_out/bench_w$W.log 2>&1
  rc=$?
  echo "bench_w${W}_rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
