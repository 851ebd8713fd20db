#!/bin/bash
# GPU iteration: parity suite, phase stamps, bench (default build).
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
VMP_LIB_PATH=$PWD/vm-placement-migration-gym_amd/build/variants/libvmp_stamps.so timeout -k 10 300 python tools/stamps.py 8192 1000 > gpurun_out/stamps.log 2>&1
rc=$?; echo "stamps_rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 100 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; exit $rc
