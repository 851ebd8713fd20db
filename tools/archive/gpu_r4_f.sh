#!/bin/bash
# Round 4: C5 variant (tools/experiments/kl_chain.patch) — parity under the
# variant library, then bench_stress A/B against the default at 512 / 2048 envs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4f; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
for v in $C5_VARIANTS; do
  VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    "tests/test_gpu_env.py::test_c5_steady_state_bestfit_kl_vs_oracle" > $O/c5_parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -1 $O/c5_parity_$v.log; [ $rc -ne 0 ] && exit $rc
done
for round in 1 2; do
for n in 512 2048; do
for v in default $C5_VARIANTS; do
  if [ $v = default ]; then L=""; else L=$VD/libvmp_$v.so; fi
  VMP_LIB_PATH=$L timeout -k 10 300 python tools/bench_stress.py --ff 2000 --envs $n > $O/c5_${v}_$n.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$v $n rc=$rc"; tail -3 $O/c5_${v}_$n.log; exit $rc; }
  echo "$v $n: $(grep -v amdgpu.ids $O/c5_${v}_$n.log | tail -1 | cut -c1-260)"
done; done; done
