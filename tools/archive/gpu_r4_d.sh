#!/bin/bash
# Round 4: bf16 head v4 — parity, timing split (GEMM-only variant), bf16 PPO
# update; then the config-4 full-share data-parallel test.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4d; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_actor_head_bf16.py > $O/tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; grep -E "PASS|FAIL|Error" $O/tests.log | head -20; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_actor_head_bf16.py > $O/head.log 2>&1
rc=$?; echo "head_rc=$rc"; tail -1 $O/head.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-hg16g}; do
  FWD_ONLY=1 VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/head_$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; tail -1 $O/head_$v.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/bench_ppo.py --precision bf16 --envs 8192 --updates 1 --warmup 1 > $O/ppo_bf16.log 2>&1
rc=$?; echo "ppo rc=$rc"; tail -1 $O/ppo_bf16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -m gpu \
  "tests/test_gpu_ppo_dp.py::test_config4_full_share_two_ranks_vs_oracle_and_one_process" > $O/dp.log 2>&1
rc=$?; echo "dp_rc=$rc"; grep -E "config 4|PASS|FAIL|Error|assert" $O/dp.log | head -20; tail -2 $O/dp.log
exit $rc
