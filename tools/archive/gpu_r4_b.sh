#!/bin/bash
# Round 4: bf16 fused training head — parity tests, the head microbench, and
# the bf16 PPO update fused vs the logits path; plus the round's other changed
# tests and the host probe for the CPU baseline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4b; mkdir -p $O
python -c "import bench; print(bench.host_cpus())"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; cat /sys/fs/cgroup/cpu.max 2>/dev/null
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_actor_head_bf16.py tests/test_gpu_act_obs.py \
  "tests/test_gpu_env.py::test_large_v_block_kernel_vs_oracle" > $O/tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; grep -E "PASS|FAIL|Error|error" $O/tests.log | head -30; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_actor_head_bf16.py > $O/head.log 2>&1
rc=$?; echo "head_rc=$rc"; tail -2 $O/head.log; [ $rc -ne 0 ] && exit $rc
for F in 1 0; do
  VMP_BF16_FUSED=$F timeout -k 10 300 python tools/bench_ppo.py --precision bf16 --envs 8192 --updates 1 --warmup 1 > $O/ppo_bf16_fused$F.log 2>&1
  rc=$?; echo "ppo fused=$F rc=$rc"; tail -1 $O/ppo_bf16_fused$F.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
