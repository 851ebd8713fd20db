#!/bin/bash
# Round 4: the changed parity tests (stats at V > 1024, act from obs), then the
# PPO f32/bf16 kernel split + MFMA-busy pass (tools/gpu_ppo_prof.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4a; mkdir -p $O
python -c "import bench; print(bench.host_cpus())"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; cat /sys/fs/cgroup/cpu.max 2>/dev/null
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_act_obs.py "tests/test_gpu_env.py::test_large_v_block_kernel_vs_oracle" > $O/tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ppo_prof.sh
