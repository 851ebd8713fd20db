#!/bin/bash
# PPO training throughput (tools/bench_ppo.py), f32 and bf16, with the
# rocprofv3 kernel split and an MFMA-busy PMC pass for each precision.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ppo
for PREC in ${PRECS:-f32 bf16}; do
  timeout -k 10 300 python tools/bench_ppo.py --precision $PREC --envs ${ENVS:-8192} --updates 1 --warmup 1 > gpurun_out/ppo/bench_$PREC.log 2>&1
  rc=$?; echo "bench $PREC rc=$rc"; tail -1 gpurun_out/ppo/bench_$PREC.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppo/kt_$PREC -o run \
    -- python tools/bench_ppo.py --precision $PREC --envs ${ENVS:-8192} --updates 1 --warmup 0 > gpurun_out/ppo/kt_$PREC.log 2>&1
  rc=$?; echo "kt $PREC rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/ppo/pmc_$PREC -o run \
    -- python tools/bench_ppo.py --precision $PREC --envs ${ENVS:-8192} --updates 1 --warmup 0 > gpurun_out/ppo/pmc_$PREC.log 2>&1
  rc=$?; echo "pmc $PREC rc=$rc"; [ $rc -ne 0 ] && exit $rc
done

timeout -k 10 120 python tools/ppo_prof_summary.py gpurun_out/ppo
