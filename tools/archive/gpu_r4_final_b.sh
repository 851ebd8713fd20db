#!/bin/bash
# Round 4 evidence, part B: rocprofv3 kernel stats + PMC of the headline window
# (k_env<16, true>), the C5 leg (k_env_big) with its workgroup timing, and the
# PPO updates (f32 / bf16 fused) and PPO eval with MFMA-busy counters.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4fb}; mkdir -p $O
ARGS="--no-cpu --no-ppo --ext-steps 0 --period-steps 0 --nominal-steps 0 --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py $ARGS > $O/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python bench.py $ARGS > $O/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/pmc_summary.py $O 32768 --write $O/traffic.json | tail -4
cp $O/kt/run_kernel_stats.csv $O/headline_kernel_stats.csv; rm -rf $O/kt $O/p1 $O/p2 $O/p3
bash tools/gpu_r3_c5prof.sh ${1:-r4fb}_c5 || exit 1
bash tools/gpu_ppo_prof.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppo/kt_eval -o run -- python tools/prof_ppo_eval.py > $O/eval_kt.log 2>&1
rc=$?; echo "eval kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/ppo/pmc_eval -o run -- python tools/prof_ppo_eval.py > $O/eval_pmc.log 2>&1
rc=$?; echo "eval pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/ppo_prof_summary.py gpurun_out/ppo eval | cut -c1-1500
