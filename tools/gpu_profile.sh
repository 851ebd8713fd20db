#!/bin/bash
# rocprofv3 evidence for bench.py (the same command the driver runs, minus the
# CPU-baseline leg): one --kernel-trace --stats pass, then PMC passes (counters
# only, one set per pass, no tracing domains) for HBM bytes and wave counters.
# Output: gpurun_out/prof/{kt,p1..p3}; summarise with tools/pmc_summary.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
STEPS=${STEPS:-100}
WARMUP=${WARMUP:-20}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o run \
  -- python bench.py --no-cpu --no-ppo --ext-steps 0 --period-steps 0 --nominal-steps 0 --steps $STEPS --warmup $WARMUP > gpurun_out/prof/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $set --output-format csv -d gpurun_out/prof/p$i -o run \
    -- python bench.py --no-cpu --no-ppo --ext-steps 0 --period-steps 0 --nominal-steps 0 --steps $STEPS --warmup $WARMUP > gpurun_out/prof/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
