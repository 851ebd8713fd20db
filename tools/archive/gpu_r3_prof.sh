#!/bin/bash
# rocprofv3 evidence for the headline window exactly as the driver runs it
# (--steps 20 --warmup 5; the other legs that launch the same kernel are
# switched off so the per-kernel averages are the headline's): one
# --kernel-trace --stats pass, then PMC passes (counters only, one set per
# pass) for HBM bytes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) and waves.
# Then one --kernel-trace --stats pass of the full default bench command.
# Output: gpurun_out/<tag>/{kt,p1..p3,ktfull}; summarise with tools/pmc_summary.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-prof3}; O=gpurun_out/$T; mkdir -p $O
ARGS="--no-cpu --no-ppo --ext-steps 0 --period-steps 0 --nominal-steps 0 --steps ${STEPS:-20} --warmup ${WARMUP:-5}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 300 --timeout-method thread > $O/env_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 $O/env_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py $ARGS > $O/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python bench.py $ARGS > $O/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/pmc_summary.py $O 32768 --write $O/traffic.json | tail -12
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktfull -o run -- python bench.py --gpus 1 --steps 20 --warmup 5 > $O/ktfull.log 2>&1
rc=$?; echo "ktfull rc=$rc"
rm -f $O/ktfull/run_kernel_trace.csv
tail -1 $O/ktfull.log | cut -c1-300
exit $rc
