#!/bin/bash
# Round-3 final evidence at HEAD: the whole -m gpu suite, smoke(), the default
# bench line, rocprofv3 kernel stats + PMC of the headline window and of the C5
# leg, and the C5 workgroup timing (VMP_WGTIME build).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-final}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-300
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
rm -f $O/kt/run_kernel_trace.csv
bash tools/gpu_r3_c5prof.sh ${1:-final}_c5
