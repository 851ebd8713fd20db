#!/bin/bash
# C5 evidence: rocprofv3 kernel stats + PMC passes of the C5 stress leg (512
# envs), the workgroup timing breakdown (VMP_WGTIME build), 2048-env timing.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c5prof}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/bench_stress.py --steps 20 > $O/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -v amdgpu.ids $O/kt.log | tail -1 | cut -c1-400
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python tools/bench_stress.py --steps 20 > $O/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python tools/pmc_summary.py $O 512 --kernel "k_env_big<40, true>" --write $O/c5_pmc_summary.json | tail -8
rm -f $O/kt/run_kernel_trace.csv
VMP_STAMP_BUF=1 VMP_LIB_PATH=$VD/libvmp_wgtime.so timeout -k 10 200 python tools/wgtime.py 512 > $O/wgtime_512.log 2>&1 || exit 1
grep -v amdgpu.ids $O/wgtime_512.log | tail -30
VMP_STAMP_BUF=1 VMP_LIB_PATH=$VD/libvmp_wgtime.so timeout -k 10 200 python tools/wgtime.py 2048 > $O/wgtime_2048.log 2>&1 || exit 1
exit 0
