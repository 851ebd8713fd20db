#!/bin/bash
# C5 block kernel A/B: bench_stress per library variant (VARIANTS="name ..." in
# build/variants/libvmp_<name>.so; "main" = the normal build) at 256 and 512
# envs, then PMC passes of the main build (counters of k_env_big<27, true>).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c5v}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
for v in main ${VARIANTS:-}; do
  LP=""; [ "$v" != main ] && LP=$VD/libvmp_$v.so
  for n in 256 512; do
    VMP_LIB_PATH=$LP timeout -k 10 300 python tools/bench_stress.py --envs $n > $O/stress_${v}_$n.log 2>&1 || exit 1
    echo "$v $n: $(grep -v amdgpu.ids $O/stress_${v}_$n.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["kernel_ms"],4), "ms frac", round(d["roofline_frac"],4))')"
  done
done
[ -n "$NOPMC" ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python tools/bench_stress.py --steps 10 > $O/kt.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_CYCLES_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python tools/bench_stress.py --steps 10 > $O/p$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"; [ $rc -ne 0 ] && break
done
python tools/pmc_summary.py $O 512 --kernel "k_env_big<27, true>"
rm -f $O/kt/run_kernel_trace.csv
exit 0
