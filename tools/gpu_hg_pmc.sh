#!/bin/bash
# PMC passes over the fused actor head (collect shape): default build vs the
# GEMM-only timing build; per-kernel counter sums into gpurun_out/hgpmc/*.txt
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hgpmc
V=$PWD/vm-placement-migration-gym_amd/build/variants
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_COUNT"
for lib in default hgonly; do
  for p in 1 2; do
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    if [ $lib = default ]; then unset VMP_LIB_PATH; else export VMP_LIB_PATH=$V/libvmp_$lib.so; fi
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/hgpmc/raw_${lib}_$p -o run -- python3 tools/hg_prof.py ${SHAPE:-collect} 10 > gpurun_out/hgpmc/log_${lib}_$p.txt 2>&1
    rc=$?; echo "$lib pass $p rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/hgpmc/log_${lib}_$p.txt; exit $rc; }
  done
done
python3 - <<'PY'
import csv, glob, os, shutil
from collections import defaultdict
d = "gpurun_out/hgpmc"
for f in sorted(glob.glob(d + "/raw_*/**/*counter_collection.csv", recursive=True)):
    acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    tag = f.split("/raw_")[1].split("/")[0]
    with open(f"{d}/{tag}.txt", "w") as o:
        for k, c in acc.items():
            o.write(f"{k} dispatches={len(n[k])}\n")
            for cn, v in sorted(c.items()):
                o.write(f"  {cn} {v / len(n[k]):.4g}\n")
    print(open(f"{d}/{tag}.txt").read())
for r in glob.glob(d + "/raw_*"):
    shutil.rmtree(r)
PY
