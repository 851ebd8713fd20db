#!/bin/bash
# PMC passes over the bf16 training head's forward (tools/hg16_prof.py):
# for each CASE "NAME:LIB:ENV" (LIB = default or a build/variants name), three
# passes; per-kernel counter means per dispatch into gpurun_out/$1/NAME.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-hg16pmc}; mkdir -p $O
V=$PWD/vm-placement-migration-gym_amd/build/variants
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
P3="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES TA_TA_BUSY_sum TD_TD_BUSY_sum"
for cs in $CASES; do
  IFS=: read -r name lib envs <<< "$cs"
  L=""; [ "$lib" != default ] && L=$V/libvmp_$lib.so
  for p in 1 2 3; do
    eval C=\$P$p
    env ${envs//,/ } VMP_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/raw_${name}_$p -o run -- python3 tools/hg16_prof.py 65536 4 > $O/log_${name}_$p.txt 2>&1
    rc=$?; echo "$name pass $p rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/log_${name}_$p.txt; exit $rc; }
  done
done
python3 - $O <<'PY'
import csv, glob, os, shutil, sys
from collections import defaultdict
d = sys.argv[1]
res = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
nd = defaultdict(lambda: defaultdict(set))
for f in sorted(glob.glob(d + "/raw_*/**/*counter_collection.csv", recursive=True)):
    name = f.split("/raw_")[1].split("/")[0].rsplit("_", 1)[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:48]
        if "hg16" not in k:
            continue
        res[name][k][r["Counter_Name"]] += float(r["Counter_Value"])
        nd[name][k].add((f, r["Dispatch_Id"]))
for name, ks in res.items():
    with open(f"{d}/{name}.txt", "w") as o:
        for k, c in ks.items():
            n = len({x[1] for x in nd[name][k]}) or 1
            o.write(f"{k} dispatches/pass~{n / 3:.1f}\n")
            for cn, v in sorted(c.items()):
                o.write(f"  {cn} {v / (n / 3):.5g}\n")
    print(name); print(open(f"{d}/{name}.txt").read())
for r in glob.glob(d + "/raw_*"):
    shutil.rmtree(r)
PY
