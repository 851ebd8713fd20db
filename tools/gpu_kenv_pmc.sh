#!/bin/bash
# k_env issue-mix PMC passes (tools/prof_step.py) for the default library and
# the variants in KV (tools/build_variants.sh names); per-kernel averages into
# gpurun_out/kpmc/<lib>_<pass>.txt. LIST=1 also saves `rocprofv3 -L`.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kpmc
if [ -n "$LIST" ]; then timeout -k 10 60 rocprofv3 -L > gpurun_out/kpmc/list.txt 2>&1; grep -o "SQ_[A-Z0-9_]*" gpurun_out/kpmc/list.txt | sort -u > gpurun_out/kpmc/sq.txt; rm gpurun_out/kpmc/list.txt; fi
V=$PWD/vm-placement-migration-gym_amd/build/variants
P1="${P1:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE}"
for lib in default $KV; do
  if [ $lib = default ]; then unset VMP_LIB_PATH; else export VMP_LIB_PATH=$V/libvmp_$lib.so; fi
  PROF_STEPS=10 timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/kpmc/raw_$lib -o run -- python3 tools/prof_step.py > gpurun_out/kpmc/log_$lib.txt 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/kpmc/log_$lib.txt; exit $rc; }
done
python3 - <<'PY'
import csv, glob, shutil
from collections import defaultdict
d = "gpurun_out/kpmc"
for f in sorted(glob.glob(d + "/raw_*/**/*counter_collection.csv", recursive=True)):
    acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        if "k_env" not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    tag = f.split("/raw_")[1].split("/")[0]
    with open(f"{d}/{tag}.txt", "w") as o:
        for k, c in acc.items():
            o.write(f"{k} dispatches={len(n[k])}\n")
            for cn, v in sorted(c.items()):
                o.write(f"  {cn} {v / len(n[k]):.4g}\n")
    print(tag); print(open(f"{d}/{tag}.txt").read())
for r in glob.glob(d + "/raw_*"):
    shutil.rmtree(r)
PY
