#!/bin/bash
# C5 PMC passes: HBM bytes (FETCH_SIZE, WRITE_SIZE) and the issue mix of the
# per-step k_env_big launches of tools/bench_stress.py (the last 21 dispatches:
# the warm step + 20 timed; the fast-forward rollouts are excluded).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5pmc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d gpurun_out/c5pmc/raw$i -o run -- python3 tools/bench_stress.py --ff 500 > gpurun_out/c5pmc/log$i.txt 2>&1
  rc=$?; echo "pass$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/c5pmc/log$i.txt; exit $rc; }
done
python3 - <<'PY'
import csv, glob, shutil, json
from collections import defaultdict
d = "gpurun_out/c5pmc"
out = {}
for f in sorted(glob.glob(d + "/raw*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "k_env_big" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})[-21:]
    keep = set(ids)
    acc = defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) in keep:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in acc.items():
        out[k] = v / len(ids)
json.dump(out, open(d + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
for r in glob.glob(d + "/raw*"):
    shutil.rmtree(r)
PY
