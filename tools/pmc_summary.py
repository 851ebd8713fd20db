"""Summarise tools/gpu_profile.sh output for the per-step env kernel.
Usage: python tools/pmc_summary.py gpurun_out/prof [envs] [--write profiles/traffic.json] [--kernel NAME]

Takes every dispatch of vmp::k_env<16, true> (the launch bench.py times) from the
kernel trace and the counter passes, and reports the average duration and the
HBM bytes per launch with the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md (FETCH_SIZE under-reports wide streaming reads by 2x;
both counters are in KiB)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_env<16, true>"
d = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 32768
vals = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    rows = [r for r in csv.DictReader(open(f)) if KERNEL in r["Kernel_Name"]]
    by_disp = defaultdict(lambda: defaultdict(float))
    for r in rows:  # counters are reported per XCD/dimension instance: sum them
        by_disp[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for disp in by_disp.values():
        for k, v in disp.items():
            vals[k].append(v)
avg = {k: sum(v) / len(v) for k, v in vals.items()}
kt = [r for r in csv.DictReader(open(os.path.join(d, "kt", "run_kernel_trace.csv")))
      if KERNEL in r["Kernel_Name"]]
dur = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt) / len(kt)
out = {"kernel": KERNEL, "envs": N, "dispatches": len(kt), "avg_ns": dur}
out.update(avg)
if "GRBM_GUI_ACTIVE" in avg:
    out["eff_clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / dur
if "SQ_WAVE_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
    out["avg_waves_resident"] = avg["SQ_WAVE_CYCLES"] / avg["SQ_BUSY_CYCLES"]
if "SQ_ACTIVE_INST_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
    # rocprofv3's derived VALUBusy: 100 * SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE
    # (per-XCD GRBM: the summed counter / 8); SQ_ACTIVE_INST_VALU is in quad-cycles
    # per SIMD, so x4 cycles / 4 SIMDs per CU cancel
    out["valu_busy"] = avg["SQ_ACTIVE_INST_VALU"] / 256 / (avg["GRBM_GUI_ACTIVE"] / 8)
if "FETCH_SIZE" in avg:
    out["hbm_read_bytes_corrected"] = 2 * avg["FETCH_SIZE"] * 1024
if "WRITE_SIZE" in avg:
    out["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    t = out["hbm_read_bytes_corrected"] + out["hbm_write_bytes"]
    out["bytes_per_launch"] = t
    out["bytes_per_env_step"] = t / N
    out["hbm_GBps"] = t / dur
print(json.dumps(out, indent=1))
if "--write" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--write") + 1], "w"), indent=1)
