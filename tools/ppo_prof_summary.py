"""Summarise tools/gpu_ppo_prof.sh output into small files (the raw per-dispatch
CSVs exceed what a GPU call may bring back):
  gpurun_out/ppo/summary_<prec>.json  kernel-time split by kernel class, and
                                      MFMA-busy per GEMM class from the PMC pass
  gpurun_out/ppo/kernel_stats_<prec>.csv  rocprofv3 --stats table (copied)
Then deletes the raw trace / counter directories.

MFMA utilisation of a kernel class = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
GRBM_GUI_ACTIVE / 8): the MFMA busy counter adds the matrix-pipe busy cycles of
every SIMD (32 per v_mfma_f32_32x32x16_bf16, MI355X_MICROARCH.md), and
GRBM_GUI_ACTIVE adds the GPU-busy cycles of the 8 XCDs, so GRBM / 8 is the
kernels' wall time in cycles. (gfx950 ships no derived-counter formulas,
MI355X_MICROARCH.md §rocprofv3 PMC slots; this ratio is the definition used
here.)
Usage: python tools/ppo_prof_summary.py gpurun_out/ppo
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def kclass(name):
    if name.startswith("Cijk_"):
        return "hipBLASLt GEMM"
    if "k_head_fwd" in name:
        return "head forward (HIP)"
    if "k_head_bwd" in name:
        return "head backward (HIP)"
    if "k_hg16" in name or "k_dsum" in name:
        return "fused bf16 GEMM + head, training (HIP)"
    if "k_head_gemm" in name or "k_hg_" in name:
        return "fused GEMM + head (HIP)"
    if "k_env" in name:
        return "env step (HIP)"
    if "k_rowsum" in name or "k_gae" in name:
        return "head sums / GAE (HIP)"
    return "torch elementwise / reduce / other"


def main():
    d = sys.argv[1]
    for prec in sys.argv[2:] or ("f32", "bf16"):
        out = {}
        st = os.path.join(d, f"kt_{prec}", "run_kernel_stats.csv")
        if os.path.exists(st):
            shutil.copy(st, os.path.join(d, f"kernel_stats_{prec}.csv"))
            rows = list(csv.DictReader(open(st)))
            tot = sum(float(r["TotalDurationNs"]) for r in rows)
            split = defaultdict(float)
            for r in rows:
                split[kclass(r["Name"])] += float(r["TotalDurationNs"])
            out["kernel_ms_total"] = tot / 1e6
            out["split_ms"] = {k: v / 1e6 for k, v in sorted(split.items(), key=lambda x: -x[1])}
        pm = os.path.join(d, f"pmc_{prec}", "run_counter_collection.csv")
        if os.path.exists(pm):
            acc = defaultdict(lambda: defaultdict(float))
            for r in csv.DictReader(open(pm)):
                acc[kclass(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
            out["pmc"] = {}
            for k, c in acc.items():
                busy = c.get("SQ_BUSY_CYCLES", 0.0)
                mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
                grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
                out["pmc"][k] = {"SQ_VALU_MFMA_BUSY_CYCLES": mf, "SQ_BUSY_CYCLES": busy,
                                 "GRBM_GUI_ACTIVE": grbm,
                                 "mfma_util": mf / (1024 * grbm / 8) if grbm else None}
        json.dump(out, open(os.path.join(d, f"summary_{prec}.json"), "w"), indent=1)
        for sub in (f"kt_{prec}", f"pmc_{prec}"):
            shutil.rmtree(os.path.join(d, sub), ignore_errors=True)
        print(prec, json.dumps(out)[:2000])


if __name__ == "__main__":
    main()
