#!/bin/bash
# Round-5 profile set, one call: the headline window (rocprofv3 kernel trace +
# 3 PMC passes, tools/gpu_profile.sh), C5's PMC passes (tools/gpu_c5_pmc.sh)
# and the bf16 PPO update's kernel split + MFMA-busy pass (tools/gpu_ppo_prof.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_profile.sh && \
  python3 tools/pmc_summary.py gpurun_out/prof 32768 --write gpurun_out/prof/summary.json > /dev/null && \
  python3 - <<'PY'
import csv, glob, shutil, os
# keep the kernel-stats table, drop the raw per-dispatch CSVs
for f in glob.glob("gpurun_out/prof/kt/**/*kernel_stats.csv", recursive=True):
    shutil.copy(f, "gpurun_out/prof/kernel_stats.csv")
for d in ["gpurun_out/prof/kt", "gpurun_out/prof/p1", "gpurun_out/prof/p2", "gpurun_out/prof/p3"]:
    shutil.rmtree(d, ignore_errors=True)
PY
rc=$?; echo "headline prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_c5_pmc.sh > gpurun_out/c5pmc.log 2>&1; rc=$?; echo "c5 pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
PRECS=bf16 bash tools/gpu_ppo_prof.sh; rc=$?; echo "ppo prof rc=$rc"; exit $rc
