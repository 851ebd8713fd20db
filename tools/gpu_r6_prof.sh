#!/bin/bash
# Round-6 closing profiles: the headline rocprofv3 evidence (kernel trace +
# PMC passes of the headline window, summarised into gpurun_out/OUT/traffic.json
# and profiles/traffic.json, which bench.py's line reads), then the ppo_eval
# leg's kernel trace (tools/gpu_evalprof.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r6prof}; mkdir -p $O
STEPS=20 WARMUP=5 bash tools/gpu_profile.sh > $O/prof.log 2>&1
rc=$?; echo "prof_rc=$rc"; [ $rc -ne 0 ] && { tail $O/prof.log; exit $rc; }
python3 tools/pmc_summary.py gpurun_out/prof 32768 --write $O/traffic.json > $O/pmc_summary.txt && cp $O/traffic.json profiles/traffic.json
find gpurun_out/prof/kt -name "*kernel_stats.csv" -exec cp {} $O/headline_kernel_stats.csv \;
rm -rf gpurun_out/prof/kt gpurun_out/prof/p1 gpurun_out/prof/p2 gpurun_out/prof/p3
bash tools/gpu_evalprof.sh ${1:-r6prof}_eval
exit $?
