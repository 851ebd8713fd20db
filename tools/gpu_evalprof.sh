#!/bin/bash
# rocprofv3 kernel trace of bench.py's ppo_eval leg alone -> gpurun_out/evalprof/kernel_stats.csv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-evalprof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -o run -- python3 tools/prof_ppo_eval.py > $O/log.txt 2>&1
rc=$?
find $O/raw -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/raw; tail -2 $O/log.txt; exit $rc
