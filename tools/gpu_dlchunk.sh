#!/bin/bash
# bf16 PPO leg at several dlogits chunk sizes (PPOConfig.dlogits_chunk_bytes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-dlchunk}; mkdir -p $O
for rep in 1 2; do
  for g in 4 8 16; do
    timeout -k 10 300 python tools/bench_ppo.py --precision bf16 --updates 2 --dl-gb $g > $O/dl${g}_$rep.log 2>&1
    rc=$?; echo "dl-gb=$g rep$rep $(tail -1 $O/dl${g}_$rep.log | cut -c1-330)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
