#!/bin/bash
# Round 4: the db column-sum layouts, then the -m gpu suite, smoke and the
# driver's bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4j}; mkdir -p $O
GEMM_AB=1 timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/gemm_ab.log 2>&1
rc=$?; echo "gemm_ab rc=$rc"; tail -1 $O/gemm_ab.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r4_final_a.sh ${1:-r4j}
