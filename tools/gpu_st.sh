#!/bin/bash
# bf16 head parity (fused vs logits path, resident / ping-pong bit-exactness),
# then store-variant timing (tools/gpu_hgvar.sh)
set -o pipefail
O=gpurun_out/${1:-st}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_actor_head_bf16.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VARS="${VARS:-default hgoldst hgns}" REPS=${REPS:-2} bash tools/gpu_hgvar.sh ${1:-st}
rc=$?; [ $rc -eq 0 ] || exit $rc
if [ -n "$CPUSPREAD" ]; then
  WITH_CUDA=1 timeout -k 10 400 python tools/cpu_spread.py $CPUSPREAD > gpurun_out/${1:-st}/cpu_spread.log 2>&1
  rc=$?; cat gpurun_out/${1:-st}/cpu_spread.log | cut -c1-200; exit $rc
fi
