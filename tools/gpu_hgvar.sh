#!/bin/bash
# bf16 head timing variants (tools/build_hg_variant.sh NAME -D...): the
# FWD_ONLY head bench through each library, REPS interleaved rounds.
#   VARS="default hggo ..." [REPS=2] [PP=0] bash tools/gpu_hgvar.sh OUT
# "default" = the normal vmp/libvmp.so; NAME@VAR=VALUE runs NAME with that
# environment variable set (e.g. hggo@VMP_HG16_DEEP=1). Optional: PARITY=1 first runs the
# bf16 head tests on the default library.
set -o pipefail
O=gpurun_out/${1:?out dir}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
if [ -n "$PARITY" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_actor_head_bf16.py -k "ping_pong or fused_matches" > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq 1 ${REPS:-2}); do
  for vv in $VARS; do
    v=${vv%%@*}; E=""; [ "$v" != "$vv" ] && E=${vv#*@}
    if [ "$v" = default ]; then L=""; else L=$VD/libvmp_$v.so; fi
    v=${vv//[@=]/_}
    env $E VMP_LIB_PATH=$L VMP_HG16_PP=${PP:-0} FWD_ONLY=1 timeout -k 10 200 python tools/bench_actor_head_bf16.py \
      > $O/${v}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 $O/${v}_$rep.log; exit $rc; }
    python - $O/${v}_$rep.log $v $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:>10} rep{sys.argv[3]} fwd {d['fused_fwd_ms']:.3f} ms  bwd {d['bwd_ms_per_204800']:.3f}  "
      f"bwd+db {d['bwd_with_dbias_ms_per_204800']:.3f}")
PY
  done
done
exit 0
