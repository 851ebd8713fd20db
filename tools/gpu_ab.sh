#!/bin/bash
# A/B of env-kernel library variants (tools/build_variant.sh NAME -D...):
#   VARIANTS="base lh ..." [PARITY="lh ..."] [REPS=2] tools/gpu_ab.sh OUT
# 1. for each variant in PARITY: tests/test_gpu_env.py through that library
#    (every golden trajectory, the batched oracle replays, the headline steady
#    state, step hints) -- a variant must stay bit-exact before it is timed;
# 2. REPS interleaved rounds of bench.py (headline, external, fused rollout,
#    period, nominal legs; no PPO / C5 / CPU) per variant, one box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:?out dir}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
for v in $PARITY; do
  VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -q -m gpu \
    --timeout 300 --timeout-method thread -k "not quiet_bit_check" > $O/parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc: $(tail -1 $O/parity_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-ppo \
      --no-cpu $BENCH_ARGS > $O/b_${v}_$rep.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 $O/b_${v}_$rep.log; exit $rc; }
    python - $O/b_${v}_$rep.log $v $rep <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
pr = d["period"] or {}
print(f"{sys.argv[2]:>8} rep{sys.argv[3]} head {d['roofline']['kernel_ms']:.4f} ms "
      f"period {pr.get('mean_ms', 0):.4f} (burst {pr.get('ms_by_100_steps', [0])[0]:.4f} "
      f"max/min {max(pr.get('ms_by_100_steps', [1])) / min(pr.get('ms_by_100_steps', [1])):.2f}) "
      f"ext {d['external_actions']['kernel_ms']:.4f} fused {d['fused_rollout']['value'] / 1e6:.1f}M "
      f"nominal {d['nominal_load']['kernel_ms']:.4f}")
PY
  done
done
exit 0
