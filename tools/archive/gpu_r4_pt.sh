#!/bin/bash
# Round 4: same-box A/B of the step kernels: libvmp_prev.so (HEAD's kernels)
# vs the working tree's library, headline + period + nominal + fused rollout.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4s}; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
ARGS="--no-cpu --no-ppo --ext-steps 0 --stress-steps 0 --steps 20 --warmup 5"
for v in default ptail default ptail; do
  L=""; [ $v != default ] && L=$VD/libvmp_$v.so
  VMP_LIB_PATH=$L timeout -k 10 300 python bench.py $ARGS > $O/bench_$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 $O/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['period']['mean_ms'],4), d['period']['ms_by_100_steps'], round(d['nominal_load']['kernel_ms'],4), round(d['fused_rollout']['value']/1e6,1))")"; [ $rc -ne 0 ] && exit $rc
done
exit 0
