#!/bin/bash
# k_env occupancy variants: the headline leg (no PPO / CPU legs) per library
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$PWD/vm-placement-migration-gym_amd/build/variants
for v in default ${OCC_VARIANTS:-w3}; do
  if [ $v = default ]; then unset VMP_LIB_PATH; else export VMP_LIB_PATH=$V/libvmp_$v.so; fi
  timeout -k 10 300 python bench.py --no-ppo --no-cpu --steps 100 --warmup 10 > gpurun_out/occ_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/occ_$v.log; exit $rc; }
  grep -v amdgpu.ids gpurun_out/occ_$v.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['external_actions']['kernel_ms'], d['fused_rollout']['value'], d['parity'])"
done
