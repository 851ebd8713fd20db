#!/bin/bash
# Round 4: bf16 head timing split (hipBLASLt reference GEMMs, GEMM-only
# variant) and the kernel split of one bf16 PPO update on the fused path.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4c; mkdir -p $O
VD=$PWD/vm-placement-migration-gym_amd/build/variants
timeout -k 10 300 python tools/bench_actor_head_bf16.py > $O/head.log 2>&1
rc=$?; echo "head_rc=$rc"; tail -1 $O/head.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-hg16g}; do
  FWD_ONLY=1 VMP_LIB_PATH=$VD/libvmp_$v.so timeout -k 10 200 python tools/bench_actor_head_bf16.py > $O/head_$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; tail -1 $O/head_$v.log; [ $rc -ne 0 ] && exit $rc
done
mkdir -p gpurun_out/ppo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppo/kt_bf16 -o run \
  -- python tools/bench_ppo.py --precision bf16 --envs 8192 --updates 1 --warmup 0 > $O/kt_bf16.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -1 $O/kt_bf16.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/ppo_prof_summary.py gpurun_out/ppo bf16 | cut -c1-1500
