#!/bin/bash
# PPO update chunk size A/B (f32 and bf16): 4 GB chunks vs auto (1/8 of HBM)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for prec in f32 bf16; do
  for gb in 4 0; do
    timeout -k 10 300 python tools/bench_ppo.py --precision $prec --chunk-gb $gb --updates 1 > gpurun_out/ppo_${prec}_${gb}.log 2>&1
    rc=$?; echo "$prec chunk_gb=$gb rc=$rc"; grep -v amdgpu.ids gpurun_out/ppo_${prec}_${gb}.log | tail -2; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
