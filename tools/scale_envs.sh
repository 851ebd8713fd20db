#!/bin/bash
mkdir -p gpurun_out
for N in 2048 8192 32768 65536; do
  timeout -k 10 300 python bench.py --no-cpu --steps 50 --envs $N > gpurun_out/scale_$N.log 2>&1 || exit 1
done
