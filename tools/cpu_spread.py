"""CPU-baseline noise on the GPU box (diagnostic): the headline cpu_baseline
pass (C oracle, FirstFit act + step, 48 envs per thread, 1 000 steps after
2 500 warm-up steps) at several OpenMP thread counts, 7 timed passes each,
with and without a CUDA context in the process.
Usage: python tools/cpu_spread.py [threads ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(threads, reps=7, ept=48):
    n_env = ept * threads
    secs, _ = O.rollout_timed(bench.CFG, n_env, 0, 4, 2500, 1000, 0, threads, eval_mode=False,
                              reps=reps + 1)
    r = n_env * 1000 / secs[1:]
    med = float(np.median(r))
    return {"threads": threads, "median": med, "per_thread": med / threads,
            "spread": float((r.max() - r.min()) / med), "rates": [round(float(x)) for x in r]}


def main():
    ths = [int(x) for x in sys.argv[1:]] or [16, 15, 14, 12]
    print(json.dumps(bench.host_cpus()), flush=True)
    for t in ths:
        print(json.dumps(run(t)), flush=True)
    if os.environ.get("WITH_CUDA") == "1":
        import torch
        torch.zeros(1, device="cuda")
        for t in ths:
            print("cuda-ctx", json.dumps(run(t)), flush=True)


if __name__ == "__main__":
    main()
