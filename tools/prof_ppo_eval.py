"""Profile target: bench.py's PPO eval leg alone (rocprofv3 --kernel-trace --stats)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

a = argparse.Namespace(ppo_eval_envs=int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
print(bench.bench_ppo_eval(a, torch.device("cuda", 0), 0, 1, None))
