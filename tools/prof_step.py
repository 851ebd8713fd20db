"""Workload for rocprofv3 passes: the bench configuration fast-forwarded to
steady state, then K per-step heuristic launches (the last K k_env dispatches)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmp import _lib  # noqa: E402
from vmp.batched import BatchedVmEnv  # noqa: E402
from vmp.config import Config  # noqa: E402

N = int(os.environ.get("PROF_ENVS", "32768"))
K = int(os.environ.get("PROF_STEPS", "20"))
cfg = Config(pms=100, vms=1000, arrival_rate=1.8182, service_length=1000, training_steps=10000,
             eval_steps=100000, seed=0, reward_function="wr", allow_null_action=True)
env = BatchedVmEnv(cfg, N, seeds=4 * np.arange(N, dtype=np.int64))
env.eval(os.environ.get("PROF_EVAL", "1") == "1")  # bench.py: PROF_EVAL=0 (training)
for _ in range(25):
    env.rollout("firstfit", 100)
D = 3 * 1000 + 200
obs = torch.empty((N, D), dtype=torch.float32, device="cuda")
rew = torch.empty((N,), dtype=torch.float64, device="cuda")
done = torch.empty((N,), dtype=torch.uint8, device="cuda")
h = env._bind()
L = _lib.lib()
torch.cuda.synchronize()
for _ in range(K):
    _lib.check(L.vmp_heuristic_step(h, 0, None, _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done), None))
torch.cuda.synchronize()
print("done", N, K)
