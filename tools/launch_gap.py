"""Wall time per launch of the headline per-step kernel with and without HIP
event pairs around each launch (host launch overhead vs kernel time).
Usage: python tools/launch_gap.py [envs] [ff_steps]  (VMP_LIB_PATH picks a library)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "vm-placement-migration-gym_amd"))
import bench  # noqa: E402  (config of the headline workload)
from vmp import _lib  # noqa: E402
from vmp.batched import BatchedVmEnv  # noqa: E402
from vmp.config import Config  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
FF = int(sys.argv[2]) if len(sys.argv) > 2 else 2500
dev = torch.device("cuda", 0)
env = BatchedVmEnv(Config(**bench.CFG), N, seeds=4 * np.arange(N, dtype=np.int64), device=dev)
left = FF
while left > 0:
    env.rollout("firstfit", min(100, left))
    left -= 100
L, h = _lib.lib(), env._bind()
D = env.D
obs = torch.empty((N, D), dtype=torch.float32, device=dev)
rew = torch.empty((N,), dtype=torch.float64, device=dev)
done = torch.empty((N,), dtype=torch.uint8, device=dev)
po, pr, pd = _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(done)
stream = torch.cuda.current_stream(dev)


def step():
    _lib.check(L.vmp_heuristic_step(h, 0, None, po, pr, pd, None))


for _ in range(20):
    step()
torch.cuda.synchronize()
for K in (20, 200):
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / K * 1e3
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    withev = (time.perf_counter() - t0) / K * 1e3
    kern = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    host = (time.perf_counter() - t0) / K * 1e3
    torch.cuda.synchronize()
    print(f"lib={os.environ.get('VMP_LIB_PATH', 'default').split('/')[-1]} K={K} wall_plain_ms={plain:.4f} "
          f"wall_events_ms={withev:.4f} kernel_ms={kern:.4f} host_issue_ms={host:.4f}", flush=True)
env.close()
