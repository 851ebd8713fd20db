"""Where the ppo_eval step's time goes: host submission rate of ActStepGraph
replays (no sync) against their device time, and the per-step time of one
graph holding 1, 2 or 4 steps (launch gaps between graphs vs inside one)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]


def main():
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import ActStepGraph, PPOAgent, PPOConfig
    dev = torch.device("cuda", 0)
    N = 4096
    cfg = Config(pms=10, vms=30, service_length=1000, arrival_rate=0.0182, training_steps=10000,
                 eval_steps=100000, seed=1, reward_function="wr", sequence="uniform",
                 cap_target_util=True, beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, N, seeds=1 + 4 * np.arange(N, dtype=np.int64), device=dev)
    env.eval(True)
    ag = PPOAgent(env, PPOConfig(hidden_size=512, masked=True, migration_ratio=0.5))
    w = np.load(os.path.join(ROOT, "tests", "golden", "ppo10_wr_weights.npz"))
    ag.model.load_state_dict({k: torch.tensor(w[k]) for k in w.files})
    ag.eval(True)
    g = ActStepGraph(ag)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    K = 400
    t0 = time.perf_counter()
    for _ in range(K):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"replay: host {1e6 * (t1 - t0) / K:.1f} us/step submit, {1e6 * (t2 - t0) / K:.1f} us/step total",
          flush=True)
    t0 = time.perf_counter()
    for _ in range(K):
        g.graph.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph.replay only: host {1e6 * (t1 - t0) / K:.1f} us/step submit, "
          f"{1e6 * (t2 - t0) / K:.1f} us/step total", flush=True)
    for n in (2, 4, 8):
        gn = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(gn):
            for _ in range(n):
                g._step()
        torch.cuda.synchronize()
        for _ in range(5):
            gn.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K // n):
            gn.replay()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{n} steps per graph: {1e6 * (t2 - t0) / (K // n * n):.1f} us/step", flush=True)
    env.close()


if __name__ == "__main__":
    main()
