"""BASELINE config 5: P1000 / V10000, lambda = 1000/0.55/1000
(100 % load), L = 1000, reward kl, BestFit act + step, envs per GPU (default
512), on the block-per-env kernel k_env_big. Fast-forwards `--ff` steps with
fused rollouts, then times K per-step launches; prints env-steps/s and the
HBM roofline of the per-step kernel (algorithmic bytes as bench.py's)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=512)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ff", type=int, default=2000)
    ap.add_argument("--policy", default="bestfit")
    ap.add_argument("--reward", default="kl")
    args = ap.parse_args()
    from vmp import _lib
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    P, V = 1000, 10000
    cfg = Config(pms=P, vms=V, arrival_rate=round(1000 / 0.55 / 1000, 3), service_length=1000,
                 training_steps=10000, eval_steps=100000, seed=0, reward_function=args.reward,
                 sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
    N = args.envs
    env = BatchedVmEnv(cfg, N, seeds=4 * np.arange(N, dtype=np.int64), device="cuda:0")
    t0 = time.perf_counter()
    left = args.ff
    while left > 0:
        env.rollout(args.policy, min(250, left))
        left -= 250
    torch.cuda.synchronize()
    ff_s = time.perf_counter() - t0
    dev = env.device
    obs = torch.empty((N, env.D), dtype=torch.float32, device=dev)
    rew = torch.empty((N,), dtype=torch.float64, device=dev)
    done = torch.empty((N,), dtype=torch.uint8, device=dev)
    L = _lib.lib()
    h = env._bind()
    pol = _lib.POLICIES[args.policy]

    def step():
        _lib.check(L.vmp_heuristic_step(h, pol, None, _lib.ptr(obs), _lib.ptr(rew),
                                        _lib.ptr(done), None))
    step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    from bench import changed_words, step_bytes
    c0 = env.counters()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(s)
        step()
        b.record(s)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    words, pms = changed_words(c0, env.counters(), N * args.steps)
    bpe = step_bytes(P, V, words, pms)  # bench.py's byte model
    st = env.state()["vm_placement"]
    print(json.dumps({"workload": f"P{P} V{V} {args.policy} act+step, reward {args.reward}",
                      "envs": N, "value": N * args.steps / el, "unit": "env-steps/s",
                      "kernel_ms": kern_ms, "bytes_per_env_step": bpe,
                      "hbm_GBps": bpe * N / (kern_ms * 1e-3) / 1e9,
                      "roofline_frac": bpe * N / (kern_ms * 1e-3) / 8e12,
                      "ff_steps": args.ff, "ff_s": ff_s,
                      "mean_waiting": float((st == P).sum(1).double().mean()),
                      "mean_running": float((st < P).sum(1).double().mean())}), flush=True)
    env.close()


if __name__ == "__main__":
    main()
