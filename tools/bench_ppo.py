"""PPO training throughput on the GPU env (BASELINE config 3: config/100.yml,
PPO from scratch, reward wr, N envs on one MI355X).

One "update" = batch_size (100) rollout steps of every env (actor forward +
HIP head sample + env step) followed by PPOAgent.update (GAE, 4 epochs x 4
minibatches, HIP head forward/backward, AdamW). Reports env-steps/s of the
whole loop and the collect / update split.

Usage: python tools/bench_ppo.py [--envs 8192] [--updates 2] [--warmup 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--updates", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pms", type=int, default=100)
    ap.add_argument("--vms", type=int, default=300)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--chunk-gb", type=float, default=0.0, help="0: auto (1/8 of HBM)")
    ap.add_argument("--precision", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--lookahead", type=int, default=1, help="PPOConfig.kl_lookahead")
    ap.add_argument("--dl-gb", type=float, default=0.0,
                    help="PPOConfig.dlogits_chunk_bytes in GiB (0: the default)")
    args = ap.parse_args()
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    torch.manual_seed(0)
    cfg = Config(pms=args.pms, vms=args.vms, service_length=1000, arrival_rate=1.8182,
                 training_steps=10000, eval_steps=100000, seed=0, reward_function="wr",
                 cap_target_util=True, sequence="uniform", beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, args.envs, device="cuda:0")
    ag = PPOAgent(env, PPOConfig(hidden_size=args.hidden, masked=True, batch_size=100,
                                 minibatch_size=25, migration_ratio=0.002,
                                 chunk_bytes=int(args.chunk_gb * (1 << 30)),
                                 precision=args.precision, kl_lookahead=bool(args.lookahead),
                                 **({"dlogits_chunk_bytes": int(args.dl_gb * (1 << 30))}
                                    if args.dl_gb > 0 else {})))
    tr = ag.trainer()
    for _ in range(args.warmup):
        tr.collect()
        tr.update()
    torch.cuda.synchronize()
    tc = tu = 0.0
    for _ in range(args.updates):
        t0 = time.perf_counter()
        tr.collect()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        st = tr.update()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        tc += t1 - t0
        tu += t2 - t1
    steps = args.envs * tr.T * args.updates
    out = {"workload": f"PPO train P{args.pms} V{args.vms} hidden {args.hidden} {args.precision}",
           "kl_lookahead": bool(args.lookahead),
           "envs": args.envs, "updates": args.updates, "env_steps": steps,
           "value": steps / (tc + tu), "unit": "env-steps/s",
           "collect_s_per_update": tc / args.updates, "update_s_per_update": tu / args.updates,
           "collect_env_steps_per_s": steps / tc, "minibatches": st["minibatches"],
           "kl_breaks": st["kl_breaks"], "peak_mem_gb": torch.cuda.max_memory_allocated() / 2**30}
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == "__main__":
    main()
