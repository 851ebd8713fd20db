"""SURVEY App. C item 6 — training-curve sanity anchor (not a parity test).

Trains the batched PPO (vmp.ppo.PPOTrainer) on config/10.yml with reward ut,
as the reference's data/exp_training/ppo-ut.csv run did (src/agents/ppo.py:
172-226: hidden 512, batch 100 / minibatch 25, 4 epochs, lr 5e-5, masked,
episodes of training_steps = 10 000 steps, one update per 100 steps), with N
envs instead of one: the same number of updates per episode (100), each on
N x 100 samples. Writes the per-episode return statistics next to the
reference's 100 published episode returns (the CSV's Value column; the data
file is read at generation time in the build container and its values are
embedded in tests/golden/ref_ppo_ut_returns.json, since /root/reference does
not exist on the GPU box).

Usage: python tools/train_curve.py [--envs 16] [--episodes 100] [--out PATH]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

REF_JSON = os.path.join(ROOT, "tests", "golden", "ref_ppo_ut_returns.json")
REF_CSV = "/root/reference/data/exp_training/ppo-ut.csv"


def reference_returns():
    """The reference's 100 episode returns (ppo-ut.csv Value column)."""
    if os.path.exists(REF_JSON):
        return np.array(json.load(open(REF_JSON))["returns"])
    import csv
    with open(REF_CSV) as f:
        rows = list(csv.DictReader(f))
    vals = [float(r["Value"]) for r in rows]
    json.dump({"source": "data/exp_training/ppo-ut.csv (Value column, steps 0..99)",
               "returns": vals}, open(REF_JSON, "w"))
    return np.array(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=16)
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "train_curve_10yml_ut.json"))
    ap.add_argument("--ref-only", action="store_true", help="write the reference fixture, exit")
    args = ap.parse_args()
    ref = reference_returns()
    if args.ref_only:
        return
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig
    torch.manual_seed(0)
    cfg = Config(pms=10, vms=30, service_length=1000, arrival_rate=0.0182, training_steps=10000,
                 eval_steps=100000, seed=1, reward_function="ut", sequence="uniform",
                 cap_target_util=True, beta=0.5, allow_null_action=True)  # config/10.yml, -r ut
    env = BatchedVmEnv(cfg, args.envs, device="cuda:0")
    ag = PPOAgent(env, PPOConfig(episodes=args.episodes, hidden_size=512, masked=True,
                                 batch_size=100, minibatch_size=25, training_progress_bar=False))
    tr = ag.trainer()
    per_ep = 10000 // tr.T
    t0 = time.perf_counter()
    for ep in range(args.episodes):
        for _ in range(per_ep):
            tr.collect()
            tr.update()
        r = tr.ep_returns[-1]
        if ep % 10 == 0 or ep == args.episodes - 1:
            print(f"episode {ep}: median return {np.median(r):.1f} (envs {r.min():.1f} .. "
                  f"{r.max():.1f}); reference {ref[min(ep, len(ref) - 1)]:.1f}; "
                  f"{time.perf_counter() - t0:.0f} s", flush=True)
    rets = np.array(tr.ep_returns)  # [episodes, envs]
    med = np.median(rets, 1)
    k = min(10, len(med))
    out = {
        "what": "batched PPO on config/10.yml, reward ut, vs data/exp_training/ppo-ut.csv "
                "(SURVEY App. C item 6: sanity anchor, not parity)",
        "envs": args.envs, "episodes": args.episodes, "updates": args.episodes * per_ep,
        "wall_s": time.perf_counter() - t0,
        "median_return_per_episode": med.tolist(),
        "min_return_per_episode": rets.min(1).tolist(),
        "max_return_per_episode": rets.max(1).tolist(),
        "reference_returns": ref.tolist(),
        "summary": {
            "ours_first10_median": float(np.median(med[:k])),
            "ours_last10_median": float(np.median(med[-k:])),
            "reference_first10_median": float(np.median(ref[:k])),
            "reference_last10_median": float(np.median(ref[-k:])),
            "reference_band_all_episodes": [float(ref.min()), float(ref.max())],
        },
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out["summary"]), flush=True)
    env.close()


if __name__ == "__main__":
    main()
