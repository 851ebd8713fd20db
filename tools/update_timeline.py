"""Where the bf16 PPO update's wall time goes beyond its kernels (VERDICT r4
item 6): per minibatch, the host time to enqueue it and the device time
between HIP events recorded at its start and end, plus the device idle gaps
between consecutive pieces (values + GAE, minibatches, tail).
Usage: python tools/update_timeline.py [--envs 8192] [--precision bf16] [--lookahead 1]"""
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
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--lookahead", type=int, default=1)
    args = ap.parse_args()
    from vmp.batched import BatchedVmEnv
    from vmp.config import Config
    from vmp.ppo import PPOAgent, PPOConfig, PPOTrainer
    torch.manual_seed(0)
    cfg = Config(pms=100, vms=300, service_length=1000, arrival_rate=1.8182, training_steps=10000,
                 eval_steps=100000, seed=0, reward_function="wr", cap_target_util=True,
                 sequence="uniform", beta=0.5, allow_null_action=True)
    env = BatchedVmEnv(cfg, args.envs, device="cuda:0")
    ag = PPOAgent(env, PPOConfig(hidden_size=512, masked=True, batch_size=100, minibatch_size=25,
                                 migration_ratio=0.002, precision=args.precision,
                                 kl_lookahead=bool(args.lookahead)))
    tr = ag.trainer()
    tr.collect()
    tr.update()
    tr.collect()
    torch.cuda.synchronize()
    marks = []  # (label, host time, device event)

    def mark(label):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((label, time.perf_counter(), ev))

    orig = PPOTrainer._minibatch_backward

    def mb(self, batch, t0, t1):
        mark("mb_start")
        out = orig(self, batch, t0, t1)
        mark("mb_bwd_end")
        return out
    PPOTrainer._minibatch_backward = mb
    orig_step = PPOTrainer._optimizer_step

    def step(self, params, clip_n, m_glob):
        r = orig_step(self, params, clip_n, m_glob)
        mark("step_end")
        return r
    PPOTrainer._optimizer_step = step
    orig_values = PPOTrainer._values

    def values(self, obs):
        mark("values_start")
        r = orig_values(self, obs)
        mark("values_end")
        return r
    PPOTrainer._values = values
    orig_gae = tr.gae

    def gae(*a, **k):
        mark("gae_start")
        r = orig_gae(*a, **k)
        mark("gae_end")
        return r
    tr.gae = gae
    orig_snap = PPOTrainer._opt_snapshot

    def snap(self, params):
        mark("snap_start")
        return orig_snap(self, params)
    PPOTrainer._opt_snapshot = snap
    t0 = time.perf_counter()
    mark("update_start")
    tr.update()
    mark("update_end")
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    e0 = marks[0][2]
    rows = []
    for (lab, ht, ev) in marks:
        rows.append((lab, (ht - t0) * 1e3, e0.elapsed_time(ev)))
    # device busy segments: mb_start -> step_end of each minibatch; gaps between
    gaps = []
    for i in range(1, len(rows)):
        gaps.append((rows[i - 1][0] + "->" + rows[i][0], rows[i][2] - rows[i - 1][2],
                     rows[i][1] - rows[i - 1][1]))
    print(json.dumps({"wall_ms": wall * 1e3, "lookahead": bool(args.lookahead),
                      "device_ms_last_event": rows[-1][2],
                      "marks": [(a, round(b, 2), round(c, 2)) for a, b, c in rows],
                      "segments_device_host_ms": [(a, round(b, 2), round(c, 2)) for a, b, c in gaps]}))
    env.close()


if __name__ == "__main__":
    main()
