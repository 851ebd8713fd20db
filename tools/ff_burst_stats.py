"""Where the headline's FirstFit heuristic spends its placement loop (DESIGN.md
§3.1, round 6), from the C oracle (analysis only; no GPU): 16 envs of the
bench workload (P100 V1000, lambda 1.8182, L 1000, wr), steps 2 000-2 999
(the refill burst at 2 001-2 200, then the quiet phase).

Per env-step:
  - placement attempts (pending VMs FirstFit assigns a PM in the f32
    observation) and valid placements (the env's f64 check, env.py:55-64);
  - "rejected-only" steps: attempts made, none valid;
  - "repeats": a rejected-only step after a step that changed nothing (no
    valid placement, no finish, no arrival): same observation, same
    decisions, same rejections - what EnvHdr::pad bit 60 skips;
  - burst placements whose first-fit PM in the pre-step state is untouched by
    the step's earlier placements (what a speculative all-hits pass would
    settle without a rescan), and the hit counts behind them."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from oracle import oracle as O  # noqa: E402

CFG = dict(pms=100, vms=1000, arrival_rate=1.8182, service_length=1000, training_steps=10000,
           eval_steps=100000, seed=0, reward_function="wr", sequence="uniform",
           cap_target_util=True, beta=0.5, allow_null_action=True)
P, V = 100, 1000


def main(n_env=16, t0=2000, t1=3000, burst_end=2200):
    tot = dict(env_steps=0, attempts=0, rejected_only=0, repeats=0)
    burst = []  # (hits, placements, untouched first-fit)
    for i in range(n_env):
        e = O.OracleEnv(dict(CFG, seed=4 * i))
        e.eval(False)
        e.reset(4 * i)
        prev_still = False
        for t in range(t1):
            obs = e.obs()
            c0 = e.counters()[0]
            a = e.firstfit()
            pl = obs[:V].astype(np.int64)
            att = int(np.sum((pl == P) & (a < P)))
            if t0 <= t < burst_end:
                vc, vm = obs[V:2 * V], obs[2 * V:3 * V]
                cpu = obs[3 * V:3 * V + P].astype(np.float32)
                mem = obs[3 * V + P:].astype(np.float32)
                first = {}
                for v in np.nonzero(pl == P)[0]:
                    f = np.nonzero((cpu + vc[v] <= 1) & (mem + vm[v] <= 1))[0]
                    if len(f):
                        first[v] = f[0]
                touched, ok = set(), 0
                for v in np.nonzero((pl == P) & (a < P))[0]:
                    ok += first.get(v) == a[v] and a[v] not in touched
                    touched.add(a[v])
                burst.append((len(first), att, ok))
            e.step(a)
            c1 = e.counters()[0]
            placed, served = c1[3] - c0[3], c1[1] - c0[1]
            acc = (c1[0] - c0[0]) - (c1[4] - c0[4])
            if t >= t0:
                tot["env_steps"] += 1
                tot["attempts"] += att > 0
                tot["rejected_only"] += att > 0 and placed == 0
                tot["repeats"] += prev_still and att > 0 and placed == 0
            prev_still = placed == 0 and served == 0 and acc == 0
    b = np.array(burst)
    print("steps %d-%d, %d envs:" % (t0, t1 - 1, n_env), tot)
    print("share of env-steps: attempts %.3f, rejected-only %.3f, skippable repeats %.3f" % (
        tot["attempts"] / tot["env_steps"], tot["rejected_only"] / tot["env_steps"],
        tot["repeats"] / tot["env_steps"]))
    print("burst %d-%d: mean hits %.1f, placements %.2f, of which untouched first-fit %.2f" % (
        t0, burst_end - 1, b[:, 0].mean(), b[:, 1].mean(), b[:, 2].mean()))
    for k in range(1, 8):
        m = b[:, 1] == k
        if m.any():
            print("  %d placements: %4d steps, mean hits %.0f, untouched %.2f" % (
                k, m.sum(), b[m, 0].mean(), b[m, 2].mean()))


if __name__ == "__main__":
    main()
