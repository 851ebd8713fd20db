"""Experiment sweeps of the reference (exp_suspension.py, exp.py) as batched GPU
runs: every (agent, load, service length) cell is one BatchedVmEnv whose envs
are the cell's seeds, all cells advance side by side on their own streams, and
the Record metrics are kept on the device (vmp_record_*), so nothing per step
comes back to the host. This replaces the reference's process fan-out
(exp.py:1-2, 8 processes of one env each) and its per-step host Record.

    python -m vmp.exp suspension --out data.csv            # heuristic rows
    python -m vmp.exp suspension --agents ppo --weights w.pt --out ppo.csv

Rows are printed in exp_suspension.py's CSV layout (exp_suspension.py:51-58):
Agent, Load, Service Length, Total Served, Valid Suspend Actions, Valid
Actions, Life, Average Pending, Average Slowdown, Max Slowdown.
"""
import argparse
from dataclasses import dataclass

import numpy as np
import torch

from .batched import BatchedVmEnv
from .config import Config

SUSPENSION_HEADER = ("Agent, Load, Service Length, Total Served, Valid Suspend Actions, "
                     "Valid Actions, Life, Average Pending, Average Slowdown, Max Slowdown")

# config/100.yml's environment section (the sweeps override reward / arrival rate)
ENV100 = dict(pms=100, vms=300, service_length=1000, arrival_rate=1.8182, training_steps=10000,
              eval_steps=100000, seed=0, reward_function="wr", cap_target_util=True,
              sequence="uniform", beta=0.5, allow_null_action=True)
PPO100 = dict(episodes=100, hidden_size=512, masked=True, batch_size=100, minibatch_size=25,
              migration_ratio=0.002)


@dataclass
class Cell:
    agent: str
    load: float
    service_length: int
    seeds: tuple = (0,)
    weights: str = None


def suspension_config(load, sr, env=ENV100):
    """exp_suspension.py:13-19: reward wr, uniform sizes, the given service length,
    arrival_rate = round(pms / 0.55 / sr * load, 3)."""
    c = dict(env)
    c.update(reward_function="wr", sequence="uniform", service_length=sr,
             arrival_rate=float(np.round(c["pms"] / 0.55 / sr * load, 3)))
    return c


def run_cells(cells, make_config, eval_steps=None, chunk=2000, device="cuda:0"):
    """Evaluate every cell (Base.test per seed, base.py:63-118) for eval_steps and
    return one list of Record summaries per cell (one dict per seed)."""
    envs, agents, streams = [], [], []
    for cell in cells:
        cfg = make_config(cell.load, cell.service_length)
        if eval_steps is not None:
            cfg["eval_steps"] = int(eval_steps)
        s = torch.cuda.Stream(device=device)
        with torch.cuda.stream(s):
            env = BatchedVmEnv(Config(**cfg), len(cell.seeds), seeds=list(cell.seeds),
                               device=device)
            env.eval(True)
            env.reset(torch.tensor(list(cell.seeds), dtype=torch.int64))
            env.record(True)  # before the graph capture, so replays are recorded too
            agent = None
            if cell.agent == "ppo":
                from .ppo import ActStepGraph, PPOAgent, PPOConfig
                ag = PPOAgent(env, PPOConfig(**PPO100))
                ag.load_model(cell.weights)
                ag.eval(True)
                agent = ActStepGraph(ag, warmup=0)
        envs.append(env)
        agents.append(agent)
        streams.append(s)
    T = int(eval_steps if eval_steps is not None else make_config(1.0, 1000)["eval_steps"])
    done = 0
    while done < T:
        k = min(chunk, T - done)
        for cell, env, agent, s in zip(cells, envs, agents, streams):
            with torch.cuda.stream(s):
                if agent is None:
                    env.rollout(cell.agent, k)
                else:
                    for _ in range(k):
                        agent.replay()
        done += k
    out = []
    for env, s in zip(envs, streams):
        with torch.cuda.stream(s):
            out.append(env.record_summary())
        env.close()
    return out


def suspension_row(cell, summaries):
    """exp_suspension.py:51-58 for one cell (mean over its seeds)."""
    f = lambda k: float(np.mean([s[k] for s in summaries]))  # noqa: E731
    name = cell.agent if cell.weights is None else cell.weights.split("/")[-1].split(".")[0]
    susp, placed = f("total suspend actions"), f("total place actions")
    return "%s,%.1f,%d,%d,%d,%d,%d,%.3f,%.3f,%.3f" % (
        name, cell.load, cell.service_length, f("total served VMs"), susp, susp + placed,
        f("_mean_life"), f("_mean_pending"), f("_mean_slowdown"), f("_max_slowdown"))


def suspension_sweep(agents=("firstfit", "bestfit"), loads=None, lengths=None, seeds=(0,),
                     weights=None, eval_steps=None):
    """The exp_suspension.py grid (load 1.0 x service lengths 100..3900 step 200,
    then service length 1000 x loads 0.2..1.0) for the given agents."""
    if lengths is None:
        lengths = list(range(100, 4100, 200))
    if loads is None:
        loads = [float(x) for x in np.arange(0.2, 1.1, 0.1)]
    cells = [Cell(a, 1.0, int(sr), tuple(seeds), weights if a == "ppo" else None)
             for sr in lengths for a in agents]
    cells += [Cell(a, float(ld), 1000, tuple(seeds), weights if a == "ppo" else None)
              for ld in loads for a in agents]
    res = run_cells(cells, suspension_config, eval_steps=eval_steps)
    return [suspension_row(c, r) for c, r in zip(cells, res)]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("experiment", choices=["suspension"])
    ap.add_argument("--agents", default="firstfit,bestfit")
    ap.add_argument("--weights", default=None, help="PPO weights (.pt) for agent ppo")
    ap.add_argument("--seeds", default="0")
    ap.add_argument("--loads", default=None, help="comma list (default: the reference grid)")
    ap.add_argument("--lengths", default=None, help="comma list of service lengths")
    ap.add_argument("--eval-steps", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    rows = suspension_sweep(
        agents=a.agents.split(","),
        loads=None if a.loads is None else [float(x) for x in a.loads.split(",")],
        lengths=None if a.lengths is None else [int(x) for x in a.lengths.split(",")],
        seeds=[int(x) for x in a.seeds.split(",")], weights=a.weights, eval_steps=a.eval_steps)
    text = SUSPENSION_HEADER + "\n" + "\n".join(rows) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text, end="")


if __name__ == "__main__":
    main()
