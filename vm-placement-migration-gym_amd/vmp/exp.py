"""Experiment sweeps of the reference (exp_suspension.py, exp.py) as batched GPU
runs: every (agent, load, service length) cell is one BatchedVmEnv whose envs
are the cell's seeds, all cells advance side by side on their own streams, and
the Record metrics are kept on the device (vmp_record_*), so nothing per step
comes back to the host. This replaces the reference's process fan-out
(exp.py:1-2, 8 processes of one env each) and its per-step host Record.

    python -m vmp.exp suspension --out data.csv            # heuristic rows
    python -m vmp.exp suspension --agents ppo --weights w.pt --out ppo.csv
    python -m vmp.exp performance --loads 1.0,0.6          # exp_performance.py summary
    python -m vmp.exp performance_small                    # exp_performance_small.py
    python -m vmp.exp vm_size                              # exp_vm_size.py summary
    python -m vmp.exp reward --agents ppo --weights 'w/ppo-{reward}.pt'   # exp_reward.py
    python -m vmp.exp migration_ratio --agents bestfit,ppo --weights 'w/ppo-{reward}.pt'

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
              eval_steps=100000, seed=0, reward_function="kl", cap_target_util=True,
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
    cfg: dict = None   # the cell's environment config (else make_config(load, length))
    ppo: dict = None   # PPOConfig overrides (exp_performance.py:28-33)
    name: str = None   # row label (jobname)


def suspension_config(load, sr, env=ENV100):
    """exp_suspension.py:13-19: reward wr, uniform sizes, the given service length,
    arrival_rate = round(pms / 0.55 / sr * load, 3)."""
    c = dict(env)
    c.update(reward_function="wr", sequence="uniform", service_length=sr,
             arrival_rate=float(np.round(c["pms"] / 0.55 / sr * load, 3)))
    return c


class _RecordedRollout:
    """`g_steps` recorded heuristic steps (act+step, then the recorder: two
    launches per step) of one env captured as a HIP graph, so a long eval costs
    one graph launch per g_steps steps instead of 2 * g_steps kernel launches."""

    def __init__(self, env, policy, g_steps):
        self.env, self.policy, self.g = env, policy, g_steps
        n = env.n_envs
        self.rew = torch.empty((g_steps, n), dtype=torch.float64, device=env.device)
        self.dc = torch.zeros(n, dtype=torch.int64, device=env.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            env.rollout(policy, g_steps, rewards=self.rew, done_count=self.dc)

    def run(self, k):
        for _ in range(k // self.g):
            self.graph.replay()
        if k % self.g:
            self.env.rollout(self.policy, k % self.g)


def run_cells(cells, make_config=None, eval_steps=None, chunk=2000, device="cuda:0",
              graph_steps=100):
    """Evaluate every cell (Base.test per seed, base.py:63-118) for its eval_steps
    and return one list of Record summaries per cell (one dict per seed). All
    seeds of a cell are the envs of one handle, so the recorder's cross-env sums
    (VMP_REC_XMEM) span exactly the cell's seeds. Heuristic cells replay a
    captured graph of graph_steps recorded steps (0 = plain launches)."""
    envs, agents, streams, steps = [], [], [], []
    for cell in cells:
        cfg = dict(cell.cfg) if cell.cfg is not None else make_config(cell.load, cell.service_length)
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
                ag = PPOAgent(env, PPOConfig(**dict(PPO100, **(cell.ppo or {}))))
                ag.load_model(cell.weights)
                ag.eval(True)
                agent = ActStepGraph(ag, warmup=0)
            elif cell.agent not in ("firstfit", "bestfit"):
                raise ValueError(f"agent {cell.agent!r} has no batched GPU path")
            elif graph_steps:
                agent = _RecordedRollout(env, cell.agent, int(graph_steps))
        envs.append(env)
        agents.append(agent)
        streams.append(s)
        steps.append(int(cfg["eval_steps"]))
    done = [0] * len(cells)
    while any(d < t for d, t in zip(done, steps)):
        for i, (cell, env, agent, s) in enumerate(zip(cells, envs, agents, streams)):
            k = min(chunk, steps[i] - done[i])
            if k <= 0:
                continue
            with torch.cuda.stream(s):
                if agent is None:
                    env.rollout(cell.agent, k)
                elif isinstance(agent, _RecordedRollout):
                    agent.run(k)
                else:
                    for _ in range(k):
                        agent.replay()
            done[i] += k
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


# ------------------------------------------------------------ exp_performance
PERFORMANCE_HEADER = ("Agent, Load, Return, Drop Rate, Served VM, Suspend Actions, CPU Mean, "
                      "CPU Variance, Memory Mean, Memory Variance, Pending Rate, Waiting Ratio, "
                      "Slowdown Rate")
# config/10.yml's environment section (exp_performance_small.py:20)
ENV10 = dict(pms=10, vms=30, service_length=1000, arrival_rate=0.0182, training_steps=10000,
             eval_steps=100000, seed=1, reward_function="kl", cap_target_util=True,
             sequence="uniform", beta=0.5, allow_null_action=True)


def performance_config(load, reward="ut", env=ENV100, jobname=""):
    """exp_performance.py:20-33: the reward override, arrival_rate =
    round(pms / 0.55 / service_length * load, 4), and the -masked / -unmasked
    job suffixes (allow_null_action; the PPO mask follows via Cell.ppo)."""
    c = dict(env)
    c.update(reward_function=reward,
             arrival_rate=float(np.round(c["pms"] / 0.55 / c["service_length"] * load, 4)))
    if "-masked" in jobname:
        c["allow_null_action"] = True
    if "-unmasked" in jobname:
        c["allow_null_action"] = False
    return c


def performance_cell(agent, jobname, load, reward="ut", weights=None, small=False, seeds=None):
    """One evaluate() call of exp_performance.py (seeds 0..4) or
    exp_performance_small.py (config/10.yml, seeds 1..5)."""
    env = ENV10 if small else ENV100
    if seeds is None:
        seeds = tuple(range(1, 6)) if small else tuple(range(5))
    ppo = None
    if "-masked" in jobname:
        ppo = {"masked": True}
    if "-unmasked" in jobname:
        ppo = {"masked": False}
    return Cell(agent, float(load), env["service_length"], tuple(seeds), weights,
                cfg=performance_config(load, reward, env, jobname), ppo=ppo, name=jobname)


def performance_row(cell, summaries):
    """exp_performance.py:94-138 for one cell from its seeds' device summaries.
    Memory Variance keeps the reference's axis: np.var(memory, axis=0) is the
    variance over the seeds per (step, PM), = mean_s E[x^2] - E[(mean_s x)^2],
    the second term from the recorder's cross-env sums."""
    f = lambda k: float(np.mean([s[k] for s in summaries]))  # noqa: E731
    S = len(summaries)
    mem_var = f("_mem2") - sum(s["_xmem"] for s in summaries) / (S * S)
    return "%s,%.2f,%.3f,%.3f,%d,%d,%.3f,%.3f,%.3f,%.3f,%.3f,%.3f,%.3f" % (
        cell.name or cell.agent, cell.load, f("_return"), f("_drop_rate"), f("total served VMs"),
        f("total suspend actions"), f("_cpu_mean"), f("_cpu_var"), f("_mem_mean"), mem_var,
        f("_mean_pending"), f("_waiting"), f("_mean_slowdown"))


def performance_sweep(cells, eval_steps=None):
    res = run_cells(cells, eval_steps=eval_steps)
    return [performance_row(c, r) for c, r in zip(cells, res)]


# ---------------------------------------------------------------- exp_vm_size
VM_SIZE_HEADER = ("Model, Return, Drop Rate, Served VM, Suspend Actions, CPU Mean, "
                  "CPU Variance, Memory Mean, Memory Variance, Waiting Ratio")


def vm_size_config(seq, env=ENV100):
    """exp_vm_size.py:12-19: config/100.yml (reward kl) with the sequence and an
    unrounded arrival rate pms / mean size / service_length."""
    c = dict(env)
    c["sequence"] = seq
    if seq == "lowuniform":
        c["arrival_rate"] = c["pms"] / 0.375 / c["service_length"]
    elif seq == "highuniform":
        c["arrival_rate"] = c["pms"] / 0.625 / c["service_length"]
    return c


def vm_size_cell(agent, seq, weights=None, seeds=tuple(range(5))):
    return Cell(agent, 1.0, ENV100["service_length"], tuple(seeds), weights,
                cfg=vm_size_config(seq), name=agent)


def vm_size_row(cell, summaries):
    """exp_vm_size.py:60-98 (variances over PMs for both resources)."""
    f = lambda k: float(np.mean([s[k] for s in summaries]))  # noqa: E731
    return "%s,%.4f,%.4f,%d,%d,%.4f,%.4f,%.4f,%.4f,%.4f" % (
        cell.name or cell.agent, f("_return"), f("_drop_rate"), f("total served VMs"),
        f("total suspend actions"), f("_cpu_mean"), f("_cpu_var"), f("_mem_mean"),
        f("_mem_var"), f("_waiting"))


def vm_size_sweep(cells, eval_steps=None):
    res = run_cells(cells, eval_steps=eval_steps)
    return [vm_size_row(c, r) for c, r in zip(cells, res)]


# ------------------------------------------------------ exp_reward / migration
REWARD_HEADER = ("Agent, Reward, Return, Drop Rate, Served VM, Suspend Actions, CPU Mean, "
                 "CPU Variance, Memory Mean, Memory Variance, Pending Rate, Waiting Ratio, "
                 "Slowdown Rate")
MIGRATION_HEADER = "Agent,Reward,Migration Ratio,CPU,Average Slowdown"


def reward_config(reward, env=ENV100):
    """exp_reward.py:24-28 / exp_migration_ratio.py:13-16: the reward, uniform
    sizes, arrival_rate = round(pms / 0.55 / service_length, 3)."""
    c = dict(env)
    c.update(reward_function=reward, sequence="uniform",
             arrival_rate=float(np.round(c["pms"] / 0.55 / c["service_length"], 3)))
    return c


def reward_cell(agent, reward, weights=None, migration_ratio=0.002, seeds=tuple(range(5))):
    """One evaluate_seeds() call of exp_reward.py (seeds 0..4)."""
    return Cell(agent, 1.0, ENV100["service_length"], tuple(seeds), weights,
                cfg=reward_config(reward), ppo={"migration_ratio": migration_ratio},
                name=agent)


def reward_row(cell, summaries):
    """exp_reward.py:108-135 (variances over PMs for both resources)."""
    f = lambda k: float(np.mean([s[k] for s in summaries]))  # noqa: E731
    return "%s,%s,%.3f,%.3f,%d,%d,%.3f,%.3f,%.3f,%.3f,%.3f,%.3f,%.3f" % (
        cell.name or cell.agent, cell.cfg["reward_function"], f("_return"), f("_drop_rate"),
        f("total served VMs"), f("total suspend actions"), f("_cpu_mean"), f("_cpu_var"),
        f("_mem_mean"), f("_mem_var"), f("_mean_pending"), f("_waiting"), f("_mean_slowdown"))


def reward_sweep(cells, eval_steps=None):
    res = run_cells(cells, eval_steps=eval_steps)
    return [reward_row(c, r) for c, r in zip(cells, res)]


def migration_cell(agent, reward, migration_ratio, weights=None):
    """One evaluate() call of exp_migration_ratio.py (config seed 0, one run)."""
    return Cell(agent, 1.0, ENV100["service_length"], (0,), weights, cfg=reward_config(reward),
                ppo={"migration_ratio": float(migration_ratio)}, name=agent)


def migration_row(cell, summaries):
    """exp_migration_ratio.py:43-48: mean CPU and mean slowdown of the one run."""
    s = summaries[0]
    return "%s,%s,%.3f,%.3f,%.3f" % (cell.name or cell.agent, cell.cfg["reward_function"],
                                     cell.ppo["migration_ratio"], s["_cpu_mean"],
                                     s["_mean_slowdown"])


def migration_sweep(cells, eval_steps=None):
    res = run_cells(cells, eval_steps=eval_steps)
    return [migration_row(c, r) for c, r in zip(cells, res)]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("experiment", choices=["suspension", "performance", "performance_small",
                                           "vm_size", "reward", "migration_ratio"])
    ap.add_argument("--agents", default="firstfit,bestfit")
    ap.add_argument("--weights", default=None, help="PPO weights (.pt) for agent ppo")
    ap.add_argument("--seeds", default=None, help="comma list (default: the driver's seeds)")
    ap.add_argument("--loads", default=None, help="comma list (default: the reference grid)")
    ap.add_argument("--lengths", default=None, help="comma list of service lengths")
    ap.add_argument("--reward", default=None,
                    help="reward function(s): performance (default ut), reward (default wr,ut,kl)")
    ap.add_argument("--eval-steps", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    agents = a.agents.split(",")
    seeds = None if a.seeds is None else [int(x) for x in a.seeds.split(",")]
    loads = None if a.loads is None else [float(x) for x in a.loads.split(",")]
    if a.experiment == "suspension":
        header = SUSPENSION_HEADER
        rows = suspension_sweep(
            agents=agents, loads=loads,
            lengths=None if a.lengths is None else [int(x) for x in a.lengths.split(",")],
            seeds=seeds or [0], weights=a.weights, eval_steps=a.eval_steps)
    elif a.experiment in ("performance", "performance_small"):
        header = PERFORMANCE_HEADER
        small = a.experiment == "performance_small"
        reward = a.reward or "ut"
        cells = [performance_cell(ag, "ppo-" + reward if ag == "ppo" else ag, ld, reward,
                                  a.weights if ag == "ppo" else None, small, seeds)
                 for ld in (loads or [1.0]) for ag in agents]
        rows = performance_sweep(cells, eval_steps=a.eval_steps)
    elif a.experiment == "reward":
        header = REWARD_HEADER
        rewards = a.reward.split(",") if a.reward else ["wr", "ut", "kl"]
        cells = [reward_cell(ag, rw, a.weights.replace("{reward}", rw) if ag == "ppo" else None,
                             seeds=tuple(seeds) if seeds else tuple(range(5)))
                 for ag in agents for rw in rewards]
        rows = reward_sweep(cells, eval_steps=a.eval_steps)
    elif a.experiment == "migration_ratio":
        header = MIGRATION_HEADER
        ratios = [round(0.001 * i, 3) for i in range(10)]
        cells = [migration_cell(ag, rw, r, a.weights.replace("{reward}", rw)
                                if ag == "ppo" else None)
                 for r in ratios for ag in agents
                 for rw in (["ut"] if ag != "ppo" else ["wr", "ut", "kl"])]
        rows = migration_sweep(cells, eval_steps=a.eval_steps)
    else:
        header = VM_SIZE_HEADER
        cells = [vm_size_cell(ag, seq, a.weights if ag == "ppo" else None,
                              tuple(seeds) if seeds else tuple(range(5)))
                 for seq in ("lowuniform", "highuniform") for ag in agents]
        rows = vm_size_sweep(cells, eval_steps=a.eval_steps)
    text = header + "\n" + "\n".join(rows) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text, end="")


if __name__ == "__main__":
    main()
