"""Agent base and the heuristic agents on the GPU env.

Reference: src/agents/base.py:13-136 (Base: set_log / test / record_testing_step),
src/agents/firstfit.py:21-38 and src/agents/bestfit.py:21-40. Same constructor
signatures and methods; act(observation) runs the heuristic scan in a HIP
kernel on the observation it is given (vmp_heuristic_act_obs).
"""
from dataclasses import asdict, dataclass, is_dataclass
from time import gmtime, strftime

import numpy as np

from .record import Record


@dataclass
class Config:
    pass


def _asdict(c):
    return asdict(c) if is_dataclass(c) else dict(vars(c))


def batched_env(env):
    """The BatchedVmEnv behind a vmp.VmEnv (or the env itself)."""
    return getattr(env, "_b", env)


class Base:
    def __init__(self, name: str, env, config):
        self.name = name
        self.env = env
        self.config = Config() if config is None else config
        self.record = Record(self.name, _asdict(self.env.config), _asdict(self.config))
        self.writer = None
        self.total_steps = 0
        self.rng = np.random.default_rng(self.env.config.seed)

    def set_log(self, jobname, logdir):
        """base.py:30-44; tensorboard is optional in this image (no-op without it)."""
        if not logdir:
            return
        try:
            from torch.utils.tensorboard import SummaryWriter
        except Exception:
            print("tensorboard is not installed: logging disabled")
            return
        self.writer = SummaryWriter(f"{logdir}/{strftime('%Y%m%d', gmtime())}-{self.name}-{jobname}")

    def learn(self):
        raise NotImplementedError

    def act(self, observation):
        raise NotImplementedError

    def save_model(self, modelpath):
        raise NotImplementedError

    def load_model(self, modelpath):
        raise NotImplementedError

    def eval(self, mode=True):
        raise NotImplementedError

    def test(self, show: bool = False, output: str = None, debug: bool = False):
        """base.py:63-118: one eval episode (eval_steps) from reset(seed=config.seed),
        every step recorded; returns the Record (saved to `output` if given). The
        Record metrics are accumulated on the device during the episode
        (vmp_record_*); the host keeps the per-step traces of the JSON. Each
        call starts a fresh Record (the reference appends the traces of every
        call while replacing vm_arrival_steps, so a second test() would pair
        two episodes' placements with one episode's arrivals): the saved
        traces and the summary always describe the same episode."""
        self.record.clear()
        self.env.eval()
        self.eval()
        obs, info = self.env.reset(seed=self.env.config.seed)
        dev = batched_env(self.env)
        dev.record(True)  # right after reset, as base.py:67-71 records from there
        done = False
        while not done:
            if debug:
                self.env.render()
            action = self.act(obs)
            obs, reward, done, _, info = self.env.step(action)
            if debug:
                print("action: \t\t%s" % (np.asarray(action).flatten()))
                print("validity: \t\t%s" % (info["valid"]))
                print("reward: \t\t%.2f" % (reward))
                print("")
            self.record_testing_step(reward, info)
        self.record.set_device_summary(dev.record_summary()[0])
        dev.record(False)
        summary = self.record.get_summary()
        if show:
            print(self.env.config)
            for k, v in summary.items():
                print("%s: %.2f" % (k, v))
            print("cpu: %s" % (info["cpu"]))
            print("memory: %s" % (info["memory"]))
        if output:
            self.record.save(output)
        return self.record

    def end_log(self):
        if self.writer:
            self.writer.close()

    def record_testing_step(self, reward: float, info):  # base.py:120-136
        r = self.record
        r.cpu.append(info["cpu"])
        r.memory.append(info["memory"])
        r.used_pm.append(len(info["cpu"]) - np.count_nonzero(info["cpu"]))  # empty PMs (quirk 12)
        r.vm_placements.append(info["vm_placement"])
        r.waiting_ratio.append(info["waiting_ratio"])
        r.actions.append(info["action"])
        r.rewards.append(reward)
        r.dropped_requests.append(info["dropped_requests"])
        r.total_requests.append(info["total_requests"])
        r.vm_arrival_steps = info["vm_arrival_steps"]
        r.target_cpu_mean.append(info["target_cpu_mean"])
        r.target_memory_mean.append(info["target_memory_mean"])
        r.served_requests.append(int(info["served_requests"]))
        r.total_cpu_requested = info["total_cpu_requested"]
        r.total_memory_requested = info["total_memory_requested"]
        r.suspended.append(info["suspend_actions"])
        r.placed.append(info["place_actions"])
        r.rank.append(info["rank"])


ACT_OBS_MAX_P = 9045  # vmp_heuristic_act_obs: 18 P + 1024 B of LDS <= 160 KB


class _HeuristicAgent(Base):
    POLICY = None

    def __init__(self, env):
        super().__init__(type(self).__name__, env, None)

    def learn(self):
        pass

    def load_model(self, modelpath):
        pass

    def save_model(self, modelpath):
        pass

    def eval(self, mode=True):
        pass

    def act(self, observation):
        """The heuristic's action computed from `observation` -> int64 [V] (or
        [N, V] for a BatchedVmEnv's [N, D] observations), as the reference
        reads only the obs it is passed (firstfit.py:22-28): an edited or stale
        observation gets its own action, not the env's. The scan runs in the
        HIP kernel (vmp_heuristic_act_obs); Base.test's fused act+step path
        (vmp_heuristic_step) acts on the env state, which is that obs."""
        b = batched_env(self.env)
        if b.P > ACT_OBS_MAX_P:
            # k_act_obs holds the PM view in one workgroup's LDS; beyond that the
            # env-state scan (vmp_heuristic_act) serves the env's own observation
            import torch
            o = torch.as_tensor(observation, dtype=torch.float32, device=b.device)
            if not torch.equal(o.reshape(b.n_envs, b.D), b.obs()):
                raise ValueError(f"act() on an edited observation supports P <= {ACT_OBS_MAX_P} "
                                 f"(this env has P = {b.P}); pass the env's own observation")
            a = b.heuristic_act(self.POLICY).cpu().numpy().astype(np.int64)
        else:
            a = b.heuristic_act_obs(observation, self.POLICY).cpu().numpy().astype(np.int64)
        return a[0] if b is not self.env else a


class FirstFitAgent(_HeuristicAgent):
    """firstfit.py:21-38: first PM (index order) that fits in f32, cpu-only update."""
    POLICY = "firstfit"


class BestFitAgent(_HeuristicAgent):
    """bestfit.py:21-40: feasible PM with the largest f32 cpu+mem, numpy scalar
    introsort tie order."""
    POLICY = "bestfit"
