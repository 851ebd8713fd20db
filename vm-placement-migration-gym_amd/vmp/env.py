"""VmEnv: the reference gymnasium environment surface (vmenv/envs/env.py:19-325)
backed by one env of a BatchedVmEnv on the GPU. Numpy in, numpy out, same
observation / action / reward / info contract, so the reference agents and
drivers (main.py, src/agents/*) can use it unchanged.
"""
import copy
from typing import Optional

import numpy as np
import torch

from .batched import BatchedVmEnv
from .config import Config

try:  # gymnasium is optional: the spaces are plain attribute holders otherwise
    from gymnasium import Env as _GymEnv
    from gymnasium import spaces as _spaces
except Exception:  # pragma: no cover - image has no gymnasium
    _GymEnv = object
    _spaces = None


class _Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype


class _MultiDiscrete:
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        self.shape = self.nvec.shape


def _box(low, high, shape):
    if _spaces is not None:
        return _spaces.Box(low=low, high=high, shape=shape)
    return _Box(low, high, shape)


def _multidiscrete(nvec):
    if _spaces is not None:
        return _spaces.MultiDiscrete(nvec)
    return _MultiDiscrete(nvec)


class VmEnv(_GymEnv):
    metadata = {"render_modes": ["ansi"]}

    def __init__(self, config: Config, device="cuda"):
        self.config = config
        self.eval_mode = False
        self.action_dim = config.pms + 2 if config.allow_null_action else config.pms + 1
        self.observation_space = _box(0, config.pms + 2, (config.vms * 3 + config.pms * 2,))
        self.action_space = _multidiscrete(np.full(config.vms, self.action_dim))
        self.WAIT_STATUS = config.pms
        self.NULL_STATUS = config.pms + 1
        # an unknown reward_function fails where the reference's does: at the
        # first step that has VMs to reward (env.py:123-156 asserts in the
        # reward's else branch); until then the env runs (reward 0, no VMs)
        from ._lib import REWARDS
        self._bad_reward = None
        cfg = config
        if getattr(config, "reward_function", None) not in REWARDS:
            self._bad_reward = getattr(config, "reward_function", None)
            cfg = copy.copy(config)
            cfg.reward_function = "wr"
        self._b = BatchedVmEnv(cfg, 1, seeds=[int(config.seed)], device=device)
        self.reset(config.seed)

    # ------------------------------------------------------- state views
    def _st(self):
        return {k: v[0].cpu().numpy() for k, v in self._b.state().items()}

    @property
    def vm_placement(self):
        return self._b.state()["vm_placement"][0].cpu().numpy()

    @property
    def cpu(self):
        return self._st()["cpu"]

    @property
    def memory(self):
        return self._st()["memory"]

    @property
    def vm_cpu(self):
        return self._st()["vm_cpu"]

    @property
    def vm_memory(self):
        return self._st()["vm_memory"]

    @property
    def vm_remaining_runtime(self):
        return self._st()["vm_remaining_runtime"]

    def _ctr(self):
        return self._b.counters()[0].cpu().numpy()

    @property
    def timestep(self):
        return int(self._ctr()[5])

    def _stats(self):
        return self._b.stats()[0].cpu().numpy()

    # ---------------------------------------------------------- gym API
    def eval(self, eval_mode=True):
        self.eval_mode = eval_mode
        self._b.eval(eval_mode)

    def seed(self, seed: Optional[int] = None):
        """env.py:172-178: reseeds the four streams (and, unlike the reference,
        restarts the episode — the reference only ever calls it from reset)."""
        self.reset(self.config.seed if seed is None else seed)

    def reset(self, seed: Optional[int] = None, options=None):
        seeds = None if seed is None else torch.tensor([int(seed)], dtype=torch.int64)
        obs = self._b.reset(seeds)
        self.vm_arrival_steps = [[] for _ in range(self.config.vms)]
        return obs[0].cpu().numpy(), self._get_info()

    def step(self, action):
        action = np.asarray(action).copy()
        a = torch.as_tensor(action.astype(np.int32)).reshape(1, -1).to(self._b.device)
        pre = self.vm_placement if self.eval_mode else None
        obs, reward, done, valid = self._b.step(a)
        ts_before = self.timestep - 1
        obs = obs[0].cpu().numpy()
        if self._bad_reward is not None and np.any(obs[:self.config.vms] <= self.WAIT_STATUS):
            raise AssertionError(f"Function does not exist: {self._bad_reward}")
        # zeros_like(action) in the reference (env.py:68)
        valid = valid[0].cpu().numpy().astype(action.dtype if action.dtype.kind in "iu" else np.int64)
        info = {}
        if self.eval_mode:
            post = self.vm_placement
            # accepted this step: WAIT now, and not WAIT after the action phase
            mid = np.where(valid.astype(bool), action, pre)
            for i in np.flatnonzero((post == self.WAIT_STATUS) & (mid != self.WAIT_STATUS)):
                self.vm_arrival_steps[i].append(ts_before + 1)  # env.py:292-293
            info = self._get_info()
            self.last_validity = valid
            self.last_reward = np.round(float(reward[0]), 3)
            self.last_action = action
        info = info | {"action": action, "valid": valid}
        return obs, float(reward[0]), bool(done[0]), False, info

    def get_invalid_action_mask(self, masked: bool = True) -> np.ndarray:
        if not masked:
            return np.zeros([self.config.vms, self.action_dim], dtype=bool)
        return self._b.mask()[0].cpu().numpy()

    def _get_info(self):
        st = self._st()
        c = self._ctr()
        s = self._stats()
        return {
            "waiting_ratio": float(s[0]),
            "served_requests": int(c[1]),
            "suspend_actions": int(c[2]),
            "place_actions": int(c[3]),
            "dropped_requests": int(c[4]),
            "total_requests": int(c[0]),
            "timestep": int(c[5]),
            "vm_arrival_steps": self.vm_arrival_steps,
            "vm_placement": st["vm_placement"],
            "cpu": st["cpu"],
            "memory": st["memory"],
            "vm_cpu": st["vm_cpu"],
            "vm_memory": st["vm_memory"],
            "target_cpu_mean": float(s[1]),
            "target_memory_mean": float(s[2]),
            "total_cpu_requested": float(s[3]),
            "total_memory_requested": float(s[4]),
            "rank": int(self._b.rank()[0]),
        }

    def render(self, mode: str = "ansi", close: bool = False):
        st, c = self._st(), self._ctr()
        print(f"Timestep: \t\t{c[5]}")
        print(f"VM placement: \t\t{st['vm_placement']}")
        print(f"CPU (%): \t\t{np.array(st['cpu'] * 100, dtype=int)} {np.round(np.sum(st['cpu']), 3)}")
        print(f"Memory (%): \t\t{np.array(st['memory'] * 100, dtype=int)}")

    def close(self):
        self._b.close()
