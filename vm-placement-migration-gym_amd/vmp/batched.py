"""BatchedVmEnv: N independent reference `VmEnv` instances resident on one
MI355X, stepped by libvmp.so kernels. Tensors in and out are torch tensors on
the env's device; nothing round-trips through the host on the step path.

Reference surface mapped per env (vmenv/envs/env.py):
  reset(seed)                    -> reset(seeds, mask)            env.py:180-226
  step(action)                   -> step(actions)                 env.py:66-103
  get_invalid_action_mask(True)  -> mask() / mask_bits()          env.py:45-53
  FirstFitAgent/BestFitAgent.act -> heuristic_act(policy)         firstfit.py:21, bestfit.py:21
Seeds default to config.seed + seed_stride*i (stride 4 keeps the four
per-env PCG64 streams seed+0..3 of different envs disjoint, env.py:175-178).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import VmpError, check, lib, ptr
from .config import Config

N_COUNTERS = 6  # total_requests, served, suspend, place, dropped, timestep
N_STATS = 5     # waiting_ratio, target_cpu_mean, target_mem_mean, total_cpu_req, total_mem_req
N_REC = 19      # VMP_NREC: recorder sums (include/vmp.h VMP_REC_*)
REC_BINS = 1001


class BatchedVmEnv:
    def __init__(self, config: Config, n_envs: int, seeds=None, device="cuda", seed_stride=4):
        if not torch.cuda.is_available():
            raise VmpError("BatchedVmEnv needs a HIP device (MI355X); no CPU fallback exists")
        self.config = config
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.n_envs = int(n_envs)
        if seeds is None:
            seeds = int(config.seed) + int(seed_stride) * np.arange(self.n_envs, dtype=np.int64)
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64))
        if seeds.shape != (self.n_envs,):
            raise ValueError("seeds must have shape (n_envs,)")
        self._ccfg = _lib.to_c_config(config)
        self.P, self.V = int(config.pms), int(config.vms)
        self.A = self.P + 2 if config.allow_null_action else self.P + 1
        self.D = 3 * self.V + 2 * self.P
        self.W = (self.A + 31) // 32
        self.WAIT_STATUS, self.NULL_STATUS = self.P, self.P + 1
        self.eval_mode = False
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().vmp_create(ctypes.byref(self._ccfg), self.n_envs,
                                   seeds.ctypes.data_as(ctypes.c_void_p), self.device.index,
                                   ctypes.byref(h)))
        self._h = h

    # ------------------------------------------------------------ plumbing
    def _bind(self):
        if self._h is None:
            raise VmpError("env is closed")
        s = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().vmp_set_stream(self._h, ctypes.c_void_p(s)))
        return self._h

    def _empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    def close(self):
        if getattr(self, "_h", None) is not None:
            torch.cuda.synchronize(self.device)
            lib().vmp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------- API
    def eval(self, mode=True):
        """VmEnv.eval (env.py:105-106): switches the termination limit to eval_steps."""
        self.eval_mode = bool(mode)
        check(lib().vmp_set_eval(self._bind(), int(self.eval_mode)))

    def reset(self, seeds=None, mask=None, obs=True):
        """reset(seed) for every env (or those where mask is true). seeds=None is
        reset(seed=None): the RNG streams continue (env.py:181-182)."""
        h = self._bind()
        s = None
        if seeds is not None:
            s = torch.as_tensor(seeds, dtype=torch.int64, device=self.device).contiguous()
            if s.numel() != self.n_envs:
                raise ValueError("seeds must have n_envs entries")
            if bool((s < 0).any()):
                raise ValueError("seeds must be non-negative")
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        o = self._empty((self.n_envs, self.D), torch.float32) if obs else None
        check(lib().vmp_reset(h, ptr(s), ptr(m), ptr(o)))
        return o

    def step(self, actions, obs=None, reward=None, done=None, valid=None, want_valid=True,
             bool_done=True, mask_out=None):
        """One VmEnv.step per env. actions: int tensor [N, V] on the device.
        Returns (obs f32[N,D], reward f64[N], done bool[N], valid u8[N,V]);
        bool_done=False returns the u8 done buffer itself (no conversion
        kernel: a captured step graph reads `done` in place). mask_out (int32
        [N, V, W]): also write the post-step invalid-action mask bits, what
        mask_bits() would give next (vmp_step_mask, same launch)."""
        h = self._bind()
        a = actions
        if a.dtype != torch.int32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=torch.int32).contiguous()
        if a.shape != (self.n_envs, self.V):
            raise ValueError(f"actions must have shape ({self.n_envs}, {self.V})")
        obs = self._empty((self.n_envs, self.D), torch.float32) if obs is None else obs
        reward = self._empty((self.n_envs,), torch.float64) if reward is None else reward
        done = self._empty((self.n_envs,), torch.uint8) if done is None else done
        if want_valid and valid is None:
            valid = self._empty((self.n_envs, self.V), torch.uint8)
        if mask_out is None:
            check(lib().vmp_step(h, ptr(a), ptr(obs), ptr(reward), ptr(done), ptr(valid)))
        else:
            if (mask_out.dtype != torch.int32 or not mask_out.is_contiguous()
                    or tuple(mask_out.shape) != (self.n_envs, self.V, self.W)):
                raise ValueError(f"mask_out must be contiguous int32 {(self.n_envs, self.V, self.W)}")
            check(lib().vmp_step_mask(h, ptr(a), ptr(obs), ptr(reward), ptr(done), ptr(valid),
                                      ptr(mask_out)))
        return obs, reward, done.bool() if bool_done else done, valid

    def heuristic_act(self, policy="firstfit"):
        """FirstFitAgent.act / BestFitAgent.act for every env -> int32 [N, V]."""
        h = self._bind()
        a = self._empty((self.n_envs, self.V), torch.int32)
        check(lib().vmp_heuristic_act(h, _lib.POLICIES[policy], ptr(a)))
        return a

    def heuristic_act_obs(self, obs, policy="firstfit"):
        """FirstFitAgent.act / BestFitAgent.act on the given observations (any
        f32 [N, D], not necessarily the envs' own; firstfit.py:21-38,
        bestfit.py:21-40) -> int32 [N, V]. Reads no env state."""
        h = self._bind()
        o = torch.as_tensor(obs, dtype=torch.float32, device=self.device).reshape(
            self.n_envs, self.D).contiguous()
        a = self._empty((self.n_envs, self.V), torch.int32)
        check(lib().vmp_heuristic_act_obs(h, _lib.POLICIES[policy], ptr(o), ptr(a)))
        return a

    def heuristic_step(self, policy="firstfit", want_actions=False, want_valid=False,
                       want_obs=True):
        """act(obs) then step(action) in one launch (the Base.test loop body)."""
        h = self._bind()
        a = self._empty((self.n_envs, self.V), torch.int32) if want_actions else None
        obs = self._empty((self.n_envs, self.D), torch.float32) if want_obs else None
        reward = self._empty((self.n_envs,), torch.float64)
        done = self._empty((self.n_envs,), torch.uint8)
        valid = self._empty((self.n_envs, self.V), torch.uint8) if want_valid else None
        check(lib().vmp_heuristic_step(h, _lib.POLICIES[policy], ptr(a), ptr(obs), ptr(reward),
                                       ptr(done), ptr(valid)))
        return obs, reward, done.bool(), valid, a

    def rollout(self, policy="firstfit", k_steps=1, rewards=None, done_count=None):
        """k_steps fused act+step iterations per env in one launch.
        Returns (rewards f64[k, N], done_count i64[N])."""
        h = self._bind()
        rewards = self._empty((k_steps, self.n_envs), torch.float64) if rewards is None else rewards
        if done_count is None:
            done_count = torch.zeros(self.n_envs, dtype=torch.int64, device=self.device)
        check(lib().vmp_rollout_heuristic(h, _lib.POLICIES[policy], int(k_steps), ptr(rewards),
                                          ptr(done_count)))
        return rewards, done_count

    def mask_bits(self, out=None):
        """Bit-packed invalid-action mask u32 [N, V, ceil(A/32)] (bit set = invalid)."""
        h = self._bind()
        b = self._empty((self.n_envs, self.V, self.W), torch.int32) if out is None else out
        if b.shape != (self.n_envs, self.V, self.W) or b.dtype != torch.int32 or not b.is_contiguous():
            raise ValueError("mask_bits out must be contiguous int32 [N, V, W]")
        check(lib().vmp_mask(h, ptr(b)))
        return b

    def mask(self):
        """get_invalid_action_mask(masked=True) as bool [N, V, A] (env.py:45-53)."""
        h = self._bind()
        m = self._empty((self.n_envs, self.V, self.A), torch.uint8)
        check(lib().vmp_mask_bool(h, ptr(m)))
        return m.bool()

    def obs(self):
        h = self._bind()
        o = self._empty((self.n_envs, self.D), torch.float32)
        check(lib().vmp_get_obs(h, ptr(o)))
        return o

    def counters(self):
        h = self._bind()
        c = self._empty((self.n_envs, N_COUNTERS), torch.int64)
        check(lib().vmp_get_counters(h, ptr(c)))
        return c

    def stats(self):
        h = self._bind()
        s = self._empty((self.n_envs, N_STATS), torch.float64)
        check(lib().vmp_get_stats(h, ptr(s)))
        return s

    def state(self):
        """Reference-dtype state tensors: placement/remaining int64 [N,V],
        vm_cpu/vm_mem f64 [N,V], cpu/mem f64 [N,P]."""
        h = self._bind()
        N, V, P = self.n_envs, self.V, self.P
        pl, rem = self._empty((N, V), torch.int64), self._empty((N, V), torch.int64)
        vc, vm = self._empty((N, V), torch.float64), self._empty((N, V), torch.float64)
        c, m = self._empty((N, P), torch.float64), self._empty((N, P), torch.float64)
        check(lib().vmp_get_state(h, ptr(pl), ptr(vc), ptr(vm), ptr(c), ptr(m), ptr(rem)))
        return dict(vm_placement=pl, vm_cpu=vc, vm_memory=vm, cpu=c, memory=m,
                    vm_remaining_runtime=rem)

    # ------------------------------------------------ eval-mode Record metrics
    def record(self, on=True):
        """Start (on=True, right after reset, as Base.test does) or stop recording
        the Record metrics of every env on the device (vmp_record_enable)."""
        check(lib().vmp_record_enable(self._bind(), int(bool(on))))

    def record_read(self):
        """(hist u32 [N, 2, 1001] pending/slowdown rate counts, sums f64 [N, 16])."""
        h = self._bind()
        hist = self._empty((self.n_envs, 2, REC_BINS), torch.int32)
        sums = self._empty((self.n_envs, N_REC), torch.float64)
        check(lib().vmp_record_read(h, ptr(hist), ptr(sums)))
        return hist, sums

    def record_summary(self):
        """Record.get_summary() (record.py:110-134) of every env -> list of dicts."""
        from .record import summary_from_device
        hist, sums = self.record_read()
        ctr, st = self.counters().cpu().numpy(), self.stats().cpu().numpy()
        hist, sums = hist.cpu().numpy().view(np.uint32), sums.cpu().numpy()
        return [summary_from_device(hist[i], sums[i], ctr[i], st[i], self.P)
                for i in range(self.n_envs)]

    def rank(self):
        h = self._bind()
        r = self._empty((self.n_envs,), torch.int64)
        check(lib().vmp_get_rank(h, ptr(r)))
        return r

    # ------------------------------------------------- checkpoint / resume
    def snapshot(self):
        """The whole batched env state (vmp_snapshot: PCG64 streams, counters,
        PM and VM words) as a device u8 tensor; `restore` on an env of the same
        config and n_envs continues bit-exactly from here. torch.save it for a
        resumable run."""
        h = self._bind()
        n = ctypes.c_int64()
        check(lib().vmp_snapshot_bytes(h, ctypes.byref(n)))
        buf = self._empty((n.value,), torch.uint8)
        check(lib().vmp_snapshot(h, ptr(buf)))
        return buf

    def restore(self, snap):
        """Load a `snapshot()` (any device or host tensor) into this env."""
        h = self._bind()
        s = torch.as_tensor(snap).to(device=self.device, dtype=torch.uint8).contiguous()
        n = ctypes.c_int64()
        check(lib().vmp_snapshot_bytes(h, ctypes.byref(n)))
        if s.numel() != n.value:
            raise ValueError(f"snapshot holds {s.numel()} bytes, this env needs {n.value}")
        check(lib().vmp_restore(h, ptr(s)))
        torch.cuda.current_stream(self.device).synchronize()  # s may be a temporary copy
