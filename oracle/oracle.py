"""ctypes binding of the C oracle (oracle/vmp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker. The product path never imports it.

`OracleEnv` mirrors the reference `VmEnv` (vmenv/envs/env.py) method for method
on a single env, with the reference's dtypes (int64 placement, float64 state).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libvmp_oracle.so")

REWARDS = {"wr": 0, "ut": 1, "kl": 2}
SEQUENCES = {"uniform": 0, "lowuniform": 1, "highuniform": 2}


class VmpConfig(ctypes.Structure):
    """Byte layout of `vmp_config` in include/vmp.h (config.py:4-15 fields)."""
    _fields_ = [("arrival_rate", ctypes.c_double), ("service_length", ctypes.c_double),
                ("pms", ctypes.c_int32), ("vms", ctypes.c_int32),
                ("training_steps", ctypes.c_int64), ("eval_steps", ctypes.c_int64),
                ("seed", ctypes.c_int64), ("reward_function", ctypes.c_int32),
                ("sequence", ctypes.c_int32), ("cap_target_util", ctypes.c_int32),
                ("allow_null_action", ctypes.c_int32), ("beta", ctypes.c_double)]


def make_config(d):
    """dict with the reference Config field names -> VmpConfig."""
    full = dict(arrival_rate=0.182, service_length=100, pms=10, vms=30, training_steps=500,
                eval_steps=100000, seed=0, reward_function="wr", sequence="uniform",
                cap_target_util=True, beta=0.5, allow_null_action=False)
    full.update(d)
    return VmpConfig(float(full["arrival_rate"]), float(full["service_length"]),
                     int(full["pms"]), int(full["vms"]), int(full["training_steps"]),
                     int(full["eval_steps"]), int(full["seed"]),
                     REWARDS[full["reward_function"]], SEQUENCES[full["sequence"]],
                     int(bool(full["cap_target_util"])), int(bool(full["allow_null_action"])),
                     float(full["beta"]))


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, i64, i32, u64, dbl = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                 ctypes.c_uint64, ctypes.c_double)
        sig = {
            "oracle_create": (P, [P]), "oracle_destroy": (None, [P]),
            "oracle_reset": (None, [P, ctypes.c_int, i64]), "oracle_set_eval": (None, [P, ctypes.c_int]),
            "oracle_step": (None, [P, P, P, P, P]), "oracle_obs": (None, [P, P]),
            "oracle_mask": (None, [P, P]), "oracle_firstfit": (None, [P, P]),
            "oracle_bestfit": (None, [P, P]), "oracle_rank": (i64, [P]),
            "oracle_get_state": (None, [P] * 7), "oracle_get_counters": (None, [P, P, P]),
            "oracle_pcg_seed": (None, [u64, P]), "oracle_pcg_raw": (None, [u64, i64, P]),
            "oracle_pcg_double": (None, [u64, i64, P]),
            "oracle_pcg_around": (None, [u64, i64, dbl, dbl, P]),
            "oracle_pcg_poisson": (u64, [u64, dbl, i64, P]),
            "oracle_pcg_advance_raw": (u64, [u64, u64]),
            "oracle_pw_sum": (dbl, [P, i64]), "oracle_argsort_f32": (None, [P, i64, P]),
            "oracle_rollout": (i64, [P, i32, i64, i64, i64, i32, i32, i32, P, P]),
            "oracle_rollout_timed": (None, [P, i32, i64, i64, i64, i64, i32, i32, i32, i32, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """Single reference-semantics env (env.py:19-325) on the CPU."""

    def __init__(self, cfg: dict):
        self.cfg = dict(cfg)
        self._c = make_config(self.cfg)
        self.P, self.V = self._c.pms, self._c.vms
        self.A = self.P + 2 if self._c.allow_null_action else self.P + 1
        self.D = 3 * self.V + 2 * self.P
        self.WAIT_STATUS, self.NULL_STATUS = self.P, self.P + 1
        self._h = lib().oracle_create(ctypes.byref(self._c))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_destroy(self._h)
            self._h = None

    def eval(self, mode=True):
        lib().oracle_set_eval(self._h, int(mode))

    def reset(self, seed=None):
        lib().oracle_reset(self._h, 0 if seed is None else 1, 0 if seed is None else int(seed))
        return self.obs()

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.int64)
        valid = np.zeros(self.V, np.uint8)
        r = ctypes.c_double()
        t = ctypes.c_int()
        lib().oracle_step(self._h, _p(a), _p(valid), ctypes.byref(r), ctypes.byref(t))
        return self.obs(), r.value, bool(t.value), valid

    def obs(self):
        o = np.zeros(self.D, np.float32)
        lib().oracle_obs(self._h, _p(o))
        return o

    def mask(self):
        m = np.zeros((self.V, self.A), np.uint8)
        lib().oracle_mask(self._h, _p(m))
        return m.astype(bool)

    def firstfit(self):
        a = np.zeros(self.V, np.int64)
        lib().oracle_firstfit(self._h, _p(a))
        return a

    def bestfit(self):
        a = np.zeros(self.V, np.int64)
        lib().oracle_bestfit(self._h, _p(a))
        return a

    def rank(self):
        return lib().oracle_rank(self._h)

    def state(self):
        pl = np.zeros(self.V, np.int64)
        vc, vm = np.zeros(self.V), np.zeros(self.V)
        c, m = np.zeros(self.P), np.zeros(self.P)
        rem = np.zeros(self.V, np.int64)
        lib().oracle_get_state(self._h, _p(pl), _p(vc), _p(vm), _p(c), _p(m), _p(rem))
        return pl, vc, vm, c, m, rem

    def counters(self):
        c = np.zeros(6, np.int64)
        st = np.zeros(5)
        lib().oracle_get_counters(self._h, _p(c), _p(st))
        return c, st


def rollout(cfg: dict, n_env, seed0, stride, steps, policy=0, eval_mode=True, threads=1):
    """OpenMP batched heuristic rollout (the CPU baseline). Returns
    (reward_sum[n_env], counters[n_env, 6])."""
    c = make_config(cfg)
    rs = np.zeros(n_env)
    ctr = np.zeros((n_env, 6), np.int64)
    lib().oracle_rollout(ctypes.byref(c), n_env, seed0, stride, steps, policy, int(eval_mode),
                         threads, _p(rs), _p(ctr))
    return rs, ctr


def rollout_timed(cfg: dict, n_env, seed0, stride, warmup, steps, policy=0, threads=1,
                  eval_mode=False, reps=1):
    """Warm-started timed CPU rollout (bench.py cpu_baseline): `reps` timed
    passes of `steps` steps over the same window (the envs are restored to
    their post-warm-up state before every pass, untimed), so every pass does
    identical work. Returns (seconds[reps], reward_sum[reps, n_env])."""
    c = make_config(cfg)
    rs = np.zeros((reps, n_env))
    secs = np.zeros(reps)
    lib().oracle_rollout_timed(ctypes.byref(c), n_env, seed0, stride, warmup, steps, policy,
                               threads, int(eval_mode), reps, _p(secs), _p(rs))
    return secs, rs
