"""ctypes binding of libvmp.so (include/vmp.h). The HIP library is the only
compute path: importing this module on a machine without the built library
or without a HIP device raises; there is no CPU fallback."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VMP_LIB_PATH") or os.path.join(_HERE, "libvmp.so")

REWARDS = {"wr": 0, "ut": 1, "kl": 2}
SEQUENCES = {"uniform": 0, "lowuniform": 1, "highuniform": 2}
POLICIES = {"firstfit": 0, "bestfit": 1}

EXPORTS = (
    "vmp_abi_version", "vmp_last_error", "vmp_create", "vmp_destroy", "vmp_set_stream",
    "vmp_set_eval", "vmp_dims", "vmp_reset", "vmp_step", "vmp_heuristic_act",
    "vmp_heuristic_act_obs",
    "vmp_heuristic_step", "vmp_rollout_heuristic", "vmp_mask", "vmp_mask_bool", "vmp_get_obs",
    "vmp_get_counters", "vmp_get_stats", "vmp_get_state", "vmp_get_rank", "vmp_gae",
    "vmp_policy_head", "vmp_policy_head_backward", "vmp_policy_head_backward_bf16",
    "vmp_actor_head", "vmp_actor_head_bf16_fwd", "vmp_actor_head_bf16_sample",
    "vmp_actor_head_bf16_bwd",
    "vmp_actor_head_bf16_bwd_workspace", "vmp_actor_mlp_packed_floats", "vmp_actor_mlp_pack",
    "vmp_actor_mlp_f32", "vmp_actor_mlp_head_f32", "vmp_step_mask", "vmp_record_enable",
    "vmp_record_read", "vmp_snapshot_bytes", "vmp_snapshot", "vmp_restore",
    "vmp_debug_fail_alloc", "vmp_debug_live_allocs", "vmp_debug_stamps", "vmp_debug_occupancy",
    "vmp_debug_quiet_violations",
)


class VmpConfig(ctypes.Structure):
    """`vmp_config` (include/vmp.h), mirrors vmenv/envs/config.py:4-15."""
    _fields_ = [("arrival_rate", ctypes.c_double), ("service_length", ctypes.c_double),
                ("pms", ctypes.c_int32), ("vms", ctypes.c_int32),
                ("training_steps", ctypes.c_int64), ("eval_steps", ctypes.c_int64),
                ("seed", ctypes.c_int64), ("reward_function", ctypes.c_int32),
                ("sequence", ctypes.c_int32), ("cap_target_util", ctypes.c_int32),
                ("allow_null_action", ctypes.c_int32), ("beta", ctypes.c_double)]


def to_c_config(cfg):
    if cfg.reward_function not in REWARDS:
        # env.py:156 asserts 'Function does not exist'
        raise ValueError(f"Function does not exist: {cfg.reward_function}")
    if cfg.sequence not in SEQUENCES:
        raise AttributeError(f"unknown sequence {cfg.sequence!r}")  # env.py:222 fails likewise
    return VmpConfig(float(cfg.arrival_rate), float(cfg.service_length), int(cfg.pms),
                     int(cfg.vms), int(cfg.training_steps), int(cfg.eval_steps), int(cfg.seed),
                     REWARDS[cfg.reward_function], SEQUENCES[cfg.sequence],
                     int(bool(cfg.cap_target_util)), int(bool(cfg.allow_null_action)),
                     float(cfg.beta))


class VmpError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libvmp.so (built in-tree by __graft_entry__.build() / make)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VmpError(f"{LIB_PATH} is missing: run `make -C vm-placement-migration-gym_amd` "
                       "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    P, i32, i64, u64, f32 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64,
                             ctypes.c_float)
    sig = {
        "vmp_abi_version": (ctypes.c_int, []),
        "vmp_last_error": (ctypes.c_char_p, []),
        "vmp_create": (ctypes.c_int, [P, i32, P, i32, ctypes.POINTER(ctypes.c_void_p)]),
        "vmp_destroy": (ctypes.c_int, [P]),
        "vmp_set_stream": (ctypes.c_int, [P, P]),
        "vmp_set_eval": (ctypes.c_int, [P, i32]),
        "vmp_dims": (ctypes.c_int, [P, P, P, P, P, P]),
        "vmp_reset": (ctypes.c_int, [P, P, P, P]),
        "vmp_step": (ctypes.c_int, [P, P, P, P, P, P]),
        "vmp_step_mask": (ctypes.c_int, [P, P, P, P, P, P, P]),
        "vmp_heuristic_act": (ctypes.c_int, [P, i32, P]),
        "vmp_heuristic_act_obs": (ctypes.c_int, [P, i32, P, P]),
        "vmp_heuristic_step": (ctypes.c_int, [P, i32, P, P, P, P, P]),
        "vmp_rollout_heuristic": (ctypes.c_int, [P, i32, i32, P, P]),
        "vmp_mask": (ctypes.c_int, [P, P]),
        "vmp_mask_bool": (ctypes.c_int, [P, P]),
        "vmp_get_obs": (ctypes.c_int, [P, P]),
        "vmp_get_counters": (ctypes.c_int, [P, P]),
        "vmp_get_stats": (ctypes.c_int, [P, P]),
        "vmp_get_state": (ctypes.c_int, [P, P, P, P, P, P, P]),
        "vmp_get_rank": (ctypes.c_int, [P, P]),
        "vmp_gae": (ctypes.c_int, [i32, i32, P, P, P, P, f32, f32, P, P, P]),
        "vmp_policy_head": (ctypes.c_int, [i32, i32, i32, i32, P, P, f32, i32, u64, u64, P, P, P,
                                            P, P, P]),
        "vmp_policy_head_backward": (ctypes.c_int, [i32, i32, i32, P, P, P, P, P, P, P]),
        "vmp_policy_head_backward_bf16": (ctypes.c_int, [i32, i32, i32, P, P, P, P, P, P, P]),
        "vmp_actor_head": (ctypes.c_int, [i32, i32, i32, i32, i32, P, P, P, P, f32, i32, u64, u64,
                                           P, P, P, P, P, P, P]),
        "vmp_actor_head_bf16_fwd": (ctypes.c_int, [i32, i32, i32, i32, P, P, P, P, P, P, P, P, P]),
        "vmp_actor_head_bf16_sample": (ctypes.c_int, [i32, i32, i32, i32, P, P, P, P, f32, i32,
                                                       u64, u64, P, P, P, P, P, P]),
        "vmp_actor_head_bf16_bwd": (ctypes.c_int, [i32, i32, i32, i32, P, P, P, P, P, P, P, P,
                                                    i32, P, P, P]),
        "vmp_actor_head_bf16_bwd_workspace": (ctypes.c_int64, [i32, i32, i32]),
        "vmp_actor_mlp_packed_floats": (ctypes.c_int64, [i32, i32, i32, i32]),
        "vmp_actor_mlp_pack": (ctypes.c_int, [i32, i32, i32, i32, P, P, P, P, P]),
        "vmp_actor_mlp_f32": (ctypes.c_int, [i32, i32, i32, i32, i32, P, P, P, P, P, P, P]),
        "vmp_actor_mlp_head_f32": (ctypes.c_int, [i32, i32, i32, i32, i32, i32, P, P, P, P, P, P,
                                                   f32, i32, u64, u64, P, i32, P, P, P, P, P]),
        "vmp_record_enable": (ctypes.c_int, [P, i32]),
        "vmp_record_read": (ctypes.c_int, [P, P, P]),
        "vmp_snapshot_bytes": (ctypes.c_int, [P, P]),
        "vmp_snapshot": (ctypes.c_int, [P, P]),
        "vmp_restore": (ctypes.c_int, [P, P]),
        "vmp_debug_fail_alloc": (ctypes.c_int, [i32]),
        "vmp_debug_live_allocs": (ctypes.c_int64, []),
        "vmp_debug_stamps": (ctypes.c_int, [P, P]),
        "vmp_debug_occupancy": (ctypes.c_int, [P, P, P]),
        "vmp_debug_quiet_violations": (ctypes.c_int, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name, None)
        if f is None and name.startswith("vmp_debug_"):
            continue  # diagnostics an older build may lack
        if f is None:
            raise VmpError(f"libvmp lacks {name}")
        f.restype, f.argtypes = res, args
    if L.vmp_abi_version() != 11:
        raise VmpError("libvmp ABI mismatch")
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise VmpError(f"libvmp error {rc}: {lib().vmp_last_error().decode()}")
    return rc


def ptr(t):
    """Device (or host) address of a torch tensor, None for None."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())
