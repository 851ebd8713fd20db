"""Workgroup start/end clocks of k_env_big (C5, BestFit kl) from a -DVMP_WGTIME
variant: how many workgroups share a CU, when they start, how long one lives.
Usage: VMP_STAMP_BUF=1 VMP_LIB_PATH=.../libvmp_wgtime.so python tools/wgtime.py [envs] [P] [V]"""
import os
import sys
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vm-placement-migration-gym_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vmp import _lib  # noqa: E402
from vmp.batched import BatchedVmEnv  # noqa: E402
from vmp.config import Config  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
P = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
V = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
cfg = Config(pms=P, vms=V, arrival_rate=round(1000 / 0.55 / 1000, 3), service_length=1000,
             training_steps=10000, eval_steps=100000, seed=0, reward_function="kl",
             sequence="uniform", cap_target_util=True, beta=0.5, allow_null_action=True)
env = BatchedVmEnv(cfg, N, seeds=4 * np.arange(N, dtype=np.int64), device="cuda:0")
for _ in range(8):
    env.rollout("bestfit", 250)
import ctypes  # noqa: E402
nb, lb = ctypes.c_int32(0), ctypes.c_int32(0)
_lib.check(_lib.lib().vmp_debug_occupancy(env._bind(), ctypes.addressof(nb), ctypes.addressof(lb)))
print(f"occupancy: {nb.value} workgroups per CU at {lb.value} B of LDS")
buf = torch.zeros((N, 24), dtype=torch.int64, device="cuda")
for rep in range(3):
    c0 = env.counters().cpu().numpy().copy()
    env.heuristic_step("bestfit")
    torch.cuda.synchronize()
    _lib.check(_lib.lib().vmp_debug_stamps(env._bind(), _lib.ptr(buf)))
    torch.cuda.synchronize()
    s = buf.cpu().numpy()
    t0, t1 = s[:, 0] - s[:, 0].min(), s[:, 1] - s[:, 0].min()
    hw, xcc = s[:, 5].astype(np.int64), s[:, 7].astype(np.int64)
    cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 0x7) << 5) | ((xcc & 0xF) << 8)
    per_cu = Counter(cu.tolist())
    dur = (t1 - t0) / 100.0  # us (100 MHz)
    print(f"N={N} rep {rep}: span {t1.max() / 100:.1f} us, wg duration mean {dur.mean():.1f} "
          f"min {dur.min():.1f} max {dur.max():.1f} us; start spread: "
          f"{np.percentile(t0 / 100, [0, 25, 50, 75, 90, 100]).round(1).tolist()} us; "
          f"CUs used {len(per_cu)}, WGs per CU {sorted(Counter(per_cu.values()).items())}")
    groups = defaultdict(list)
    for i, c in enumerate(cu.tolist()):
        groups[c].append(i)
    ov = [min(t1[a], t1[b]) - max(t0[a], t0[b]) for g in groups.values() if len(g) == 2 for a, b in [g]]
    if ov:
        print(f"   pairs sharing a CU: {len(ov)}, overlap mean {np.mean(ov) / 100:.1f} us")
    # duration against the step's events (vmp_get_counters columns: total_requests, served, suspend, place, dropped, timestep)
    dc = env.counters().cpu().numpy() - c0
    names = ["c%d" % i for i in range(dc.shape[1])]
    for i in range(dc.shape[1]):
        if dc[:, i].std() > 0:
            r = np.corrcoef(dc[:, i], dur)[0, 1]
            print(f"   counter {i}: mean {dc[:, i].mean():.2f}, corr with duration {r:+.2f}")
    pl = dc[:, 3]  # place_action
    ties = s[:, 23]
    print(f"   BestFit tie sorts per env-step: mean {ties.mean():.2f} (envs with >= 1: {(ties > 0).mean():.2f}); "
          f"duration with ties {dur[ties > 0].mean() if (ties > 0).any() else 0:.1f} us, without {dur[ties == 0].mean():.1f} us")
    # phases between the stamp points (slot = STAMP id; 0 start, 1 end)
    seq = [(0, "start"), (13, "prologue"), (16, "heuristic"), (8, "run: time words"),
           (9, "run: row counts"), (10, "run: rank+frees"), (2, "run: null"), (14, "acc: null counts"),
           (15, "acc: draw+assign"), (3, "acc: state store"),
           (11, "rank+compact"), (17, "A: obs issue (w0)"), (18, "A: w0 sum tasks"), (20, "A: barrier"),
           (19, "B: w0 sum tasks"), (21, "B: barrier"), (12, "stats final"),
           (4, "tail-rest"), (6, "mask/hdr"), (1, "end")]
    prev = s[:, 0].astype(np.float64)
    parts = []
    for sl, nm in seq[1:]:
        cur = s[:, sl].astype(np.float64)
        ok = cur > 0
        d = np.where(ok, cur - prev, 0.0) / 100.0
        parts.append((nm, d.mean(), d[pl == 0].mean() if (pl == 0).any() else 0.0, np.corrcoef(d, pl)[0, 1] if d.std() > 0 else 0.0))
        prev = np.where(ok, cur, prev)
    print("   phase                mean us   (0-placement envs)  corr(placements)")
    for nm, a, b, r in parts:
        print(f"   {nm:20s} {a:8.2f}   {b:8.2f}   {r:+.2f}")
    for k in sorted(set(pl.tolist()))[:8]:
        m = pl == k
        print(f"   placements {k}: {m.sum()} envs, duration mean {dur[m].mean():.1f} us")
