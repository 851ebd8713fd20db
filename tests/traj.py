"""Replay of the golden trajectories (tests/golden/traj_*.npz) against any
backend that exposes the reference VmEnv surface. Shared by the oracle tests
(CPU) and the HIP parity tests (GPU)."""
import glob
import json
import os

import numpy as np

from tests.golden_hash import obs_hash, state_hash

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def traj_names():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN, "traj_*.npz")))


def load(name):
    z = np.load(os.path.join(GOLDEN, "traj_%s.npz" % name), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["config"] = json.loads(str(d["config"]))
    d["rewards"] = json.loads(str(d["rewards"]))
    d["policy"] = str(d["policy"])
    for k in ("T", "eval_mode", "reset_none_at"):
        d[k] = int(d[k])
    return d


def sparse_actions(d):
    """{step: (vm_idx, targets, valid)} from the fixture's sparse action stream."""
    out = {}
    st, vm, tg, va = d["act_step"], d["act_vm"], d["act_tgt"], d["act_valid"]
    bounds = np.flatnonzero(np.diff(st)) + 1
    for lo, hi in zip(np.r_[0, bounds], np.r_[bounds, st.size]):
        if hi > lo:
            out[int(st[lo])] = (vm[lo:hi], tg[lo:hi], va[lo:hi])
    return out


def kl_close(a, b):
    return abs(a - b) <= 1e-12 * max(1.0, abs(b))
