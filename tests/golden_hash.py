"""State/obs hashing shared by the fixture generator and the parity tests.

The reference state arrays (env.py:186-196) are hashed in the reference's own
dtypes (int64 placement/runtime, float64 resources) so a hash match is a
bit-exact match of the full post-step state."""
import hashlib

import numpy as np


def _h(*arrays):
    h = hashlib.blake2b(digest_size=8)
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return np.frombuffer(h.digest(), dtype="<u8")[0]


def state_hash(placement, vm_cpu, vm_mem, cpu, mem, remaining):
    return _h(np.asarray(placement, "<i8"), np.asarray(vm_cpu, "<f8"),
              np.asarray(vm_mem, "<f8"), np.asarray(cpu, "<f8"), np.asarray(mem, "<f8"),
              np.asarray(remaining, "<i8"))


def obs_hash(obs):
    return _h(np.asarray(obs, "<f4"))
