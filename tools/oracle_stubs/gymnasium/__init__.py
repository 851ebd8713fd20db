"""Minimal gymnasium stand-in so the reference package can be imported for
fixture generation only (gymnasium 0.28.1 is pinned by the reference but is
not installed in this image). Test infrastructure, never shipped."""
import numpy as _np
from . import spaces, envs  # noqa: F401

_REGISTRY = {}


class Env:
    np_random = None

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.np_random = _np.random.default_rng(seed)
        return None


def make(id, **kwargs):
    mod, attr = _REGISTRY[id].split(":")
    import importlib
    cls = getattr(importlib.import_module(mod), attr)
    return cls(**kwargs)
