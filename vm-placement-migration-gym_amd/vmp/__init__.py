"""vmp — MI355X-native batched VM placement/migration environment.

Drop-in for the reference's `VmEnv` gym plugin path (vmenv/__init__.py:3-6) and
the heuristic / PPO agents that drive it (src/agents/*). The compute path is
libvmp.so (HIP, gfx950); see include/vmp.h for the C ABI.
"""
from .config import Config  # noqa: F401

__all__ = ["Config", "VmEnv", "BatchedVmEnv", "register"]


def __getattr__(name):  # lazy: importing torch-backed pieces needs a HIP device later
    if name == "VmEnv":
        from .env import VmEnv
        return VmEnv
    if name == "BatchedVmEnv":
        from .batched import BatchedVmEnv
        return BatchedVmEnv
    raise AttributeError(name)


def register():
    """register(id="VmEnv-v1", ...) exactly as vmenv/__init__.py:3-6 does, so
    gym.make("VmEnv-v1", config=Config(...)) builds the GPU env."""
    from gymnasium.envs.registration import register as _reg
    _reg(id="VmEnv-v1", entry_point="vmp.env:VmEnv")
