"""CPU-side checks of the C ABI: libvmp.so loads and exports every entry point
include/vmp.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "vmp.h")
LIB = os.path.join(ROOT, "vm-placement-migration-gym_amd", "vmp", "libvmp.so")


def declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*(vmp_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = declared()
    assert "vmp_step" in names and "vmp_create" in names and len(names) >= 20


@pytest.mark.skipif(not os.path.exists(LIB), reason="libvmp.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    lib.vmp_abi_version.restype = ctypes.c_int
    m = re.search(r"#define VMP_ABI_VERSION (\d+)", open(HDR).read())
    assert lib.vmp_abi_version() == int(m.group(1))


def test_python_binding_covers_header():
    from vmp import _lib
    assert sorted(_lib.EXPORTS) == declared()


def test_config_mirrors_reference_fields():
    import dataclasses
    from vmp.config import Config
    names = [f.name for f in dataclasses.fields(Config)]
    assert names == ["arrival_rate", "service_length", "pms", "vms", "training_steps",
                     "eval_steps", "seed", "reward_function", "sequence", "cap_target_util",
                     "beta", "allow_null_action"]


def test_bad_reward_raises_like_reference():
    from vmp import _lib
    from vmp.config import Config
    with pytest.raises(ValueError):
        _lib.to_c_config(Config(reward_function="nope"))
