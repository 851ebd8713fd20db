"""SURVEY §5 sanitizer builds (the reference has none), on CPU:

  - the C oracle under AddressSanitizer and under UndefinedBehaviorSanitizer
    (oracle/Makefile `asan` / `ubsan`, driver oracle/sanitize_main.c: every
    oracle entry point the tests use, FirstFit / BestFit / perturbed external
    actions incl. invalid and negative ones, wr / ut / kl, the three
    sequences, drops, reset(seed=None), the OpenMP baseline, tie-heavy and
    NaN argsort, the RNG known-answer entry points);
  - the library's host code (csrc/vmp_capi.cpp) under ASan + UBSan with the
    normal gfx950 kernel objects (vm-placement-migration-gym_amd/Makefile
    `sanitize`), driven by tests/native/capi_faults.cpp: every entry point's
    null-argument checks, vmp_create's config validation and its clean
    failure without a device. The same binary's `--device` mode (allocation
    failures injected at every point of vmp_create / vmp_record_enable /
    vmp_mask_bool) runs on the GPU box: tests/test_gpu_sanitizers.py.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "vm-placement-migration-gym_amd")


def _run(cmd, env=None, timeout=600):
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    return out


def test_oracle_under_asan_and_ubsan():
    _run(["make", "-s", "-C", "oracle", "asan", "ubsan"])
    out = _run([os.path.join(ROOT, "oracle", "build", "oracle_asan")],
               {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert "oracle sanitize ok" in out
    out = _run([os.path.join(ROOT, "oracle", "build", "oracle_ubsan")],
               {"UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"})
    assert "oracle sanitize ok" in out


def test_capi_host_code_under_asan_ubsan():
    _run(["make", "-s", "-j", "8", "-C", PKG, "sanitize"], timeout=1500)
    out = _run([os.path.join(PKG, "build", "san", "capi_faults")],
               {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"})
    assert "capi faults ok" in out
    assert out.count("ok  EINVAL") >= 30
