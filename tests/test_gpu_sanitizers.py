"""The C ABI's device failure paths under the host sanitizers, on the MI355X
(tests/native/capi_faults.cpp `--device`, built on CPU by
tests/test_sanitizers_cpu.py / `make -C vm-placement-migration-gym_amd
sanitize`): for every allocation of vmp_create the injected out-of-memory
returns VMP_EOOM with no host leak (LeakSanitizer) and the device memory back
to its starting level; vmp_record_enable failing at each of its 9
allocations leaves the handle usable; vmp_mask_bool likewise; a full
create / BestFit steps / record / destroy cycle runs clean. Host-only
instrumentation: the kernels are the normal gfx950 objects."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "vm-placement-migration-gym_amd", "build", "san", "capi_faults")


def test_capi_device_failure_paths_under_asan_ubsan():
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} is missing: build it on the CPU side (make sanitize)")
    # protect_shadow_gap=0: the HIP runtime maps device-visible memory where
    # ASan would otherwise reserve its shadow gap
    env = dict(os.environ,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:protect_shadow_gap=0",
               LSAN_OPTIONS="suppressions=" + os.path.join(ROOT, "tests", "native", "lsan.supp"),
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([EXE, "--device"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=120)
    out = p.stdout + p.stderr
    print(out[-3000:])
    assert p.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
    assert "device failure paths" in out and "capi faults ok" in out
