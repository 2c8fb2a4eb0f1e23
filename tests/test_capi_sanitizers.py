"""The C ABI's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

tests/asan/build.sh compiles the library sources with the sanitizers on the host pass only
(-Xarch_host; no GPU sanitizer) and links tests/asan/capi_host_check.cpp, which drives every
validation path, error message and size / layout computation of include/*.h without a GPU.
The binary is cached under build/asan/ (rebuilt when a source is newer)."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

SOURCES = [os.path.join(REPO, "montecarlo-gated-mil_amd", "csrc", f) for f in os.listdir(
    os.path.join(REPO, "montecarlo-gated-mil_amd", "csrc"))] + \
    [os.path.join(REPO, "include", h) for h in os.listdir(os.path.join(REPO, "include"))] + \
    [os.path.join(REPO, "tests", "asan", f) for f in ("capi_host_check.cpp", "build.sh")]


def _binary():
    out = os.path.join(REPO, "build", "asan")
    exe = os.path.join(out, "capi_host_check")
    if os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(s) for s in SOURCES):
        return exe
    subprocess.run(["bash", os.path.join(REPO, "tests", "asan", "build.sh"), out], check=True,
                   capture_output=True, timeout=900)
    return exe


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_capi_host_code_under_asan_ubsan():
    exe = _binary()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
