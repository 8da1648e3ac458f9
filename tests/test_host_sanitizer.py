"""The CPU runtime (csrc/host/*.cpp) under AddressSanitizer + UBSan.

SURVEY §5.2 asks for sanitizer coverage of the native code.  GPU sanitizers
are not available on the MI355X pool, so the host code is built with
``-fsanitize=address,undefined`` together with a self-test driver that drives
every exported entry point (CRD sampling in all four modes, alias tables)
and checks their invariants; a sanitizer report aborts the run."""
import shutil
import subprocess

import pytest


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_runtime_asan_ubsan(tmp_path):
    from mdistiller_ddp_amd.ops.build import build_host_sanitized
    exe = build_host_sanitized(str(tmp_path))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "OMP_NUM_THREADS": "4"})
    assert r.returncode == 0, r.stderr[-4000:]
    assert "host selftest ok" in r.stdout
