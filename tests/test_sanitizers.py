"""Host-code race / memory checking: the native core built under
ThreadSanitizer and AddressSanitizer+UBSan, running csrc/stress (concurrent epoch
cache, on-disk light cache, HostDag lazy fill, KawPow, X16R search, HeaderChain
writer + readers). Any sanitizer report fails the run (halt_on_error)."""
import os
import subprocess

import pytest


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_stress_under_sanitizer(kind, tmp_path):
    from nodexa_chain_core_amd import _build

    exe = _build.build_sanitized(kind)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path), "--quick"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "stress: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
