"""Host-side race / memory checks: the native runtime's host-only code
(csrc/runtime/ordered_worker.h -- the background staging worker and the bucket planner) built
and run under AddressSanitizer + UBSan and under ThreadSanitizer (scripts/host_sanitize.sh).
GPU sanitizers are not available on this pool; this is the CPU half."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_host_runtime_clean_under_asan_ubsan_tsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "host_sanitize.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "host sanitizers: clean" in r.stdout
