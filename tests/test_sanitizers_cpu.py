"""Host-code sanitizers: the C oracle built with AddressSanitizer + UndefinedBehaviorSanitizer
(-fno-sanitize-recover) and driven through clustering (both presets), alignment with CIGARs, DUST and k-mer
extraction on seeded structured UMIs (oracle/asan_main.c).  A sanitizer report fails the test.  (GPU code
is not sanitized: GPU ASan / XNACK runs are unavailable on the GPU pool.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_oracle_under_asan_ubsan(tmp_path):
    out = str(tmp_path)
    b = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan_check", f"OUT={out}"],
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(out, "orc_asan_check"), "2500"], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.strip().endswith("ok")
    assert "runtime error" not in r.stderr
