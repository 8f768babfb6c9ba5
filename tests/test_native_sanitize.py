"""Host-native C++ under AddressSanitizer + UBSan: the pybind11
module is compiled into an instrumented executable and the repo's native-facing
tests (AES-GCM NIST vectors, envelope rotation, guided-decoding grammar) run
inside it.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("python3-config") is None,
                    reason="needs g++ and python3-config")
def test_native_code_clean_under_asan_ubsan(tmp_path):
    env = dict(os.environ, OUT=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "native_sanitize.sh")],
                       capture_output=True, text=True, env=env, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "<builtin, sanitized>" in out  # the instrumented module was the one exercised
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out
    assert " passed" in out
