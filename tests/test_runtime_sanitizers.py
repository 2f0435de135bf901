"""Native runtime (block manager + scheduler + constrained-decoding matcher) randomised self-test under ASan + UBSan."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_selftest_asan_ubsan(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools/sanitize_runtime.sh"), "4"], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime selftest OK" in r.stdout
    assert "grammar selftest:" in r.stdout  # constrained-decoding matcher walks
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
