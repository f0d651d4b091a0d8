"""The CPU oracle under AddressSanitizer + UBSan: oracle/san_driver.c runs the
restatement over every row shape and query kind; a leak, overflow or undefined behaviour fails
the run.  tools/oracle_san.sh additionally runs the whole CPU suite on the UBSan library."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_asan_ubsan_driver():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True)
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "san_driver")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "clean" in r.stdout
    assert "ERROR" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
