"""bench.py's command-line contract on a machine without the GPUs it is asked for: `--gpus N`
(no launcher) must refuse with exit status 2 instead of reporting a smaller run as N GPUs."""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_more_gpus_than_visible_exits_2():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "1", "--warmup", "0",
                        "--no-config3", "--md-timeout", "120"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300, cwd=ROOT)
    assert r.returncode == 2, r.stderr.decode(errors="replace")[-2000:]
    err = r.stderr.decode(errors="replace")
    assert "refusing to report" in err
    assert not r.stdout.strip(), "no bench line may be printed"
