#!/usr/bin/env python3
"""Load-time row index (k_index) timing on the bench configs: synthesises each store in HBM
(which runs k_index) a few times and prints the index kernels' time per load."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opentsdb_amd.engine import Engine  # noqa: E402

T0 = 1356998400
CONFIGS = {
    "config2": (1_000_000, T0, 3600, 1000, 0, 64, 1),
    "config3_1h": (10_000_000, T0, 360, 10000, 2, 1000, 30000),
    "config1": (1000, T0, 8640, 10000, 1, 1, 2000),
    # config 3's two row kinds alone (5M one-hour rows each): float32 / vle integers
    "c3_float": (5_000_000, T0, 360, 10000, 0, 1000, 1),
    "c3_vle": (5_000_000, T0, 360, 10000, 1, 1000, 30000),
}
eng = Engine(0)
for name in (sys.argv[1:] or CONFIGS):
    n, t0, npts, period, kind, groups, mod = CONFIGS[name]
    ms = []
    for _ in range(3):
        eng.synth(n, t0, npts, period, kind, groups, mod, 0x5EED)
        ms.append(eng.timing().index_ms)
    bytes_ = n * npts * (2 + (4 if kind == 0 else 3)) 
    print(json.dumps({"config": name, "index_ms": ms, "approx_bytes": bytes_}), flush=True)
eng.close()
