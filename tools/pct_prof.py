#!/usr/bin/env python3
"""Profiling driver: config-5-shaped batch, NONE-aggregator 1h-p99 (k_pct_rows) and the sum
group-by over it.  usage: pct_prof.py [series] [runs]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opentsdb_amd import abi  # noqa: E402
from opentsdb_amd.engine import Engine, parse_downsample  # noqa: E402

T0 = 1356998400
n = int(sys.argv[1]) if len(sys.argv) > 1 else 312500
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
eng = Engine(0)
eng.synth(n, T0, 8640, 10000, 0, 64, 1, 0x5EED)
eng.sync()
for agg, spec in [("sum", "1h-p99"), ("sum", "1h-median")]:
    d = parse_downsample(spec)
    q = abi.new_query(T0, T0 + 86399, agg, ds_function=d.ds_function, ds_interval_ms=d.ds_interval_ms,
                      ds_fill=d.ds_fill)
    for _ in range(runs):
        eng.run(q)
    t = eng.timing()
    print(f"{agg}:{spec}: decode {t.decode_downsample_ms:.3f} ms reduce {t.group_reduce_ms:.3f} ms", flush=True)
eng.close()
