#!/usr/bin/env python3
"""Profiling driver: config-5-shaped batch (float32 @10 s x 1 day), rollup generation and the
comparable k_fast NONE query, a few runs each.  usage: rollup_prof.py [series] [runs]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opentsdb_amd import abi, engine  # noqa: E402
from opentsdb_amd.engine import Engine, parse_downsample  # noqa: E402

T0 = 1356998400
n = int(sys.argv[1]) if len(sys.argv) > 1 else 312500
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
vk = int(sys.argv[3]) if len(sys.argv) > 3 else 0
eng = Engine(0)
eng.synth(n, T0, 8640, 10000, vk, 64, 30000 if vk == 2 else 1, 0x5EED)
eng.sync()
for iv, span in [("1h", "1d"), ("1d", "1n")]:
    riv = engine.rollup_interval(iv, span)
    for _ in range(runs):
        eng.rollup_run(riv, T0, T0 + 86400)
    t = eng.timing()
    print(f"rollup {iv}: fused {t.decode_downsample_ms:.3f} ms cells {t.group_reduce_ms:.3f} ms", flush=True)
for spec in ["1h-sum", "1h-max"]:
    d = parse_downsample(spec)
    q = abi.new_query(T0, T0 + 86399, "none", ds_function=d.ds_function, ds_interval_ms=d.ds_interval_ms,
                      ds_fill=d.ds_fill)
    for _ in range(runs):
        eng.run(q)
    t = eng.timing()
    print(f"none:{spec}: fast {t.fast_ms:.3f} ms decode {t.decode_downsample_ms:.3f} ms redo {t.redo_tiles}", flush=True)
eng.close()
