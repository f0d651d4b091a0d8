"""A/B timing of two libtsdbhip builds on one query shape, through the bare C ABI (no engine.py,
so an older build with fewer exports loads too).  Prints one JSON line per (lib, query).

  python tools/ab_lib.py --libs a.so,b.so --config 5 --fns p99,ep99r7,median
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opentsdb_amd import abi  # noqa: E402

T0 = 1356998400


class Timing(C.Structure):   # the ABI-8 prefix of tsdbhip_timing (later fields are appended)
    _fields_ = [("decode_downsample_ms", C.c_double), ("group_reduce_ms", C.c_double), ("total_ms", C.c_double),
                ("datapoints", C.c_int64), ("bytes", C.c_int64), ("tiles", C.c_int64), ("redo_tiles", C.c_int64),
                ("fast_ms", C.c_double), ("index_ms", C.c_double), ("compact_ms", C.c_double),
                ("fused_queries", C.c_int64), ("pad", C.c_double * 8)]


def run(lib_path, cfg, fns, steps):
    L = C.CDLL(lib_path)
    vp = C.c_void_p
    L.tsdbhip_init.argtypes = [C.c_int, C.POINTER(vp)]
    L.tsdbhip_synth.argtypes = [vp, C.POINTER(abi.SynthSpec)]
    L.tsdbhip_run.argtypes = [vp, C.POINTER(abi.Query), C.POINTER(C.POINTER(abi.Result))]
    L.tsdbhip_result_free.argtypes = [C.POINTER(abi.Result)]
    L.tsdbhip_last_timing.argtypes = [vp, C.POINTER(Timing)]
    L.tsdbhip_destroy.argtypes = [vp]
    ctx = vp()
    assert L.tsdbhip_init(0, C.byref(ctx)) == 0
    if cfg == 5:
        sp = abi.SynthSpec(1_250_000, T0, 8640, 10000, 0, 64, 2000, 0x5EED)
        end, interval = T0 + 86399, 3600000
    elif cfg == 2:
        sp = abi.SynthSpec(1_000_000, T0, 3600, 1000, 0, 64, 1, 0x5EED)
        end, interval = T0 + 3599, 60000
    else:
        sp = abi.SynthSpec(10_000_000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
        end, interval = T0 + 3599, 60000
    assert L.tsdbhip_synth(ctx, C.byref(sp)) == 0
    for fn in fns:
        agg, ds = ("sum", fn) if cfg == 5 else (fn, "avg")
        if cfg == 2 and ":" in fn:
            agg, ds = fn.split(":")
            interval = {"1m": 60000, "1h": 3600000}[ds.split("-")[0]]
            ds = ds.split("-")[1]
        q = abi.new_query(T0, end, agg, ds_function=abi.AGG[ds], ds_interval_ms=interval)
        res = C.POINTER(abi.Result)()
        for _ in range(2):
            assert L.tsdbhip_run(ctx, C.byref(q), C.byref(res)) == 0
            L.tsdbhip_result_free(res)
        ms, dev = [], []
        for _ in range(steps):
            t = time.perf_counter()
            assert L.tsdbhip_run(ctx, C.byref(q), C.byref(res)) == 0
            ms.append((time.perf_counter() - t) * 1000)
            L.tsdbhip_result_free(res)
            tm = Timing()
            L.tsdbhip_last_timing(ctx, C.byref(tm))
            dev.append(tm.decode_downsample_ms)
        print(json.dumps({"lib": os.path.basename(lib_path), "config": cfg, "query": f"{agg}:{ds}",
                          "ms_per_step": sum(ms) / len(ms), "device_ms": sum(dev) / len(dev)}), flush=True)
    L.tsdbhip_destroy(ctx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--fns", default="p99,ep99r7,median")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    for lib in a.libs.split(","):
        run(lib, a.config, a.fns.split(","), a.steps)


if __name__ == "__main__":
    main()
