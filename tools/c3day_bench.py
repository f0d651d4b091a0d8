"""Config 3's full day on one GPU's share: N series x 8640 dp @10 s (int/float32 alternating),
1000 groups, sum with 1m / 10m / 1h avg downsampling (K = 1440 / 144 / 24 slots): the shape each
GPU holds in bench.py's strong-scaled config3_strong block.  Prints one JSON line per query."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0 = 1356998400


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1_250_000)
    ap.add_argument("--hours", type=int, default=24)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from opentsdb_amd import abi
    from opentsdb_amd.engine import Engine
    eng = Engine(0)
    eng.synth(a.series, T0, a.hours * 360, 10000, 2, 1000, 30000, 0x5EED)
    eng.sync()
    for iv in ("1m", "10m", "1h"):
        q = abi.new_query(T0, T0 + a.hours * 3600 - 1, "sum", ds_function=abi.AGG["avg"],
                          ds_interval_ms={"1m": 60000, "10m": 600000, "1h": 3600000}[iv])
        eng.run(q)
        eng.sync()
        t = time.perf_counter()
        kms = []
        for _ in range(a.steps):
            eng.run(q)
            tm = eng.timing()
            kms.append(tm.decode_downsample_ms)
        eng.sync()
        ms = (time.perf_counter() - t) * 1000 / a.steps
        tm = eng.timing()
        k = sum(kms) / len(kms)
        print(json.dumps({"query": f"sum:{iv}-avg", "series": a.series, "hours": a.hours, "ms_per_step": ms,
                          "decode_downsample_ms": k, "fast_ms": tm.fast_ms, "redo_tiles": int(tm.redo_tiles),
                          "tiles": int(tm.tiles), "bytes": int(tm.bytes),
                          "hbm_frac_kernel": tm.bytes / (k / 1000) / 8e12}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
