"""Config 3's full day on one GPU's share: N series x 8640 dp @10 s (int/float32 alternating),
1000 groups, sum with 1m / 10m / 1h avg downsampling (K = 1440 / 144 / 24 slots): the shape each
GPU holds in bench.py's strong-scaled config3_strong block.  With --multi, also the five
aggregators avg/min/max/count/dev:1m-avg through one tsdbhip_run_multi (k_hwin's MULTI pass).
Prints one JSON line per query."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0 = 1356998400
IV = {"1m": 60000, "10m": 600000, "1h": 3600000}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1_250_000)
    ap.add_argument("--hours", type=int, default=24)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--only", default="1m,10m,1h")
    ap.add_argument("--multi", action="store_true")
    a = ap.parse_args()
    from opentsdb_amd import abi
    from opentsdb_amd.engine import Engine
    eng = Engine(0)
    eng.synth(a.series, T0, a.hours * 360, 10000, 2, 1000, 30000, 0x5EED)
    eng.sync()

    def q(agg, iv):
        return abi.new_query(T0, T0 + a.hours * 3600 - 1, agg, ds_function=abi.AGG["avg"], ds_interval_ms=IV[iv])

    def timed(fn):
        fn()
        eng.sync()
        t = time.perf_counter()
        kms, fms = [], []
        for _ in range(a.steps):
            fn()
            tm = eng.timing()
            kms.append(tm.decode_downsample_ms)
            fms.append(tm.fast_ms)
        eng.sync()
        return (time.perf_counter() - t) * 1000 / a.steps, sum(kms) / len(kms), sum(fms) / len(fms), eng.timing()

    sum_ms = {}
    for iv in a.only.split(","):
        ms, k, f, tm = timed(lambda: eng.run(q("sum", iv)))
        sum_ms[iv] = ms
        print(json.dumps({"query": f"sum:{iv}-avg", "series": a.series, "hours": a.hours, "ms_per_step": ms,
                          "decode_downsample_ms": k, "fast_ms": f, "redo_tiles": int(tm.redo_tiles),
                          "tiles": int(tm.tiles), "bytes": int(tm.bytes),
                          "hbm_frac_kernel": tm.bytes / (k / 1000) / 8e12,
                          "hbm_frac_step": tm.bytes / (ms / 1000) / 8e12}), flush=True)
    if a.multi:
        aggs = ["avg", "min", "max", "count", "dev"]
        ms, k, f, tm = timed(lambda: eng.run_multi([q(x, "1m") for x in aggs]))
        print(json.dumps({"query": "{" + ",".join(aggs) + "}:1m-avg run_multi", "series": a.series, "hours": a.hours,
                          "ms_per_step": ms, "fused_queries": int(tm.fused_queries), "decode_downsample_ms": k,
                          "fast_ms": f, "hbm_frac_kernel": tm.bytes / (k / 1000) / 8e12,
                          "ratio_to_sum_step": ms / sum_ms["1m"] if "1m" in sum_ms else None}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
