"""Sequential (Java-order) float64 sums: full-mantissa doubles (ROW_NOCERT rows) downsampled with
sum / avg, which k_seq_wave (one wave a series) or k_seq_dense (one series a lane,
--seq-wave 0) run.   python tools/seq_bench.py [--series 200000] [--points 360] [--steps 5]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opentsdb_amd import abi, synth  # noqa: E402
from opentsdb_amd.engine import Engine, set_option  # noqa: E402

T0 = 1356998400


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=200_000)
    ap.add_argument("--points", type=int, default=360)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--seq-wave", type=int, default=1, help="0: k_seq_dense (developer option SEQ_WAVE)")
    a = ap.parse_args()
    if a.seq_wave == 0:
        set_option("SEQ_WAVE", 0)
    b = synth.generate(a.series, T0, a.points, 10000, value_kind=4, n_groups=64, seed=23)
    eng = Engine(0)
    eng.load(b)
    for ds in ("sum", "avg"):
        q = abi.new_query(T0, T0 + a.points * 10 - 1, "sum", ds_function=abi.AGG[ds], ds_interval_ms=60000)
        eng.run(q)
        eng.sync()
        t = time.perf_counter()
        for _ in range(a.steps):
            eng.run(q)
        eng.sync()
        ms = (time.perf_counter() - t) * 1000 / a.steps
        n = a.series * a.points
        print(json.dumps({"query": f"sum:1m-{ds} over full-mantissa float64", "series": a.series, "points": a.points,
                          "seq_wave": a.seq_wave, "ms_per_step": ms,
                          "device_ms": eng.timing().decode_downsample_ms, "datapoints_per_s": n / (ms / 1000),
                          "value_bytes_GBps": n * 10 / (ms / 1000) / 1e9}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
