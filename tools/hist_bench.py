"""Histogram-path benchmark: a synthetic store of SimpleHistogram columns
(the bytes TSDB.addHistogramPoint writes), loaded once, then TsdbQuery.runHistogram-shaped
queries timed on the device.

    python tools/hist_bench.py [--series 20000] [--buckets 20] [--period 10] [--hours 1]
                               [--groups 64] [--ds 1m-sum] [--steps 10] [--check] [--unsorted N]

--unsorted N: the first two columns of the first row of N series (spread over the groups) trade
qualifiers, so those spans yield a receding timestamp; with --ds none their groups take
k_hist_walk (HistogramAggregationIterator's greedy walk) instead of the sorted union path.

One JSON line: columns/s and the algorithmic bytes rate of the query (value bytes of the columns
plus 21 B of per-column index: column offset 8, position->column 8, kind 1, slot 4).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from opentsdb_amd import abi  # noqa: E402
from opentsdb_amd import engine as E  # noqa: E402
from opentsdb_amd import histogram as H  # noqa: E402

T0 = 1356998400


def synth(n_series, n_buckets, period_s, hours, groups, seed=1, unsorted=0):
    """Vectorised SimpleHistogram columns: one layout (log-spaced buckets), counts 0..999
    (1-2 byte varints), underflow / overflow < 128."""
    rng = np.random.default_rng(seed)
    per_row = 3600 // period_s
    n_rows = n_series * hours
    n = n_rows * per_row
    edges = np.geomspace(1.0, 10000.0, n_buckets + 1).astype(np.float32)
    keyb = np.ascontiguousarray(np.stack([edges[:-1], edges[1:]], 1).astype(">f4")).view(np.uint8).reshape(n_buckets, 8)
    cnt = rng.integers(0, 1000, (n, n_buckets), dtype=np.int64)
    W = 3 + n_buckets * 10 + 2
    mat = np.zeros((n, W), np.uint8)
    msk = np.zeros((n, W), bool)
    mat[:, 0] = 0          # codec id
    mat[:, 1] = 0
    mat[:, 2] = n_buckets
    msk[:, :3] = True
    for b in range(n_buckets):
        o = 3 + 10 * b
        mat[:, o:o + 8] = keyb[b]
        msk[:, o:o + 8] = True
        c = cnt[:, b]
        two = c >= 128
        mat[:, o + 8] = np.where(two, (c & 0x7F) | 0x80, c)
        mat[:, o + 9] = np.where(two, c >> 7, 0)
        msk[:, o + 8] = True
        msk[:, o + 9] = two
    mat[:, W - 2] = rng.integers(0, 128, n)
    mat[:, W - 1] = rng.integers(0, 128, n)
    msk[:, W - 2:] = True
    vlen = msk.sum(1)
    val = mat[msk]
    voff = np.zeros(n + 1, np.uint64)
    np.cumsum(vlen, out=voff[1:])
    offs = np.arange(per_row, dtype=np.int64) * period_s
    q1 = np.stack([np.full(per_row, 6, np.uint8), (offs >> 8).astype(np.uint8), (offs & 0xFF).astype(np.uint8)], 1)
    qual = np.tile(q1.reshape(-1), n_rows)
    if unsorted:   # columns 0 and 1 of the series' first row trade qualifiers (a receding timestamp)
        for sr in np.linspace(0, n_series - 1, unsorted).astype(np.int64):
            c0 = int(sr) * hours * per_row
            a, b = qual[3 * c0:3 * c0 + 3].copy(), qual[3 * c0 + 3:3 * c0 + 6].copy()
            qual[3 * c0:3 * c0 + 3], qual[3 * c0 + 3:3 * c0 + 6] = b, a
    qoff = np.arange(n + 1, dtype=np.uint64) * 3
    srp = np.arange(n_series + 1, dtype=np.int64) * hours
    base = np.tile(T0 + 3600 * np.arange(hours, dtype=np.int64), n_series).astype(np.uint32)
    rcp = np.arange(n_rows + 1, dtype=np.int64) * per_row
    gid = (np.arange(n_series) % groups).astype(np.int32)
    return H.HostHistBatch(srp, base, rcp, qoff, voff, qual, val, gid, {0: H.HCODEC_SIMPLE}), int(val.size)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=20000)
    ap.add_argument("--buckets", type=int, default=20)
    ap.add_argument("--period", type=int, default=10)
    ap.add_argument("--hours", type=int, default=1)
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--ds", default="1m-sum")
    ap.add_argument("--agg", default="sum")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--buckets-out", action="store_true", help="show_buckets")
    ap.add_argument("--check", action="store_true", help="compare with the oracle (test infrastructure)")
    ap.add_argument("--unsorted", type=int, default=0, help="series with a receding timestamp (k_hist_walk groups)")
    a = ap.parse_args()
    t = time.time()
    hb, vbytes = synth(a.series, a.buckets, a.period, a.hours, a.groups, unsorted=a.unsorted)
    synth_s = time.time() - t
    n = int(hb.cell_val_off.size - 1)
    eng = E.Engine(0)
    t = time.time()
    eng.load_histograms(hb)
    load_s = time.time() - t
    q = abi.new_query(T0, T0 + 3600 * a.hours - 1, a.agg)
    if a.ds != "none":
        d = E.parse_downsample(a.ds)
        q.ds_function, q.ds_interval_ms, q.ds_all, q.ds_calendar = d.ds_function, d.ds_interval_ms, d.ds_all, d.ds_calendar
    pcts = [50.0, 95.0, 99.0]
    for _ in range(a.warmup):
        res = eng.run_histogram(q, pcts, a.buckets_out)
    eng.sync()
    t = time.perf_counter()
    for _ in range(a.steps):
        res = eng.run_histogram(q, pcts, a.buckets_out)
    eng.sync()
    dt = (time.perf_counter() - t) / a.steps
    points = sum(len(g[0].ts) for g in res if g)
    alg = vbytes + 21 * n
    line = {"metric": "histogram columns/s through decode + downsample + group-by + percentiles",
            "value": n / dt, "unit": "columns/s", "ms_per_query": dt * 1e3, "columns": n, "value_bytes": vbytes,
            "algorithmic_bytes": alg, "GBps_alg": alg / dt / 1e9, "points_out": points, "groups": len(res),
            "config": {"series": a.series, "buckets": a.buckets, "period_s": a.period, "hours": a.hours,
                       "groups": a.groups, "downsample": a.ds, "aggregator": a.agg, "percentiles": pcts,
                       "show_buckets": a.buckets_out, "unsorted_series": a.unsorted},
            "synth_s": synth_s, "load_s": load_s}
    if a.check:
        from oracle import oracle as O
        from tests import hist_util as U
        want = O.run_hist(hb, q, pcts, a.buckets_out)
        U.same(res, want, "bench")
        line["check"] = "bit-exact vs oracle"
    print(json.dumps(line))
    eng.close()


if __name__ == "__main__":
    main()
