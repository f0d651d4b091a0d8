"""Rollup read-path benchmark: a rollup table scanned as tsdbhip_load_rollup
takes it (RollupSpan / RollupSeq rows of value cells and count cells), then rollup queries timed
on the device.

    python tools/rollup_read_bench.py [--series 1000000] [--days 1] [--interval 10m] [--span 1d]
                                      [--groups 64] [--steps 10] [--check]

Table: --series series x --days days of --interval rollups in --span rows, every cell present:
sum cells as float64 (8-byte values, flags 0xF), count cells as 1-byte longs (flags 0x0) -- what
TSDB.addAggregatePoint stores for a double sum and a small count.  Queries: avg:1h-avg (value and
count series: two SUM passes + k_rollup_combine + the group-by), sum:1h-sum and max:1h-max (value
series only).  One JSON line per query: datapoints/s (rollup cells read per second) and the
algorithmic bytes rate (per cell read: 2 B qualifier + value bytes; per row 4 B base time + 2 x 8 B
offsets).  --check runs the oracle (oracle.run_rollup_query) on a 200-series slice of the same
table and compares."""
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

T0 = 1356998400


def table(n_series, days, interval, span, groups, seed=7):
    iv = E.rollup_interval(interval, span)
    step = iv.interval_s
    ts = np.arange(T0, T0 + days * 86400, step, dtype=np.int64)
    bases = np.array([E.rollup_basetime(int(t), iv) for t in ts], np.int64)
    offs = (ts - bases) // step
    ub, first = np.unique(bases, return_index=True)
    per_row = np.diff(np.append(first, len(ts)))
    nrow_s = len(ub)
    rng = np.random.default_rng(seed)
    n = len(ts)
    cnt = rng.integers(1, 61, (n_series, n), dtype=np.int64)
    sums = (cnt * rng.normal(100.0, 20.0, (n_series, n))).astype(">f8")
    vq1 = ((offs << 4) | 0xF).astype(">u2").view(np.uint8)
    cq1 = ((offs << 4) | 0x0).astype(">u2").view(np.uint8)
    qual = np.tile(vq1, n_series)
    cqual = np.tile(cq1, n_series)
    val = sums.view(np.uint8).reshape(-1)
    cval = cnt.astype(np.int8).view(np.uint8).reshape(-1)
    cells_per_row = np.tile(per_row, n_series)
    ncell = np.concatenate([[0], np.cumsum(cells_per_row)]).astype(np.uint64)
    srp = np.arange(n_series + 1, dtype=np.int64) * nrow_s
    base_t = np.tile(ub, n_series).astype(np.uint32)
    gid = (np.arange(n_series) * groups // n_series).astype(np.int32)
    cells = abi.HostBatch(srp, base_t, ncell * 2, ncell * 8, qual, val, gid)
    rb = abi.HostRollupBatch(cells, (ncell * 2, ncell, cqual, cval), iv)
    return rb, n_series * n


def query(spec, agg, t1):
    q = abi.new_query(T0, t1, agg)
    d = E.parse_downsample(spec)
    q.ds_function, q.ds_interval_ms = d.ds_function, d.ds_interval_ms
    return q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1_000_000)
    ap.add_argument("--days", type=int, default=1)
    ap.add_argument("--interval", default="10m")
    ap.add_argument("--span", default="1d")
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--opt", action="append", default=[], help="developer option NAME=VALUE (A/B runs)")
    a = ap.parse_args()
    for kv in a.opt:
        k, v = kv.split("=")
        E.set_option(k, v)
    t = time.perf_counter()
    rb, n_cells = table(a.series, a.days, a.interval, a.span, a.groups)
    gen_s = time.perf_counter() - t
    eng = E.Engine(0)
    t = time.perf_counter()
    eng.load_rollup(rb)
    eng.sync()
    load_s = time.perf_counter() - t
    t1 = T0 + a.days * 86400 - 1
    for agg, spec in (("avg", "1h-avg"), ("sum", "1h-sum"), ("max", "1h-max")):
        q = query(spec, agg, t1)
        for _ in range(2):
            eng.run(q)
        eng.sync()
        t = time.perf_counter()
        cc = 0.0
        for _ in range(a.steps):
            eng.run(q)
            cc += eng.last_call_ms
        eng.sync()
        ms = (time.perf_counter() - t) * 1000 / a.steps
        tm = eng.timing()
        reads_counts = agg == "avg"
        # value cells: 2 B qualifier + 8 B value; count cells: 2 B + 1 B; per row 4 + 16 B
        nrows = int(rb.cells.n_series * (len(rb.cells.row_base_time) // max(1, rb.cells.n_series)))
        alg = n_cells * (10 + (3 if reads_counts else 0)) + nrows * (20 * (2 if reads_counts else 1))
        line = {"workload": f"rollup table {a.series} series x {a.days} d of {a.interval} rollups in {a.span} rows "
                            f"(sum float64 + count cells), {a.groups} groups",
                "query": f"{agg}:{spec}", "ms_per_step": ms, "cells": n_cells,
                "cells_per_s": n_cells / (ms / 1000), "algorithmic_bytes": alg,
                "algorithmic_GBps": alg / (ms / 1000) / 1e9, "hbm_frac_of_8tbs": alg / (ms / 1000) / 8e12,
                "device_decode_downsample_ms": tm.decode_downsample_ms, "group_reduce_ms": tm.group_reduce_ms,
                "c_call_ms": cc / a.steps, "device_total_ms": tm.total_ms,
                "gen_s": gen_s, "load_s": load_s}
        if a.check:
            from oracle import oracle as O
            from tests.test_gpu_parity import assert_groups_match
            sub = 200
            rb2, _ = table(sub, a.days, a.interval, a.span, min(a.groups, sub))
            eng2 = E.Engine(0)
            eng2.load_rollup(rb2)
            assert_groups_match(eng2.run(q), O.run_rollup_query(rb2, q), agg, tol=1e-12, ctx=f"{agg}:{spec}")
            eng2.close()
            line["check"] = f"oracle == GPU on a {sub}-series table of the same shape"
        print(json.dumps(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
