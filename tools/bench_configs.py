#!/usr/bin/env python3
"""Secondary BASELINE configs (the headline config 2 is bench.py).  One JSON line each.

  --config 4   100k jittered counters x 1 h (ms qualifiers), 64 groups:
               sum: without downsampling (raw union LERP, long arithmetic) and
               sum:rate{counter,2^32,1e6} (RateSpan + step semantics).
               Compute-bound: besides datapoints/s it reports span-evaluations/s
               (sum over groups of union size x spans in the group, the reference's
               O(U*k) AggregationIterator work).
  The CPU baseline is the oracle (oracle/refcpu.c, single thread) on ONE full group of the
  same workload, scaled by the number of groups (every group has the same shape).
  --config 3   the 1-GPU point of config 3: 10M series x 1 h @10 s (even series int
               [0, 30000), odd float32), {avg,min,max,count,dev}:1m-avg, 1000 groups -- one
               pass per aggregator, as the reference runs one TsdbQuery per sub-query.
  --config 5   one GPU's shard of config 5: 1.25M series x 1 day @10 s float32 (the 8-GPU
               run holds 10M), sum:1h-p99 and sum:1h-ep99r7, 64 groups.
  Configs 3 and 5 report HBM GB/s of the dominant kernel like bench.py (SURVEY 8d bytes);
  their CPU baseline is the oracle on a 256-series sample of the same query.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

T0 = 1356998400


def grid_config(args, eng, queries, n_series, n_points, value_kind, int_mod, groups, period_ms=10000):
    from opentsdb_amd import abi
    t = time.perf_counter()
    eng.synth(n_series, T0, n_points, period_ms, value_kind, groups, int_mod, 0x5EED)
    eng.sync()
    gen_s = time.perf_counter() - t
    for name, q in queries.items():
        eng.run(q)
        ms, kms = [], []
        for _ in range(args.steps):
            t = time.perf_counter()
            eng.run(q)
            ms.append((time.perf_counter() - t) * 1000)
            tm = eng.timing()
            kms.append(tm.fast_ms if tm.fast_ms > 0 and tm.redo_tiles == 0 else tm.decode_downsample_ms)
        step_ms = sum(ms) / len(ms)
        k_ms = sum(kms) / len(kms)
        line = {"config": args.config, "query": name, "series": n_series, "points": n_points, "groups": groups,
                "datapoints": int(tm.datapoints), "ms_per_step": step_ms,
                "datapoints_per_s": tm.datapoints / (step_ms / 1000), "kernel_ms": k_ms,
                "kernel": "k_fast" if tm.fast_ms > 0 and tm.redo_tiles == 0 else "decode+downsample kernels",
                "redo_tiles": int(tm.redo_tiles), "tiles": int(tm.tiles),
                "bytes": int(tm.bytes), "hbm_gbs": tm.bytes / (k_ms / 1000) / 1e9,
                "hbm_frac_of_8tbs": tm.bytes / (k_ms / 1000) / 8e12, "gen_s": gen_s}
        if args.cpu:
            from oracle import oracle as O
            from opentsdb_amd import synth
            b = synth.generate(256, T0, n_points, 10000, value_kind=value_kind, n_groups=min(groups, 256),
                               int_mod=int_mod, seed=0x5EED)
            t = time.perf_counter()
            O.run_query(b, q)
            cpu_s = time.perf_counter() - t
            line["cpu_baseline"] = {"kind": "port", "cores": 1, "sample": f"256 series x {n_points} dp, same query",
                                    "datapoints_per_s": 256 * n_points / cpu_s}
        print(json.dumps(line), flush=True)


def rollup_bench(args, eng, n_series):
    """Config 5 rollup generation over the resident batch: 1 h rollups in 1 d rows and
    1 d rollups in monthly rows, sum/count/max/min each."""
    from opentsdb_amd import engine
    tm = eng.timing()
    in_bytes = int(tm.bytes)
    for iv, span in [("1h", "1d"), ("1d", "1n")]:
        riv = engine.rollup_interval(iv, span)
        nc, nb = eng.rollup_run(riv, T0, T0 + 86400)
        ms = []
        for _ in range(args.steps):
            t = time.perf_counter()
            nc, nb = eng.rollup_run(riv, T0, T0 + 86400)
            ms.append((time.perf_counter() - t) * 1000)
        step_ms = sum(ms) / len(ms)
        rt = eng.timing()
        out_bytes = nc * (4 + 4 + 3 + 8) + nb
        line = {"config": args.config, "query": f"rollup {iv} in {span} rows x sum,count,max,min",
                "series": n_series, "datapoints": int(tm.datapoints), "cells": nc, "value_bytes": nb,
                "ms_per_step": step_ms, "datapoints_per_s": tm.datapoints / (step_ms / 1000),
                "fused_pass_ms": rt.decode_downsample_ms, "cell_write_ms": rt.group_reduce_ms,
                "fused_pass_hbm_frac_of_8tbs": in_bytes / (rt.decode_downsample_ms / 1000) / 8e12,
                "algorithmic_bytes": in_bytes + out_bytes,
                "hbm_frac_of_8tbs": (in_bytes + out_bytes) / (step_ms / 1000) / 8e12,
                "note": "one fused input pass (k_rollup_agg: sum, count, max, min per bucket), then cell "
                        "sizing / scans / writes per function"}
        print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--series", type=int, default=100_000)
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true", help="time the oracle on one group")
    ap.add_argument("--only", default="", help="comma-separated group-by aggregators to run (config 3)")
    ap.add_argument("--ordered", action="store_true", help="TSDB_QF_ORDERED (bit-exact span-order float reductions)")
    ap.add_argument("--multi", action="store_true", help="config 3: the queries through one tsdbhip_run_multi call")
    ap.add_argument("--fns", default="p99,ep99r7", help="config 5: comma-separated 1h downsampling functions")
    ap.add_argument("--dbg", type=int, default=0, help="developer option DBG (profiling switches; -DTSDBHIP_KDBG builds only)")
    ap.add_argument("--no-extra", action="store_true", help="config 5: skip the run_multi and rollup lines")
    args = ap.parse_args()
    from opentsdb_amd import abi, dist, synth
    from opentsdb_amd.engine import Engine, parse_downsample, set_option
    if args.dbg:
        set_option("DBG", args.dbg)

    def dsq(agg, spec, end):
        d = parse_downsample(spec)
        return abi.new_query(T0, end, agg, ds_function=d.ds_function, ds_interval_ms=d.ds_interval_ms,
                             ds_fill=d.ds_fill)

    if args.config == 2:   # 1M float32 series x 3600 dp @1 s, 64 groups (the bench.py workload)
        eng = Engine(0)
        series = args.series if args.series != 100_000 else 1_000_000
        aggs = args.only.split(",") if args.only else ["sum", "avg", "dev"]
        qs = {f"{a}:1m-avg": dsq(a, "1m-avg", T0 + 3599) for a in aggs}
        if args.ordered:
            for q in qs.values():
                q.flags = abi.QF_ORDERED
            qs = {k + " (ordered)": v for k, v in qs.items()}
        grid_config(args, eng, qs, series, 3600, 0, 1, args.groups, period_ms=1000)
        eng.close()
        return
    if args.config == 3:
        eng = Engine(0)
        series = args.series if args.series != 100_000 else 10_000_000
        groups = args.groups if args.groups != 64 else 1000
        aggs = args.only.split(",") if args.only else ["sum", "avg", "min", "max", "count", "dev", "p99", "median"]
        qs = {f"{a}:1m-avg": dsq(a, "1m-avg", T0 + 3599) for a in aggs}
        if args.ordered:
            for q in qs.values():
                q.flags = abi.QF_ORDERED
            qs = {k + " (ordered)": v for k, v in qs.items()}
        if args.multi:
            eng.synth(series, T0, 360, 10000, 2, groups, 30000, 0x5EED)
            eng.sync()
            ql = list(qs.values())
            eng.run_multi(ql)
            ms = []
            for _ in range(args.steps):
                t = time.perf_counter()
                eng.run_multi(ql)
                ms.append((time.perf_counter() - t) * 1000)
            tm = eng.timing()
            step = sum(ms) / len(ms)
            print(json.dumps({"config": 3, "query": "run_multi " + ",".join(qs), "series": series, "groups": groups,
                              "datapoints": int(tm.datapoints), "ms_per_step": step,
                              "fused_queries": int(tm.fused_queries), "fast_ms": tm.fast_ms, "total_ms": tm.total_ms,
                              "separate_queries_note": "compare with the per-query ms_per_step lines",
                              "datapoints_per_s_per_query": tm.datapoints * len(ql) / (step / 1000)}), flush=True)
        else:
            grid_config(args, eng, qs, series, 360, 2, 30000, groups)
        eng.close()
        return
    if args.config == 5:
        eng = Engine(0)
        series = args.series if args.series != 100_000 else 1_250_000
        qs = {f"sum:1h-{f}": dsq("sum", f"1h-{f}", T0 + 86399) for f in args.fns.split(",")}
        grid_config(args, eng, qs, series, 8640, 0, 1, args.groups)
        if args.no_extra:
            eng.close()
            return
        # four group-by aggregators over one 1h-p99 downsampling: shared selection pass
        ql = [dsq(a, "1h-p99", T0 + 86399) for a in ["sum", "max", "min", "avg"]]
        eng.run_multi(ql)
        ms = []
        for _ in range(args.steps):
            t = time.perf_counter()
            eng.run_multi(ql)
            ms.append((time.perf_counter() - t) * 1000)
        print(json.dumps({"config": 5, "query": "run_multi {sum,max,min,avg}:1h-p99", "series": series,
                          "ms_per_step": sum(ms) / len(ms)}), flush=True)
        rollup_bench(args, eng, series)
        eng.close()
        return

    t = time.perf_counter()
    b = synth.generate_counters(args.series, T0, 360, n_groups=args.groups, seed=0x5EED)
    gen_s = time.perf_counter() - t
    eng = Engine(0)
    t = time.perf_counter()
    eng.load(b)
    load_s = time.perf_counter() - t
    queries = {
        "sum (raw union LERP)": abi.new_query(T0, T0 + 3599, "sum"),
        "p99 (raw union LERP, per-point selection)": abi.new_query(T0, T0 + 3599, "p99"),
        "sum:rate{counter,4294967296,1000000}": abi.new_query(T0, T0 + 3599, "sum", rate=True, counter=True,
                                                              counter_max=1 << 32, reset_value=1000000),
    }
    for name, q in queries.items():
        res = eng.run(q)   # warm-up
        U = [len(g[1]) for g in res]
        k = [int((b.group_id == g[0]).sum()) for g in res]
        evals = sum(u * kk for u, kk in zip(U, k))
        ms, ev, cc, dv = [], [], [], []
        for _ in range(args.steps):
            t = time.perf_counter()
            eng.run(q)
            ms.append((time.perf_counter() - t) * 1000)
            tm = eng.timing()
            ev.append(tm.group_reduce_ms)
            dv.append(tm.decode_downsample_ms)
            cc.append(eng.last_call_ms)
        step_ms = sum(ms) / len(ms)
        eval_ms = sum(ev) / len(ev)
        line = {
            "config": args.config, "query": name, "series": args.series, "groups": args.groups,
            "datapoints": int(tm.datapoints), "union_points": sum(U), "span_evaluations": evals,
            "ms_per_step": step_ms, "datapoints_per_s": tm.datapoints / (step_ms / 1000),
            "k_raw_eval_ms": eval_ms, "device_ms": sum(dv) / len(dv), "c_call_ms": sum(cc) / len(cc),
            "step_ms_median": sorted(ms)[len(ms) // 2], "steps_ms": [round(x, 2) for x in ms],
            "device_steps_ms": [round(x, 2) for x in dv],
            "span_evaluations_per_s": evals / (eval_ms / 1000) if eval_ms > 0 else None,
            "gen_s": gen_s, "load_s": load_s,
        }
        if args.cpu:
            import numpy as np
            from oracle import oracle as O
            idx = np.flatnonzero(b.group_id == res[0][0])
            g0 = dist.select_series(b, idx)
            t = time.perf_counter()
            O.run_query(g0, q)
            cpu_s = time.perf_counter() - t
            line["cpu_baseline"] = {
                "kind": "port", "cores": 1,
                "sample": f"group {res[0][0]} ({len(idx)} spans) of the same query, oracle single thread",
                "sample_s": cpu_s, "span_evaluations_per_s": (U[0] * k[0]) / cpu_s,
                "datapoints_per_s": tm.datapoints / args.groups / cpu_s,
                "extrapolated_full_query_s": cpu_s * args.groups,
            }
        print(json.dumps(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
