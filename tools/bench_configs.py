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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--series", type=int, default=100_000)
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true", help="time the oracle on one group")
    args = ap.parse_args()
    from opentsdb_amd import abi, dist, synth
    from opentsdb_amd.engine import Engine

    t = time.perf_counter()
    b = synth.generate_counters(args.series, T0, 360, n_groups=args.groups, seed=0x5EED)
    gen_s = time.perf_counter() - t
    eng = Engine(0)
    t = time.perf_counter()
    eng.load(b)
    load_s = time.perf_counter() - t
    queries = {
        "sum (raw union LERP)": abi.new_query(T0, T0 + 3599, "sum"),
        "sum:rate{counter,4294967296,1000000}": abi.new_query(T0, T0 + 3599, "sum", rate=True, counter=True,
                                                              counter_max=1 << 32, reset_value=1000000),
    }
    for name, q in queries.items():
        res = eng.run(q)   # warm-up
        U = [len(g[1]) for g in res]
        k = [int((b.group_id == g[0]).sum()) for g in res]
        evals = sum(u * kk for u, kk in zip(U, k))
        ms, ev = [], []
        for _ in range(args.steps):
            t = time.perf_counter()
            eng.run(q)
            ms.append((time.perf_counter() - t) * 1000)
            tm = eng.timing()
            ev.append(tm.group_reduce_ms)
        step_ms = sum(ms) / len(ms)
        eval_ms = sum(ev) / len(ev)
        line = {
            "config": args.config, "query": name, "series": args.series, "groups": args.groups,
            "datapoints": int(tm.datapoints), "union_points": sum(U), "span_evaluations": evals,
            "ms_per_step": step_ms, "datapoints_per_s": tm.datapoints / (step_ms / 1000),
            "k_raw_eval_ms": eval_ms, "device_ms": tm.decode_downsample_ms,
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
