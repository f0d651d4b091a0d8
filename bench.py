#!/usr/bin/env python3
"""Benchmark of the OpenTSDB query-aggregation hot path on MI355X (libtsdbhip).

Workload (BASELINE.json configs[1] = BASELINE.md config 2): 1,000,000 series x 1 h
@ 1 s float32 (3.6e9 raw datapoints, ~21.6 GB of compacted cells resident in HBM),
query sum:1m-avg grouped by a 64-valued tag.  A "step" is one full tsdbhip_run over the
resident cells: decode -> 1m-avg downsample -> 64-group sum -> results on the host.

Multi-GPU (torch.distributed.run, one process per GPU): weak scaling -- every rank holds
its own 1M-series shard (disjoint series ids); per-(group, slot) partial states are
all-gathered over RCCL and merged in rank order (tsdbhip_partials_* in the C ABI).

Prints ONE JSON line on rank 0 (see README / DESIGN.md for the fields).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

T0 = 1356998400
BYTES_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--series", type=int, default=1_000_000, help="series per GPU")
    ap.add_argument("--points", type=int, default=3600)
    ap.add_argument("--period-ms", type=int, default=1000)
    ap.add_argument("--groups", type=int, default=64)
    ap.add_argument("--interval", default="1m")
    ap.add_argument("--ds", default="avg")
    ap.add_argument("--agg", default="sum")
    ap.add_argument("--value-kind", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline work (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(args, target_s: float):
    """Oracle (oracle/refcpu.c, the C port of the reference CPU path) on a bounded
    sample of the same workload, single thread, on this host."""
    from oracle import oracle as O
    from opentsdb_amd import abi, synth
    n = 256
    b = synth.generate(n, T0, args.points, args.period_ms, value_kind=args.value_kind,
                       n_groups=min(args.groups, n), seed=0x5EED)
    q = query(args)
    t = time.perf_counter()
    O.run_query(b, q)
    dt = time.perf_counter() - t
    reps = max(1, int(target_s / max(dt, 1e-3)))
    t = time.perf_counter()
    for _ in range(reps):
        O.run_query(b, q)
    dt = time.perf_counter() - t
    dps = n * args.points * reps
    return {"value": dps / dt, "unit": "datapoints/s", "cores": 1, "kind": "port",
            "sample": f"{n} series x {args.points} dp ({args.ds} {args.interval}, {args.agg} over "
                      f"{min(args.groups, n)} groups), {reps} reps, {dt:.1f} s, oracle/refcpu.c single thread"}


def query(args):
    from opentsdb_amd import abi, engine
    q = abi.new_query(T0, T0 + args.points * args.period_ms // 1000 - 1, args.agg)
    ds = engine.parse_downsample(f"{args.interval}-{args.ds}")
    q.ds_function, q.ds_interval_ms, q.ds_fill = ds.ds_function, ds.ds_interval_ms, ds.ds_fill
    return q


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_
        torch.cuda.set_device(local_rank)
        dist_.init_process_group("nccl")
        dist = dist_
    from opentsdb_amd.engine import Engine
    from opentsdb_amd import abi

    eng = Engine(local_rank)
    t_gen = time.perf_counter()
    eng.synth(args.series, T0, args.points, args.period_ms, args.value_kind, args.groups, 2000,
              0x5EED ^ (rank * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF))
    eng.sync()
    t_gen = time.perf_counter() - t_gen
    q = query(args)

    def step():
        if dist is None:
            return eng.run(q)
        return eng.run_distributed(q, dist, args.groups)

    for _ in range(args.warmup):
        step()
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    eng.sync()
    kernel_ms = []
    reduce_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        tm = eng.timing()
        kernel_ms.append(tm.decode_downsample_ms)
        reduce_ms.append(tm.group_reduce_ms)
    eng.sync()
    if dist is not None:
        import torch
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tm = eng.timing()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    dps_step = tm.datapoints * world
    value = dps_step / (ms_per_step / 1000.0)
    k_avg = sum(kernel_ms) / len(kernel_ms)
    achieved = tm.bytes / (k_avg / 1000.0) / 1e9
    if rank == 0:
        cpu = None if args.no_cpu_baseline else cpu_baseline(args, args.cpu_seconds)
        line = {
            "metric": "raw datapoints/sec through downsample+group-by; % of HBM BW, 1-8 GPUs",
            "value": value,
            "unit": "datapoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded splitmix64, generated in HBM with the MockBase cell encoding)",
            "config": {
                "workload": f"{args.agg}:{args.interval}-{args.ds} group-by {args.groups} groups over "
                            f"{args.series} series/GPU x {args.points} dp @{args.period_ms} ms "
                            f"({'float32' if args.value_kind == 0 else 'int/mixed'}) -- BASELINE config 2",
                "series_per_gpu": args.series,
                "datapoints_per_gpu": tm.datapoints,
                "groups": args.groups,
                "parallelism": f"series-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": BYTES_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / BYTES_PEAK_GBS,
                "traffic": None,
                "kernel": "k_grid (fused decode+downsample+tile group partials)",
                "kernel_ms": k_avg,
                "bytes_per_launch": tm.bytes,
                "group_reduce_ms": sum(reduce_ms) / len(reduce_ms),
            },
            "cpu_baseline": cpu,
            "synth_s": t_gen,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
