#!/usr/bin/env python3
"""Benchmark of the OpenTSDB query-aggregation hot path on MI355X (libtsdbhip).

Workload (BASELINE.json configs[1] = BASELINE.md config 2): 1,000,000 series x 1 h
@ 1 s float32 (3.6e9 raw datapoints, ~21.6 GB of compacted cells resident in HBM),
query sum:1m-avg grouped by a 64-valued tag.  A "step" is one full tsdbhip_run over the
resident cells: decode -> 1m-avg downsample -> 64-group sum -> results on the host.

Multi-GPU, two launch forms, both weak scaling by default (1M series per GPU):
  * `python bench.py --gpus N` (no launcher): ONE process drives N distinct GPUs through one
    multi-device context (tsdbhip_init_devices, the handle a TSD JVM would hold): series-sharded
    shards, per-(group, slot) partial states gathered to devices[0] with RCCL send / recv over
    xGMI and merged in device order.  Exits non-zero when fewer than N GPUs are visible.
  * `torch.distributed.run --nproc-per-node N bench.py --gpus N`: one process per GPU, each
    rank its own shard, partial states all-gathered over RCCL (tsdbhip_partials_* in the C ABI).

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
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: --series per GPU (each rank its own store); strong: --series in total, one global "
                         "store split over the ranks (tsdbhip_synth_shard), e.g. config 3's 10M series 1/2/4/8 ways")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline work (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 FETCH/WRITE_SIZE child passes")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 (10M series) block in `extra`")
    ap.add_argument("--no-config5", action="store_true", help="--gpus N > 1: skip the config-5 block in `extra`")
    ap.add_argument("--c5-series", type=int, default=10_000_000, help=argparse.SUPPRESS)   # rehearsals only
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the parity checks against the one-GPU reference (exploratory runs only)")
    ap.add_argument("--transport", choices=["auto", "rccl", "copy"], default="auto",
                    help="multi-device context (--gpus N, no launcher): RCCL send / recv or peer copies")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-child-config3", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--md-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--c3-series", type=int, default=10_000_000, help=argparse.SUPPRESS)   # rehearsals only
    ap.add_argument("--md-timeout", type=float, default=480.0,
                    help="--gpus N > 1: seconds the multi-device run may take before it is retried over peer copies")
    return ap.parse_args()


def host_cpu():
    """(CPU model, last-level cache bytes summed over its distinct instances) of this host."""
    import glob
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    llc, seen, top = 0, set(), 0
    for d in glob.glob("/sys/devices/system/cpu/cpu[0-9]*/cache/index[0-9]*"):
        try:
            level = int(open(os.path.join(d, "level")).read())
            if level < top:
                continue
            shared = open(os.path.join(d, "shared_cpu_list")).read().strip()
            size = open(os.path.join(d, "size")).read().strip()
        except (OSError, ValueError):
            continue
        if level > top:
            top, llc, seen = level, 0, set()
        if shared in seen:
            continue
        seen.add(shared)
        mult = {"K": 1024, "M": 1 << 20, "G": 1 << 30}.get(size[-1:], 1)
        llc += int(size.rstrip("KMG") or 0) * mult
    return model, llc


def cpu_baseline(args, target_s: float):
    """Oracle (oracle/refcpu.c, the C port of the reference CPU path) on a bounded sample of
    the same workload on this host: single thread, and parallel over the groups with one
    thread per host core of this job's share (OMP_NUM_THREADS, 16 on the GPU box) -- the
    reported value.  The sample's cells are at least 10x the host's last-level cache (and at
    least 20k series), so the CPU streams them from DRAM as the GPU streams HBM."""
    from oracle import oracle as O
    from opentsdb_amd import synth
    model, llc = host_cpu()
    bytes_per_series = args.points * (2 + 4) + 64
    n = max(20_000, int(10 * llc / bytes_per_series) + 1)
    n = min(n, int(8e9 / bytes_per_series))   # (host memory bound: 8 GB of cells)
    t = time.perf_counter()
    b = synth.generate(n, T0, args.points, args.period_ms, value_kind=args.value_kind,
                       n_groups=min(args.groups, n), int_mod=30000 if args.value_kind == 2 else 2000, seed=0x5EED)
    gen_s = time.perf_counter() - t
    sample_bytes = int(b.qual.nbytes + b.val.nbytes)
    q = query(args)

    def timed(threads, budget):
        t = time.perf_counter()
        O.run_query(b, q, threads=threads)
        dt = time.perf_counter() - t
        reps = max(0, int(budget / max(dt, 1e-3)) - 1)
        if reps == 0:
            return 1, dt
        t = time.perf_counter()
        for _ in range(reps):
            O.run_query(b, q, threads=threads)
        return reps, time.perf_counter() - t

    threads = max(1, int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1)))
    reps1, dt1 = timed(1, target_s / 2)
    repsn, dtn = timed(threads, target_s / 2)
    dps1 = n * args.points * reps1 / dt1
    dpsn = n * args.points * repsn / dtn
    return {"value": dpsn, "unit": "datapoints/s", "cores": threads, "kind": "port",
            "single_thread_value": dps1, "cpu_model": model, "llc_bytes": llc, "sample_bytes": sample_bytes,
            "sample": f"{n} series x {args.points} dp ({sample_bytes / 1e6:.0f} MB of cells, "
                      f"{sample_bytes / max(1, llc):.1f}x the {llc / 2**20:.0f} MiB last-level cache of {model}; "
                      f"{args.ds} {args.interval}, {args.agg} over {min(args.groups, n)} groups, generated in "
                      f"{gen_s:.1f} s); oracle/refcpu.c, {threads} threads over groups: {repsn} reps in {dtn:.1f} s; "
                      f"1 thread: {reps1} reps in {dt1:.1f} s"}


def pmc_traffic(args, kernel_prefix: str, config3: bool = False):
    """HBM bytes per step of the dominant kernel (every launch of it in the step: k_fast once;
    config 3's k_short once per row class) from rocprofv3 PMC counters.

    Two separate child runs of this script (FETCH_SIZE and WRITE_SIZE cannot share a pass,
    MI355X_MICROARCH.md "rocprofv3 PMC slots"), each profiling 3 steps of the same
    workload.  FETCH_SIZE is in KiB and on gfx950 reports half the bytes of a 16-B/lane
    streaming read, so it is doubled; WRITE_SIZE is exact (same guide, "HBM").  Returns
    (bytes_per_step, detail) or (None, reason)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found"
    steps = 3
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", str(steps), "--warmup", "0",
             "--series", str(args.series), "--points", str(args.points), "--period-ms", str(args.period_ms),
             "--groups", str(args.groups), "--interval", args.interval, "--ds", args.ds, "--agg", args.agg,
             "--value-kind", str(args.value_kind)] + (["--pmc-child-config3"] if config3 else [])
    out = {}
    tmp = tempfile.mkdtemp(prefix="tsdb_pmc_")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", "120", exe, "--pmc", ctr, "--kernel-trace", "--output-format", "csv",
                   "-d", d, "-o", "run", "--"] + child
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, cwd=ROOT)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {ctr} exited {r.returncode}"
            vals = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if row["Counter_Name"] == ctr and row["Kernel_Name"].startswith(kernel_prefix):
                            vals.append(float(row["Counter_Value"]))
            if not vals:
                return None, f"no {ctr} rows for {kernel_prefix}"
            out[ctr] = sum(vals) / steps
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch = out["FETCH_SIZE"] * 1024.0 * 2.0
    write = out["WRITE_SIZE"] * 1024.0
    return fetch + write, {"fetch_bytes": fetch, "write_bytes": write, "fetch_size_kib_raw": out["FETCH_SIZE"],
                           "write_size_kib_raw": out["WRITE_SIZE"],
                           "traffic_uncorrected": out["FETCH_SIZE"] * 1024.0 + write,
                           "correction": "FETCH_SIZE x2 and KiB->B, as /opt/skills/guides/MI355X_MICROARCH.md's "
                                         "HBM / rocprofv3 section prescribes for gfx950 (FETCH_SIZE reports half "
                                         "the bytes of 16-B-per-lane streaming reads); WRITE_SIZE exact"}


def config3_block(args, device: int):
    """BASELINE config 3's one-GPU point, the north-star target (>= 50 % of HBM for 1m-avg + sum
    over 10M series): 10M series x 1 h @10 s (even series vle int [0, 30000), odd float32), 1000
    groups.  Times (a) sum:1m-avg, (b) the five aggregators avg/min/max/count/dev:1m-avg
    through one tsdbhip_run_multi (one fused streaming pass + one group reduction per query) and
    (c) p99:1m-avg (percentile group-by),
    with the same barrier-free wall clock per step as the headline, plus the streaming kernels'
    hipEvent time for the roofline."""
    from opentsdb_amd import abi
    from opentsdb_amd.engine import Engine
    eng = Engine(device)
    try:
        spec = c3_spec(args, 1)
        # k_index at load: row classes, certificate, the vle -> int16 copy.  The store is loaded
        # twice: the first load of a process also pays the first touch of ~25 GB of fresh device
        # allocations; a serving process reloads into reused buffers, as the second load does
        eng.synth(*spec)
        eng.sync()
        index_first_ms = eng.timing().index_ms
        eng.synth(*spec)
        eng.sync()
        index_ms = eng.timing().index_ms

        def q(agg):
            return abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)

        out = {"workload": "BASELINE config 3 (1 h window): 10M series x 360 dp @10 s, int/float32 alternating, "
                           "1000 groups, 1m-avg", "index_ms": index_ms,
               "index_first_load_ms": index_first_ms,
               "index_note": "load-time k_index pass (untimed in ms_per_step): row classification, the exactness "
                             "certificate and the int16 copy of the vle integer values that k_short reads; "
                             "index_ms is a reload into the process's reused buffers, index_first_load_ms the "
                             "process's first load of the store (fresh allocations)"}
        if not args.no_parity:
            out["parity"] = md_parity(eng, device, spec, parity_queries(T0, T0 + 3599, 60000),
                                      "config 3, 1 h store", bounds=[0, spec[0]])
        qs = q("sum")
        steps = max(3, args.steps)
        for _ in range(2):
            eng.run(qs)
        eng.sync()
        t = time.perf_counter()
        kms = []
        for _ in range(steps):
            eng.run(qs)
            kms.append(eng.timing().fast_ms)
        eng.sync()
        sum_ms = (time.perf_counter() - t) * 1000 / steps
        tm = eng.timing()
        k_ms = sum(kms) / len(kms)
        out["sum"] = {"ms_per_step": sum_ms, "value": tm.datapoints / (sum_ms / 1000), "unit": "datapoints/s",
                      "kernel": "k_short (both row classes)", "kernel_ms": k_ms, "bytes_per_launch": tm.bytes,
                      "hbm_frac": tm.bytes / (k_ms / 1000) / 1e9 / BYTES_PEAK_GBS,
                      "hbm_frac_step": tm.bytes / (sum_ms / 1000) / 1e9 / BYTES_PEAK_GBS,
                      "cold_value": tm.datapoints / ((index_ms + sum_ms) / 1000),
                      "cold_value_first_load": tm.datapoints / ((index_first_ms + sum_ms) / 1000),
                      "cold_note": "datapoints / (k_index at load + one step): every query on freshly scanned cells, "
                                   "the vle bytes decoded once"}
        ql = [q(a) for a in ("avg", "min", "max", "count", "dev")]
        for _ in range(2):
            eng.run_multi(ql)
        eng.sync()
        t = time.perf_counter()
        for _ in range(steps):
            eng.run_multi(ql)
        eng.sync()
        multi_ms = (time.perf_counter() - t) * 1000 / steps
        tm = eng.timing()
        out["multi_avg_min_max_count_dev"] = {
            "ms_per_step": multi_ms, "fused_queries": int(tm.fused_queries),
            "value": 5 * tm.datapoints / (multi_ms / 1000), "unit": "datapoints/s (x5 queries)",
            "fused_pass_ms": tm.decode_downsample_ms, "ratio_to_sum_step": multi_ms / sum_ms}
        # (c) p99 as the group-by aggregator (PercentileAgg over each (group, slot)'s 10000 span
        # values: the sampled-window select)
        qp = q("p99")
        w0 = eng.debug_sel_window()
        for _ in range(2):
            eng.run(qp)
        eng.sync()
        t = time.perf_counter()
        for _ in range(steps):
            eng.run(qp)
        eng.sync()
        p99_ms = (time.perf_counter() - t) * 1000 / steps
        w1 = eng.debug_sel_window()
        tm = eng.timing()
        out["p99"] = {"ms_per_step": p99_ms, "value": tm.datapoints / (p99_ms / 1000), "unit": "datapoints/s",
                      "ratio_to_sum_step": p99_ms / sum_ms, "window_runs": w1[0] - w0[0],
                      "window_fallbacks": w1[1] - w0[1]}
        return out
    finally:
        eng.close()


def config3_pmc_child(args, device: int):
    """--pmc-child-config3: the config-3 sum:1m-avg step alone, args.steps times (pmc_traffic)."""
    from opentsdb_amd import abi
    from opentsdb_amd.engine import Engine
    eng = Engine(device)
    eng.synth(10_000_000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
    eng.sync()
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    for _ in range(args.steps):
        eng.run(q)
    eng.sync()
    eng.close()


# ---- parity: the timed answer against an independent one-GPU answer ----------------------
#
# The multi-GPU exchange between DISTINCT GPUs (RCCL all-gather / all-to-all under the launcher,
# RCCL send / recv or peer copies in the one-process context) runs nowhere but on the node the
# driver benches on, so every bench run checks its own answer before the timed loop: the same
# queries through the same (sharded, exchanged) path, against the one-GPU engine over each
# checked group's series synthesized ALONE (tsdbhip_synth_shard of the group's batch positions:
# one context, no partial states, no exchange).  That engine is itself held to the oracle at
# full size (tests/test_gpu_scale.py, tests/test_gpu_fullsize.py).  A group the reference fills
# one span at a time is one SpanGroup aggregated in span order (TsdbQuery.java:916-1049).
# Bar: timestamps, is_int flags, integer values bit for bit; order statistics, min/max/count and
# TSDB_QF_ORDERED folds bit for bit; float sums / avg relative 1e-12 and dev 1e-9 (their tiles
# associate differently over a smaller store).  A mismatch makes bench.py exit 1 after its line.

PARITY_TOL = {"sum": 1e-12, "avg": 1e-12, "zimsum": 1e-12, "dev": 1e-9}
PARITY_REF = ("one-GPU engine (one context, tsdbhip_run) over each checked group's series synthesized alone: "
              "no partial states, no exchange")


def group_span(n_series: int, n_groups: int, g: int):
    """Batch positions [p0, p1) of group g in the group-major synthetic store (series i in
    group i % n_groups, synth.series_order)."""
    base, extra = divmod(n_series, n_groups)
    p0 = g * base + min(g, extra)
    return p0, p0 + base + (1 if g < extra else 0)


def group_at(n_series: int, n_groups: int, pos: int) -> int:
    base, extra = divmod(n_series, n_groups)
    if pos < extra * (base + 1):
        return pos // (base + 1)
    return extra + (pos - extra * (base + 1)) // max(1, base)


def checked_groups(n_series: int, n_groups: int, bounds, k: int = 4, cap: int = 10):
    """Every group a shard boundary cuts or touches (both sides), then k strided groups and the
    last one, at most `cap` in all."""
    edge = []
    for b in list(bounds)[1:-1]:
        for p in (b - 1, b):
            if 0 <= p < n_series:
                g = group_at(n_series, n_groups, p)
                if g not in edge:
                    edge.append(g)
    stride = [g for g in list(range(0, n_groups, max(1, n_groups // k))) + [n_groups - 1] if g not in edge]
    out = edge[:cap] + stride[:max(0, cap - len(edge[:cap]))]
    return sorted(set(out))


def parity_queries(t0: int, t1: int, ds_ms: int, head=None, ordered: bool = True):
    """[(name, aggregator, query, route)]; route: "partials" (decomposable, partial states),
    "sel" (percentile group-by / ordered fold: values to the owner), "multi" (one fused pass)."""
    from opentsdb_amd import abi

    def q(agg, **kw):
        return abi.new_query(t0, t1, agg, ds_function=abi.AGG["avg"], ds_interval_ms=ds_ms, **kw)
    out = []
    if head is not None:
        out.append(("headline", head[0], head[1], "sel" if head[0].startswith(("p", "ep", "median")) else "partials"))
    else:
        out.append(("sum", "sum", q("sum"), "partials"))
    out.append(("p99", "p99", q("p99"), "sel"))
    if ordered:
        out.append(("ordered_sum", "sum", q("sum", flags=abi.QF_ORDERED), "sel"))
    for a in ("avg", "min", "max", "count", "dev"):
        out.append(("multi." + a, a, q(a), "multi"))
    return out


def groups_map(groups, keep=None):
    """{group id: (ts, bits, is_int)} copies of a result (only the ids in `keep`)."""
    import numpy as np
    out = {}
    for g, ts, bits, isi in groups:
        if keep is None or int(g) in keep:
            out[int(g)] = (np.array(ts), np.array(bits), np.array(isi))
    return out


def compare_groups(got: dict, want: dict, agg: str, exact: bool = False):
    """Per-query parity stats of `got` against `want` over want's groups."""
    import numpy as np
    tol = 0.0 if exact or agg not in PARITY_TOL else PARITY_TOL[agg]
    st = {"groups": 0, "points": 0, "bit_exact_points": 0, "max_rel_err": 0.0, "tol": tol, "mismatch": []}
    for g, (ts2, b2, i2) in sorted(want.items()):
        st["groups"] += 1
        if g not in got:
            st["mismatch"].append(f"group {g} missing")
            continue
        ts1, b1, i1 = got[g]
        st["points"] += len(ts2)
        if len(ts1) != len(ts2) or not np.array_equal(ts1, ts2):
            st["mismatch"].append(f"group {g}: timestamps differ ({len(ts1)} vs {len(ts2)} points)")
            continue
        if not np.array_equal(i1, i2):
            st["mismatch"].append(f"group {g}: is_int flags differ")
            continue
        st["bit_exact_points"] += int(np.count_nonzero(b1 == b2))
        ints = i2.astype(bool)
        if not np.array_equal(b1[ints], b2[ints]):
            st["mismatch"].append(f"group {g}: integer values differ")
        d1, d2 = b1[~ints].view(np.float64), b2[~ints].view(np.float64)
        n1, n2 = np.isnan(d1), np.isnan(d2)
        if not np.array_equal(n1, n2):
            st["mismatch"].append(f"group {g}: NaN positions differ")
            continue
        a, b = d1[~n1], d2[~n2]
        if a.size:
            with np.errstate(invalid="ignore", divide="ignore"):
                rel = np.where(a == b, 0.0, np.abs(a - b) / np.maximum(np.abs(b), np.finfo(np.float64).tiny))
            m = float(rel.max())
            st["max_rel_err"] = max(st["max_rel_err"], m)
            if m > tol:
                st["mismatch"].append(f"group {g}: max relative error {m:.3g} > {tol:g}")
    return st


def reference_results(device: int, spec, groups, named):
    """The independent answer: for each checked group, a one-GPU context over that group's
    series alone (tsdbhip_synth_shard of its batch positions), every named query through
    tsdbhip_run.  spec = tsdbhip_synth arguments (n_series, start_s, n_points, period_ms,
    value_kind, n_groups, int_mod, seed).  Returns {name: {group: (ts, bits, is_int)}}."""
    from opentsdb_amd.engine import Engine
    out = {name: {} for name, _, _, _ in named}
    ref = Engine(device)
    try:
        for g in groups:
            p0, p1 = group_span(spec[0], spec[5], g)
            ref.synth_shard(p0, p1, *spec)
            for name, _, q, _ in named:
                out[name].update(groups_map(ref.run(q), {g}))
    finally:
        ref.close()
    return out


def run_named(named, run_one, run_many, want_ids=None):
    """The named queries through the path under test: run_one(q, route) -> groups,
    run_many(qs) -> [groups] for the "multi" ones (one fused call).  Returns {name: map} and
    {name: error string} for queries the path refused."""
    got, errs = {}, {}
    for name, _, q, route in named:
        if route == "multi":
            continue
        try:
            got[name] = groups_map(run_one(q, route), want_ids)
        except Exception as ex:   # noqa: BLE001 (an engine refusal, recorded and reported)
            errs[name] = str(ex)
    multi = [(name, q) for name, _, q, route in named if route == "multi"]
    if multi:
        try:
            res = run_many([q for _, q in multi])
            for (name, _), r in zip(multi, res):
                got[name] = groups_map(r, want_ids)
        except Exception as ex:   # noqa: BLE001
            for name, _ in multi:
                errs[name] = str(ex)
    return got, errs


def parity_stats(named, got, errs, want):
    """{name: stats} of the checked queries; refused ones carry "skipped"."""
    out = {}
    for name, agg, q, route in named:
        if name in errs:
            out[name] = {"skipped": errs[name]}
            continue
        from opentsdb_amd import abi
        exact = route == "sel" or (q.flags & abi.QF_ORDERED) != 0
        out[name] = compare_groups(got.get(name, {}), want.get(name, {}), agg, exact=exact)
    return out


def parity_block(stats: dict, groups, what: str, extra=None):
    """The line's parity block: ok unless some checked query mismatched (a query the path under
    test refused is listed, and does not count as checked)."""
    checked = {k: v for k, v in stats.items() if "skipped" not in v}
    bad = {k: v["mismatch"][:4] for k, v in checked.items() if v["mismatch"]}
    blk = {"ok": not bad and bool(checked), "checked": sorted(checked), "groups": [int(g) for g in groups],
           "what": what, "reference": PARITY_REF,
           "bit_exact_ok": all(v["bit_exact_points"] == v["points"] for k, v in checked.items() if v["tol"] == 0.0),
           "max_rel_err": max([v["max_rel_err"] for v in checked.values()] or [0.0]),
           "queries": {k: ({kk: vv for kk, vv in v.items() if kk != "mismatch"} if "skipped" not in v else v)
                       for k, v in stats.items()}}
    if bad:
        blk["mismatch"] = bad
    if extra:
        blk.update(extra)
    return blk


def merge_rank_stats(dist, dev, stats: dict):
    """Sum the ranks' per-query stats (each rank checked its share of the groups), max of the
    errors; mismatch messages stay on the rank that saw them (printed to its stderr) and are
    counted here."""
    import torch
    names = sorted(stats)
    s = torch.zeros(max(1, len(names)) * 5, dtype=torch.float64, device=dev)
    m = torch.zeros(max(1, len(names)), dtype=torch.float64, device=dev)
    for i, k in enumerate(names):
        v = stats[k]
        if "skipped" in v:
            s[5 * i + 4] = 1
            continue
        s[5 * i:5 * i + 4] = torch.tensor([v["groups"], v["points"], v["bit_exact_points"], len(v["mismatch"])],
                                          dtype=torch.float64)
        m[i] = v["max_rel_err"]
    dist.all_reduce(s)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    s, m = s.cpu().tolist(), m.cpu().tolist()
    out = {}
    for i, k in enumerate(names):
        v = stats[k]
        if s[5 * i + 4] > 0:
            out[k] = v if "skipped" in v else {"skipped": "refused on some rank"}
            continue
        out[k] = {"groups": int(s[5 * i]), "points": int(s[5 * i + 1]), "bit_exact_points": int(s[5 * i + 2]),
                  "max_rel_err": m[i], "tol": v["tol"],
                  "mismatch": v["mismatch"] + [f"{int(s[5 * i + 3]) - len(v['mismatch'])} on other ranks"]
                  if int(s[5 * i + 3]) > len(v["mismatch"]) else v["mismatch"]}
    return out


def workload_label(args) -> str:
    kind = {0: "float32", 1: "vle int", 2: "int/float32 alternating"}.get(args.value_kind, "?")
    per = "series/GPU" if args.scaling == "weak" else "series in total (strong scaling)"
    label = (f"{args.agg}:{args.interval}-{args.ds} group-by {args.groups} groups over {args.series} {per} x "
             f"{args.points} dp @{args.period_ms} ms ({kind})")
    shape = (args.series, args.points, args.period_ms, args.groups, args.interval, args.ds, args.agg, args.value_kind)
    if shape == (1_000_000, 3600, 1000, 64, "1m", "avg", "sum", 0) and args.scaling == "weak":
        label += " -- BASELINE config 2"
    elif shape[:4] == (10_000_000, 360, 10000, 1000) and args.value_kind == 2 and args.scaling == "strong":
        label += " -- BASELINE config 3 (1 h window)"
    return label


def query(args):
    from opentsdb_amd import abi, engine
    q = abi.new_query(T0, T0 + args.points * args.period_ms // 1000 - 1, args.agg)
    ds = engine.parse_downsample(f"{args.interval}-{args.ds}")
    q.ds_function, q.ds_interval_ms, q.ds_fill = ds.ds_function, ds.ds_interval_ms, ds.ds_fill
    return q


def visible_gpus() -> int:
    # the library's hipGetDeviceCount: torch.cuda.device_count() would bring up torch's own
    # HIP runtime beside the library's, which broke ncclCommInitAll in the same process
    from opentsdb_amd import engine
    try:
        return engine.device_count()
    except engine.EngineError:   # no ROCm device at all
        return 0


def md_devices(n):
    """GPUs 0..n-1; TSDBHIP_BENCH_DEVICES="0,0" (rehearsal hook) repeats devices so the
    multi-device bench path runs on a one-GPU box (peer copies between shards of one GPU)."""
    env = os.environ.get("TSDBHIP_BENCH_DEVICES")
    if env:
        devs = [int(x) for x in env.split(",") if x.strip()]
        if len(devs) != n:
            raise SystemExit(f"bench.py: TSDBHIP_BENCH_DEVICES lists {len(devs)} devices, --gpus {n}")
        return devs
    return list(range(n))


def md_engine(args, n):
    """One multi-device context over GPUs 0..n-1, series shards.  RCCL unless --transport copy;
    when the RCCL communicator cannot be built, peer copies (reported in the line)."""
    from opentsdb_amd import engine as E
    tr = {"auto": E.MD_AUTO, "rccl": E.MD_RCCL, "copy": E.MD_COPY}[args.transport]
    note = None
    try:
        eng = E.Engine(devices=md_devices(n), transport=tr)
    except E.EngineError as ex:
        if args.transport != "auto":
            raise
        note = f"RCCL init failed ({ex}); peer copies used"
        eng = E.Engine(devices=md_devices(n), transport=E.MD_COPY)
    eng.shard_mode(E.SHARD_SERIES)
    return eng, note


STAGES = ("devices_ms", "xfer_ms", "select_ms", "assemble_ms")


def md_step_stats(eng, steps_stats):
    per, ranks, moved = eng.md_stats()
    tm = eng.timing()
    st = {k: getattr(tm, k) for k in STAGES + ("total_ms",)}
    st["c_call_ms"] = getattr(eng, "last_call_ms", 0.0)
    steps_stats.append(([(t.fast_ms, t.decode_downsample_ms, t.datapoints, t.bytes) for t in per], moved, st))
    return ranks


def md_stages(stats):
    """Mean per-stage host wall times of the timed calls (tsdbhip_timing, multi-device context):
    the devices' own passes, device-to-device moves, the owners' merge / selection, the result on
    the host -- and their sum against the call's wall time."""
    out = {k: sum(s[2][k] for s in stats) / len(stats) for k in STAGES + ("total_ms", "c_call_ms")}
    out["sum_of_stages_ms"] = sum(out[k] for k in STAGES)
    return out


SEL_LIMIT = 0x7FFFFFFF   # (series, slot) values one context's percentile group-by indexes (engine.cpp sel_values)


def c3_spec(args, hours: int):
    """tsdbhip_synth arguments of BASELINE config 3's store: 10M series @10 s, int/float32
    alternating, 1000 groups."""
    return (args.c3_series, T0, hours * 360, 10000, 2, 1000, 30000, 0x5EED)


STRADDLE_SPEC = (48_000, T0, 360, 10000, 2, 61, 30000, 0x5EED ^ 0x5171)


def straddle_note(bounds):
    return (f"{STRADDLE_SPEC[0]} series x 1 h @10 s over {STRADDLE_SPEC[5]} groups, shards at batch positions "
            f"{list(bounds)}: groups straddle the shard edges, so partial states merge across GPUs and the "
            "straddling groups' span values move to their owners; every group against one GPU over the whole store")


def straddle_reference(device: int, named):
    """One context over the whole small straddle store: {name: {group: ...}} of every group."""
    from opentsdb_amd.engine import Engine
    ref = Engine(device)
    try:
        ref.synth(*STRADDLE_SPEC)
        return {name: groups_map(ref.run(q)) for name, _, q, _ in named}
    finally:
        ref.close()


def md_parity(eng, ref_device: int, spec, named, what: str, bounds=None):
    """The context's answers (tsdbhip_run / tsdbhip_run_multi; on a multi-device context over
    its shards, the exchange included) for the checked groups against the one-GPU reference."""
    if bounds is None:
        per = eng.md_info()[3]
        bounds = [0] + [int(x) for x in __import__("numpy").cumsum(per)]
    groups = checked_groups(spec[0], spec[5], bounds)
    got, errs = run_named(named, lambda q, route: eng.run(q), eng.run_multi, set(groups))
    want = reference_results(ref_device, spec, groups, named)
    return parity_block(parity_stats(named, got, errs, want), groups, what,
                        {"shard_bounds": bounds})


def md_straddle(args, n, ref_device: int):
    """The small straddle store on a fresh multi-device context (series shards), every group
    against one GPU over the whole store."""
    eng, _ = md_engine(args, n)
    try:
        eng.synth(*STRADDLE_SPEC)
        named = parity_queries(T0, T0 + 3599, 60000)
        per = eng.md_info()[3]
        bounds = [0] + [int(x) for x in __import__("numpy").cumsum(per)]
        got, errs = run_named(named, lambda q, route: eng.run(q), eng.run_multi)
        _, _, moved = eng.md_stats()
    finally:
        eng.close()
    want = straddle_reference(ref_device, named)
    return parity_block(parity_stats(named, got, errs, want), sorted(next(iter(want.values()))),
                        straddle_note(bounds), {"xfer_bytes_last_query": moved})


def md_config3(args, n):
    """BASELINE config 3 strong-scaled over the n GPUs of the context: 10M series @10 s, 1000
    groups, int/float32 alternating -- the full 1-day store (8.64e10 dp, ~437 GB of cells) from
    4 GPUs on, 12 h at 2 GPUs (what fits 288 GB per GPU with the int16 value copy).  Series
    shards, so the 1000 x 1440 partial states cross devices every query (RCCL).  Checked against
    one GPU on strided / shard-edge groups before the timed queries (`parity`)."""
    from opentsdb_amd import abi
    from opentsdb_amd import engine as E
    hours = 24 if n >= 4 else 12
    spec = c3_spec(args, hours)
    eng, note = md_engine(args, n)
    try:
        t = time.perf_counter()
        eng.synth(*spec)
        eng.sync()
        synth_s = time.perf_counter() - t

        def q(agg):
            return abi.new_query(T0, T0 + hours * 3600 - 1, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)

        out = {"workload": f"BASELINE config 3: {args.c3_series / 1e6:g}M series x {hours} h @10 s (int/float32 alternating), 1000 groups, "
                           f"1m-avg, strong-scaled over {n} GPUs (series shards, partial states over "
                           f"{'RCCL' if eng.md_info()[1] == 1 else 'peer copies'})",
               "hours": hours, "synth_s": synth_s, "transport_note": note}
        if not args.no_parity:
            out["parity"] = md_parity(eng, md_devices(n)[0], spec,
                                      parity_queries(T0, T0 + hours * 3600 - 1, 60000, ordered=False),
                                      f"config 3 strong, {hours} h store")
        steps = max(3, args.steps)
        for name, qs in (("sum", [q("sum")]), ("p99", [q("p99")]),
                         ("multi_avg_min_max_count_dev", [q(a) for a in ("avg", "min", "max", "count", "dev")])):
            try:
                for _ in range(2):
                    eng.run_multi(qs) if len(qs) > 1 else eng.run(qs[0])
            except E.EngineError as ex:   # e.g. more (series, slot) values per device than the select indexes
                out[name] = {"skipped": str(ex)}
                continue
            eng.sync()
            stats = []
            t = time.perf_counter()
            for _ in range(steps):
                eng.run_multi(qs) if len(qs) > 1 else eng.run(qs[0])
                md_step_stats(eng, stats)
            eng.sync()
            ms = (time.perf_counter() - t) * 1000 / steps
            tm = eng.timing()
            fast = [max(s[0][d][0] for s in stats) for d in range(n)]
            out[name] = {"ms_per_step": ms, "value": len(qs) * tm.datapoints / (ms / 1000),
                         "unit": "datapoints/s" + (f" (x{len(qs)} queries)" if len(qs) > 1 else ""),
                         "fused_queries": int(tm.fused_queries), "stages": md_stages(stats),
                         "exchange_ms": tm.exchange_ms, "xfer_bytes": stats[-1][1],
                         "device_kernel_ms_max": [round(x, 4) for x in fast],
                         "hbm_frac_step_per_gpu": tm.bytes / n / (ms / 1000) / 1e9 / BYTES_PEAK_GBS}
        m5, s1 = out.get("multi_avg_min_max_count_dev", {}), out.get("sum", {})
        if "ms_per_step" in m5 and "ms_per_step" in s1:
            out["multi_ratio_to_sum_step"] = m5["ms_per_step"] / s1["ms_per_step"]
        return out
    finally:
        eng.close()


# ---- BASELINE config 5 at N GPUs: percentile downsampling + rollup generation ----------------
C5_FNS = ("p99", "ep99r7")
C5_ROLLUPS = (("1h", "1d"), ("1d", "1n"))


def c5_spec(args, hours: int):
    """Config 5's store: 10M float32 series @10 s, 64 groups (the 1-GPU shard in
    tools/bench_configs.py --config 5 is 1.25M series of it)."""
    return (args.c5_series, T0, hours * 360, 10000, 0, 64, 1, 0x5EED)


def c5_queries(t1: int):
    """sum:1h-p99 and sum:1h-ep99r7 (PercentileAgg downsampling, Aggregators.java:397-431,
    657-708; the group-by a decomposable sum)."""
    from opentsdb_amd import abi
    return [(f"sum:1h-{f}", abi.new_query(T0, t1, "sum", ds_function=abi.AGG[f], ds_interval_ms=3600000)) for f in C5_FNS]


def c5_parity_named(t1: int):
    return [(name.replace(":", "_"), "sum", q, "partials") for name, q in c5_queries(t1)]


def rollup_cells_equal(a, b) -> bool:
    import numpy as np
    return all(np.array_equal(getattr(a, f), getattr(b, f)) for f in ("series", "base_time", "qualifier", "val_off", "value"))


def c5_rollup_timing(eng, hours: int, steps: int, L=None):
    """tsdbhip_rollup_run over the resident store per (interval, row span): sum, count, max, min
    cells (RollupUtils.java:52-171) left on the device(s).  Max over ranks under a launcher."""
    from opentsdb_amd import engine as E
    out = {}
    for iv, span in C5_ROLLUPS:
        riv = E.rollup_interval(iv, span)
        nc, nb = eng.rollup_run(riv, T0, T0 + hours * 3600)
        if L is not None:
            L.sync(eng)
        t = time.perf_counter()
        for _ in range(steps):
            nc, nb = eng.rollup_run(riv, T0, T0 + hours * 3600)
        if L is not None:
            L.sync(eng)
        ms = (time.perf_counter() - t) * 1000 / steps
        if L is not None:
            ms, nc, nb = L.max(ms), L.sum(int(nc)), L.sum(int(nb))
        out[f"rollup {iv} in {span} rows x sum,count,max,min"] = {"ms_per_step": ms, "cells": int(nc), "value_bytes": int(nb)}
    return out


def md_config5(args, n):
    """BASELINE config 5 over the n GPUs of one multi-device context: 10M float32 series x 1 day
    @10 s (12 h at 2 GPUs), 64 groups, series shards -- sum:1h-p99 and sum:1h-ep99r7 (parity vs
    one GPU on shard-edge / strided groups), then 1h/1d and 1d/1n rollup generation over the
    store (each device its series; parity of the cells vs one GPU on the straddle store)."""
    from opentsdb_amd import engine as E
    hours = 24 if n >= 4 else 12
    spec = c5_spec(args, hours)
    t1 = T0 + hours * 3600 - 1
    eng, note = md_engine(args, n)
    try:
        t = time.perf_counter()
        eng.synth(*spec)
        eng.sync()
        out = {"workload": f"BASELINE config 5: {spec[0] / 1e6:g}M float32 series x {hours} h @10 s, 64 groups, over {n} "
                           "GPUs (series shards)", "hours": hours, "synth_s": time.perf_counter() - t, "transport_note": note}
        if not args.no_parity:
            out["parity"] = md_parity(eng, md_devices(n)[0], spec, c5_parity_named(t1), f"config 5, {hours} h store")
        steps = max(3, args.steps)
        for name, q in c5_queries(t1):
            try:
                eng.run(q)
            except E.EngineError as ex:
                out[name] = {"skipped": str(ex)}
                continue
            eng.sync()
            t = time.perf_counter()
            for _ in range(steps):
                eng.run(q)
            eng.sync()
            ms = (time.perf_counter() - t) * 1000 / steps
            tm = eng.timing()
            out[name] = {"ms_per_step": ms, "value": tm.datapoints / (ms / 1000), "unit": "datapoints/s",
                         "devices_ms": tm.devices_ms, "exchange_ms": tm.exchange_ms}
        out.update(c5_rollup_timing(eng, hours, steps))
    finally:
        eng.close()
    if not args.no_parity:   # rollup cells, byte for byte, on the straddle store
        md, _ = md_engine(args, n)
        one = E.Engine(md_devices(n)[0])
        try:
            ok = True
            for x in (md, one):
                x.synth(*STRADDLE_SPEC)
            for iv, span in C5_ROLLUPS:
                riv = E.rollup_interval(iv, span)
                ok = ok and rollup_cells_equal(md.rollup(riv, T0, T0 + 3600), one.rollup(riv, T0, T0 + 3600))
            out["rollup_parity"] = {"ok": bool(ok), "what": "straddle store, 1h/1d and 1d/1n cells byte for byte vs one GPU"}
        finally:
            md.close()
            one.close()
    return out


def launch_config5(args, L):
    """BASELINE config 5 over the launch's ranks (one process per GPU): rank r synthesizes its
    contiguous shard of the 10M-series store; sum:1h-p99 / ep99r7 through the partial-state
    all-gather; rollup generation per rank over its own series (no exchange)."""
    from opentsdb_amd.dist import synth_bounds
    from opentsdb_amd.engine import Engine, EngineError
    hours = 24 if L.world >= 4 else 12
    spec = c5_spec(args, hours)
    bounds = synth_bounds(spec[0], L.world)
    t1 = T0 + hours * 3600 - 1
    eng = Engine(L.device)
    try:
        t = time.perf_counter()
        eng.synth_shard(bounds[L.rank], bounds[L.rank + 1], *spec)
        eng.sync()
        out = {"workload": f"BASELINE config 5: {spec[0] / 1e6:g}M float32 series x {hours} h @10 s, 64 groups, over "
                           f"{L.world} ranks (one process per GPU, series shards)", "hours": hours,
               "synth_s": L.max(time.perf_counter() - t)}
        if not args.no_parity:
            out["parity"] = launch_parity(L, eng, spec, bounds, c5_parity_named(t1), f"config 5, {hours} h store")
        one, _ = L.runner(eng, spec[5])
        steps = max(3, args.steps)
        for name, q in c5_queries(t1):
            try:
                one(q, "partials")
            except EngineError as ex:
                out[name] = {"skipped": str(ex)}
                continue
            L.sync(eng)
            t = time.perf_counter()
            for _ in range(steps):
                one(q, "partials")
            L.sync(eng)
            ms = L.max((time.perf_counter() - t) * 1000 / steps)
            dps = L.sum(int(eng.timing().datapoints))
            out[name] = {"ms_per_step": ms, "value": dps / (ms / 1000), "unit": "datapoints/s"}
        out.update(c5_rollup_timing(eng, hours, steps, L))
        return out
    finally:
        eng.close()


def run_child(cmd, timeout):
    """One bench child: (returncode or None on a time-out, its last JSON line or None, stderr tail).
    Its stderr is passed through."""
    import subprocess
    try:
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout, cwd=ROOT)
    except subprocess.TimeoutExpired as ex:
        err = (ex.stderr or b"").decode(errors="replace")
        sys.stderr.write(err)
        return None, None, f"timed out after {timeout:.0f} s; " + err[-600:]
    err = r.stderr.decode(errors="replace")
    sys.stderr.write(err)
    lines = [ln for ln in r.stdout.decode(errors="replace").splitlines() if ln.startswith("{")]
    return r.returncode, (lines[-1] if lines else None), err[-600:]


def md_supervise(args, child=None):
    """--gpus N > 1: the multi-device run in a child process (this one touches no GPU), under a
    time limit.  RCCL between distinct GPUs is first exercised on the node the driver runs this on.
    Outcomes:
      * the child prints its line and exits 0 -> that line;
      * it exits 1 WITH a line -> its parity check failed: the line (parity.ok false), exit 1 --
        a wrong answer is never retried over another transport;
      * it refuses the GPU count (exit 2), or the transport was forced -> exit with its status;
      * it fails or hangs over RCCL (transport auto) -> ONE fresh child over peer copies (never a
        re-exec); that line is printed with `rccl_failed: true` and the RCCL error at top level
        (its own parity block checks the peer-copy answers)."""
    argv = [a for a in sys.argv[1:]]
    if child is None:
        def child(extra):
            return run_child([sys.executable, os.path.abspath(__file__)] + argv + ["--md-child"] + extra,
                             args.md_timeout)
    rc, line, err = child([])
    if rc == 0 and line:
        print(line, flush=True)
        return 0
    if rc == 1 and line:
        print(line, flush=True)
        print("bench.py: the multi-device answer does not match the one-GPU reference (parity block)",
              file=sys.stderr, flush=True)
        return 1
    if rc == 2 or args.transport != "auto":
        print(f"bench.py: multi-device run failed (exit {rc}): {err}", file=sys.stderr, flush=True)
        return rc if rc else 1
    first = f"exit {rc}" if rc is not None else "time-out"
    rc2, line2, err2 = child(["--transport", "copy"])
    if rc2 not in (0, 1) or not line2:
        print(f"bench.py: multi-device run failed over RCCL ({first}: {err}) and over peer copies "
              f"(exit {rc2}: {err2})", file=sys.stderr, flush=True)
        return rc2 if rc2 else 1
    d = json.loads(line2)
    d["rccl_failed"] = True
    d["rccl_error"] = f"{first}: {err[-400:]}"
    d["transport_note"] = "the RCCL child failed (rccl_error); this line is the fresh peer-copy child's"
    print(json.dumps(d), flush=True)
    return rc2


def main_md(args):
    """--gpus N > 1 without a launcher: one process, one multi-device context over N GPUs."""
    n = args.gpus
    have = visible_gpus()
    if have <= max(md_devices(n)):
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible; refusing to report a {have}-GPU number "
              f"as {n}", file=sys.stderr, flush=True)
        sys.exit(2)
    eng, note = md_engine(args, n)
    n_dev, transport, _, _ = eng.md_info()
    total_series = args.series * n if args.scaling == "weak" else args.series
    int_mod = 30000 if args.value_kind == 2 else 2000
    spec = (total_series, T0, args.points, args.period_ms, args.value_kind, args.groups, int_mod, 0x5EED)
    t_gen = time.perf_counter()
    eng.synth(*spec)
    eng.sync()
    t_gen = time.perf_counter() - t_gen
    _, _, mode, per_series = eng.md_info()
    index_ms = eng.timing().index_ms
    q = query(args)
    parity = None
    if not args.no_parity:
        t1 = T0 + args.points * args.period_ms // 1000 - 1
        parity = md_parity(eng, md_devices(n)[0], spec,
                           parity_queries(T0, t1, q.ds_interval_ms, head=(args.agg, q)), "headline store")
    for _ in range(args.warmup):
        eng.run(q)
    eng.sync()
    stats = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run(q)
        ranks = md_step_stats(eng, stats)
    eng.sync()
    elapsed = time.perf_counter() - t0
    tm = eng.timing()
    ms_per_step = elapsed * 1000.0 / args.steps
    value = tm.datapoints / (ms_per_step / 1000.0)
    # per device: its k_fast hipEvent time, its algorithmic bytes
    dev_ms = [sum(s[0][d][0] for s in stats) / len(stats) for d in range(n)]
    dev_bytes = [stats[-1][0][d][3] for d in range(n)]
    dev_gbs = [b / (ms / 1000.0) / 1e9 if ms > 0 else 0.0 for b, ms in zip(dev_bytes, dev_ms)]
    achieved = sum(dev_gbs) / n
    eng.close()
    if parity is not None:
        parity["straddle"] = md_straddle(args, n, md_devices(n)[0])
    extra = None if args.no_config3 else {"config3_strong": md_config3(args, n)}
    if not args.no_config5:
        extra = dict(extra or {}, config5=md_config5(args, n))
    ok = parity_all_ok(parity, extra)
    line = {
        "metric": "raw datapoints/sec through downsample+group-by; % of HBM BW, 1-8 GPUs",
        "value": value,
        "unit": "datapoints/s",
        "n_gpus": n_dev,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded splitmix64, generated in HBM with the MockBase cell encoding)",
        "index_ms": index_ms,
        "launch": "one process, one multi-device context (tsdbhip_init_devices) over GPUs 0..N-1",
        "devices": md_devices(n),
        "transport": {0: "peer copies", 1: "RCCL send/recv"}.get(transport, str(transport)),
        "transport_note": note,
        "rccl_failed": False,
        "rccl_ranks": ranks,
        "parity_ok": ok,
        "parity": parity,
        "exchange_ms": tm.exchange_ms,
        "stages": md_stages(stats),
        "xfer_bytes_per_step": stats[-1][1],
        "config": {
            "workload": workload_label(args),
            "series_per_gpu": [int(x) for x in per_series],
            "datapoints_per_gpu": [int(stats[-1][0][d][2]) for d in range(n)],
            "groups": args.groups,
            "parallelism": f"series-sharded x{n} ({'series' if mode == 0 else 'groups'} shards)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": BYTES_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / BYTES_PEAK_GBS,
            "frac_note": "per GPU (mean over the devices): each device's algorithmic bytes / its k_fast hipEvent "
                         "time; frac_step: all bytes / (N x step time)",
            "frac_step": tm.bytes / n / (ms_per_step / 1000.0) / 1e9 / BYTES_PEAK_GBS,
            "per_gpu_frac": [g / BYTES_PEAK_GBS for g in dev_gbs],
            "traffic": None,
            "traffic_detail": "PMC passes are collected at N=1 only",
            "kernel": "k_fast (streaming decode+downsample+tile group partials), per device",
            "kernel_ms": dev_ms,
            "bytes_per_launch": dev_bytes,
        },
        "cpu_baseline": None,
        "synth_s": t_gen,
        "extra": extra,
    }
    print(json.dumps(line), flush=True)
    if not ok:
        sys.exit(1)


def parity_all_ok(parity, extra) -> bool:
    """Every parity block of the line (headline, straddle, config 3) is ok."""
    blocks = []
    if parity is not None:
        blocks.append(parity)
        if parity.get("straddle") is not None:
            blocks.append(parity["straddle"])
    for v in (extra or {}).values():
        if isinstance(v, dict) and v.get("parity") is not None:
            blocks.append(v["parity"])
        if isinstance(v, dict) and v.get("rollup_parity") is not None:
            blocks.append(v["rollup_parity"])
    return all(b.get("ok") for b in blocks)


# ---- one process per GPU (torch.distributed.run) ------------------------------------------
class Launch:
    """This rank under torch.distributed.run: RANK / WORLD_SIZE / LOCAL_RANK from the env; the
    backend is RCCL ("nccl").  Rehearsal hooks for a one-GPU box: TSDBHIP_BENCH_DIST=gloo (host
    tensors; several ranks may share a GPU), TSDBHIP_BENCH_DEVICES="0,0" (GPU per local rank),
    TSDBHIP_BENCH_FORCE_DIST=1 (the distributed path at WORLD_SIZE 1: a one-rank RCCL
    communicator)."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        devs = os.environ.get("TSDBHIP_BENCH_DEVICES")
        self.device = int(devs.split(",")[self.local_rank]) if devs else self.local_rank
        self.backend = os.environ.get("TSDBHIP_BENCH_DIST", "nccl")
        self.dist = None
        self.tdev = "cpu"

    def init(self):
        if self.world > 1 or os.environ.get("TSDBHIP_BENCH_FORCE_DIST") == "1":
            import torch
            import torch.distributed as td
            if self.backend == "nccl":
                torch.cuda.set_device(self.device)
                self.tdev = f"cuda:{self.device}"
            td.init_process_group(self.backend)
            self.dist = td
        return self

    def sync(self, eng=None):
        if eng is not None:
            eng.sync()
        if self.dist is not None:
            import torch
            if self.backend == "nccl":
                torch.cuda.synchronize(self.device)
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=self.tdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: int) -> int:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.int64, device=self.tdev)
        self.dist.all_reduce(t)
        return int(t.item())

    def runner(self, eng, n_groups: int):
        """(run_one(q, route), run_many(qs)) through this launch's path: the one-GPU calls without
        a process group; the exchange of opentsdb_amd.dist with one."""
        from opentsdb_amd import dist as D
        if self.dist is None:
            return (lambda q, route: eng.run(q)), eng.run_multi
        gdev = self.tdev if self.backend == "nccl" else None

        def one(q, route):
            if route == "sel":
                return D.run_distributed_sel(eng, q, self.dist, n_groups, device=gdev)
            return D.run_distributed(eng, q, self.dist, n_groups, device=gdev)
        return one, (lambda qs: D.run_distributed_multi(eng, qs, self.dist, n_groups, device=gdev))


def sel_fits(bounds, n_slots: int) -> bool:
    """Every shard's percentile group-by fits one context's select index (the same answer on
    every rank, so no rank enters a collective the others skip)."""
    return max(b1 - b0 for b0, b1 in zip(bounds[:-1], bounds[1:])) * n_slots <= SEL_LIMIT


def launch_parity(L: Launch, eng, spec, bounds, named, what: str):
    """The launch's answers for the checked groups (every rank runs every query: collectives),
    each rank checking its share of the groups against the one-GPU reference on its own GPU."""
    groups = checked_groups(spec[0], spec[5], bounds)
    one, many = L.runner(eng, spec[5])
    got, errs = run_named(named, one, many, set(groups))
    mine = groups[L.rank::L.world]
    want = reference_results(L.device, spec, mine, named)
    stats = parity_stats(named, got, errs, want)
    for k, v in stats.items():
        for m in v.get("mismatch", []):
            print(f"bench.py rank {L.rank}: parity {what} {k}: {m}", file=sys.stderr, flush=True)
    if L.dist is not None:
        stats = merge_rank_stats(L.dist, L.tdev, stats)
    return parity_block(stats, groups, what, {"shard_bounds": [int(b) for b in bounds]})


def launch_straddle(L: Launch):
    """The small straddle store split over the ranks; every rank checks every group against
    one GPU over the whole store."""
    from opentsdb_amd.dist import synth_bounds
    from opentsdb_amd.engine import Engine
    bounds = synth_bounds(STRADDLE_SPEC[0], L.world)
    named = parity_queries(T0, T0 + 3599, 60000)
    eng = Engine(L.device)
    try:
        eng.synth_shard(bounds[L.rank], bounds[L.rank + 1], *STRADDLE_SPEC)
        one, many = L.runner(eng, STRADDLE_SPEC[5])
        got, errs = run_named(named, one, many)
    finally:
        eng.close()
    want = straddle_reference(L.device, named)
    stats = parity_stats(named, got, errs, want)
    bad = sum(len(v.get("mismatch", [])) for v in stats.values())
    if L.dist is not None:   # every rank compared the same groups: agree on the verdict
        import torch
        t = torch.tensor([bad], dtype=torch.int64, device=L.tdev)
        L.dist.all_reduce(t)
        if int(t.item()) and not bad:
            stats["_other_ranks"] = {"groups": 0, "points": 0, "bit_exact_points": 0, "max_rel_err": 0.0,
                                     "tol": 0.0, "mismatch": [f"{int(t.item())} mismatches on other ranks"]}
    return parity_block(stats, sorted(next(iter(want.values()))), straddle_note(bounds))


def launch_config3(args, L: Launch):
    """BASELINE config 3 strong-scaled over the launch's ranks (one process per GPU): the global
    10M-series store, rank r synthesizing its contiguous shard (tsdbhip_synth_shard) -- the full
    day from 4 GPUs on, 12 h at 2 -- sum through the partial-state all-gather, p99 through the
    owner exchange, avg/min/max/count/dev through one fused pass and one all-gather.  Checked
    against one GPU on strided / shard-edge groups first."""
    from opentsdb_amd import abi
    from opentsdb_amd.dist import synth_bounds
    from opentsdb_amd.engine import Engine, EngineError
    hours = 24 if L.world >= 4 else 12
    spec = c3_spec(args, hours)
    bounds = synth_bounds(spec[0], L.world)
    t1 = T0 + hours * 3600 - 1
    K = hours * 60
    eng = Engine(L.device)
    try:
        t = time.perf_counter()
        eng.synth_shard(bounds[L.rank], bounds[L.rank + 1], *spec)
        eng.sync()
        synth_s = L.max(time.perf_counter() - t)
        index_ms = L.max(eng.timing().index_ms)
        fits = sel_fits(bounds, K)
        out = {"workload": f"BASELINE config 3: {spec[0] / 1e6:g}M series x {hours} h @10 s (int/float32 alternating), "
                           f"1000 groups, 1m-avg, strong-scaled over {L.world} ranks (one process per GPU, series shards, "
                           f"{'RCCL' if L.backend == 'nccl' else L.backend} collectives)",
               "hours": hours, "synth_s": synth_s, "index_ms_max": index_ms}
        named = parity_queries(T0, t1, 60000, ordered=False)
        if not fits:
            named = [x for x in named if x[3] != "sel"]
        if not args.no_parity:
            out["parity"] = launch_parity(L, eng, spec, bounds, named, f"config 3 strong, {hours} h store")
            if not fits:
                out["parity"]["queries"]["p99"] = {"skipped": "more (series, slot) values per rank than the select indexes"}

        def q(agg):
            return abi.new_query(T0, t1, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        one, many = L.runner(eng, 1000)
        steps = max(3, args.steps)
        plan = [("sum", [q("sum")], "partials"), ("p99", [q("p99")], "sel"),
                ("multi_avg_min_max_count_dev", [q(a) for a in ("avg", "min", "max", "count", "dev")], "multi")]
        for name, qs, route in plan:
            if route == "sel" and not fits:
                out[name] = {"skipped": f"{max(b1 - b0 for b0, b1 in zip(bounds[:-1], bounds[1:]))} series x {K} "
                                        "slots per rank exceed the select index (2^31)"}
                continue

            def step():
                return many(qs) if route == "multi" else one(qs[0], route)
            try:
                for _ in range(2):
                    step()
            except EngineError as ex:
                out[name] = {"skipped": str(ex)}
                continue
            L.sync(eng)
            kms = []
            t = time.perf_counter()
            for _ in range(steps):
                step()
                kms.append(eng.timing().decode_downsample_ms)
            L.sync(eng)
            ms = L.max((time.perf_counter() - t) * 1000 / steps)
            tm = eng.timing()
            dps = L.sum(int(tm.datapoints))
            byts = L.sum(int(tm.bytes))
            out[name] = {"ms_per_step": ms, "value": len(qs) * dps / (ms / 1000),
                         "unit": "datapoints/s" + (f" (x{len(qs)} queries)" if len(qs) > 1 else ""),
                         "device_pass_ms_max": L.max(sum(kms) / len(kms)),
                         "hbm_frac_step_per_gpu": byts / L.world / (ms / 1000) / 1e9 / BYTES_PEAK_GBS}
        m5, s1 = out.get("multi_avg_min_max_count_dev", {}), out.get("sum", {})
        if "ms_per_step" in m5 and "ms_per_step" in s1:
            out["multi_ratio_to_sum_step"] = m5["ms_per_step"] / s1["ms_per_step"]
        return out
    finally:
        eng.close()


def main():
    args = parse()
    L = Launch()
    if L.world > 1 and args.gpus not in (1, L.world):
        print(f"bench.py: --gpus {args.gpus} under a launcher with WORLD_SIZE={L.world}", file=sys.stderr, flush=True)
        sys.exit(2)
    if L.world == 1 and args.gpus > 1 and not args.pmc_child:
        if args.md_child:
            return main_md(args)
        sys.exit(md_supervise(args))
    if args.pmc_child_config3:
        return config3_pmc_child(args, L.device)
    L.init()
    rank, world = L.rank, L.world
    from opentsdb_amd.engine import Engine
    from opentsdb_amd.dist import synth_bounds

    eng = Engine(L.device)
    # a tiny store first: loads the index kernels' code objects, so index_ms is the load of
    # the real store alone
    eng.synth(256, T0, args.points, args.period_ms, args.value_kind, min(args.groups, 256), 30000, 1)
    int_mod = 30000 if args.value_kind == 2 else 2000
    # one global store (series i in group i % G, batch group-major): weak scaling gives every rank
    # --series of it, strong scaling splits --series over the ranks; rank r synthesizes its
    # contiguous shard of batch positions (tsdbhip_synth_shard), the same bytes a one-GPU store has
    total = args.series * world if args.scaling == "weak" else args.series
    spec = (total, T0, args.points, args.period_ms, args.value_kind, args.groups, int_mod, 0x5EED)
    bounds = synth_bounds(total, world)
    t_gen = time.perf_counter()
    if world == 1:
        eng.synth(*spec)
    else:
        eng.synth_shard(bounds[rank], bounds[rank + 1], *spec)
    eng.sync()
    t_gen = time.perf_counter() - t_gen
    index_ms = eng.timing().index_ms   # k_index at load (row classification / validation)
    q = query(args)
    one, _ = L.runner(eng, args.groups)

    def step():
        return one(q, "sel" if args.agg.startswith(("p", "ep", "median")) else "partials")

    if args.pmc_child:
        for _ in range(args.steps):
            step()
        eng.sync()
        eng.close()
        return
    parity = None
    if not args.no_parity:
        named = parity_queries(T0, T0 + args.points * args.period_ms // 1000 - 1, q.ds_interval_ms, head=(args.agg, q))
        if not sel_fits(bounds, max(1, args.points * args.period_ms // max(1, q.ds_interval_ms))):
            named = [x for x in named if x[3] != "sel"]
        parity = launch_parity(L, eng, spec, bounds, named, "headline store")
    for _ in range(args.warmup):
        step()
    L.sync(eng)
    kernel_ms = []
    fast_ms = []
    reduce_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        tm = eng.timing()
        kernel_ms.append(tm.decode_downsample_ms)
        fast_ms.append(tm.fast_ms)
        reduce_ms.append(tm.group_reduce_ms)
    L.sync(eng)
    elapsed = L.max(time.perf_counter() - t0)
    tm = eng.timing()
    ms_per_step = elapsed * 1000.0 / args.steps
    dps_step = L.sum(int(tm.datapoints))   # datapoints of every rank's shard
    value = dps_step / (ms_per_step / 1000.0)
    # dominant kernel: the streaming kernel k_fast when the batch's row class allows it
    # (every tile handed back to k_grid otherwise); hipEvents on the engine stream
    use_fast = min(fast_ms) > 0 and tm.redo_tiles == 0
    # a reference query arrives with freshly scanned Spans (TsdbQuery.java:916-1049): "cold"
    # = the load-time row index + one step, per query
    cold_value = dps_step / ((L.max(index_ms) + ms_per_step) / 1000.0)
    k_avg = sum(fast_ms if use_fast else kernel_ms) / args.steps
    kname = "k_fast" if use_fast else "k_grid"
    achieved = tm.bytes / (k_avg / 1000.0) / 1e9
    eng.close()   # free the headline store before config 3
    if parity is not None and L.dist is not None:
        parity["straddle"] = launch_straddle(L)
    extra = None
    if not args.no_config3:
        extra = {"config3": config3_block(args, L.device)} if L.dist is None else {"config3_strong": launch_config3(args, L)}
    if L.dist is not None and not args.no_config5:
        extra = dict(extra or {}, config5=launch_config5(args, L))
    ok = parity_all_ok(parity, extra)
    if rank == 0:
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(args, args.cpu_seconds)
        traffic, traffic_note = (None, "not collected (--no-pmc or N>1)")
        if not args.no_pmc and world == 1:
            traffic, traffic_note = pmc_traffic(args, f"void tsdb::{kname}")
            if extra is not None and "config3" in extra:   # config 3: both k_short row classes of a step
                c3t, c3note = pmc_traffic(args, "void tsdb::k_short", config3=True)
                extra["config3"]["sum"]["traffic"] = c3t
                extra["config3"]["sum"]["traffic_detail"] = c3note
        line = {
            "metric": "raw datapoints/sec through downsample+group-by; % of HBM BW, 1-8 GPUs",
            "value": value,
            "unit": "datapoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded splitmix64, generated in HBM with the MockBase cell encoding)",
            "index_ms": index_ms,
            "cold_value": cold_value,
            "cold_note": "datapoints / (k_index at load + one step): the per-query rate when every query "
                         "brings freshly scanned cells",
            "launch": ("one process per GPU (torch.distributed.run), partial states all-gathered over "
                       f"{'RCCL' if L.backend == 'nccl' else L.backend}") if L.dist is not None else "one process, one GPU",
            "parity_ok": ok,
            "parity": parity,
            "config": {
                "workload": workload_label(args),
                "series_per_gpu": args.series if args.scaling == "weak" else args.series / world,
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
                "frac_note": "kernel-only: algorithmic bytes / the dominant kernel's hipEvent time; frac_step is "
                             "the same bytes over the whole step (decode + group-by + results to the host)",
                "frac_step": tm.bytes / (ms_per_step / 1000.0) / 1e9 / BYTES_PEAK_GBS,
                "traffic": traffic,
                "traffic_detail": traffic_note,
                "kernel": kname + (" (streaming decode+downsample+tile group partials)" if use_fast
                                   else " (fused decode+downsample+tile group partials)"),
                "kernel_ms": k_avg,
                "bytes_per_launch": tm.bytes,
                "bytes_per_dp": tm.bytes / max(1, tm.datapoints),
                "group_reduce_ms": sum(reduce_ms) / len(reduce_ms),
            },
            "cpu_baseline": cpu,
            "synth_s": t_gen,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if L.dist is not None:
        L.dist.destroy_process_group()
    if not ok:
        print(f"bench.py rank {rank}: parity check FAILED (see the line's parity blocks)", file=sys.stderr, flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
