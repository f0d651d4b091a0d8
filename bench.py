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
        eng.synth(10_000_000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
        eng.sync()
        index_ms = eng.timing().index_ms   # k_index at load: row classes, certificate, the vle -> int16 copy

        def q(agg):
            return abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)

        out = {"workload": "BASELINE config 3 (1 h window): 10M series x 360 dp @10 s, int/float32 alternating, "
                           "1000 groups, 1m-avg", "index_ms": index_ms,
               "index_note": "load-time k_index pass (untimed in ms_per_step): row classification, the exactness "
                             "certificate and the int16 copy of the vle integer values that k_short reads"}
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


def md_config3(args, n):
    """BASELINE config 3 strong-scaled over the n GPUs of the context: 10M series @10 s, 1000
    groups, int/float32 alternating -- the full 1-day store (8.64e10 dp, ~437 GB of cells) from
    4 GPUs on, 12 h at 2 GPUs (what fits 288 GB per GPU with the int16 value copy).  Series
    shards, so the 1000 x 1440 partial states cross devices every query (RCCL)."""
    from opentsdb_amd import abi
    from opentsdb_amd import engine as E
    hours = 24 if n >= 4 else 12
    eng, note = md_engine(args, n)
    try:
        t = time.perf_counter()
        eng.synth(args.c3_series, T0, hours * 360, 10000, 2, 1000, 30000, 0x5EED)
        eng.sync()
        synth_s = time.perf_counter() - t

        def q(agg):
            return abi.new_query(T0, T0 + hours * 3600 - 1, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)

        out = {"workload": f"BASELINE config 3: {args.c3_series / 1e6:g}M series x {hours} h @10 s (int/float32 alternating), 1000 groups, "
                           f"1m-avg, strong-scaled over {n} GPUs (series shards, partial states over "
                           f"{'RCCL' if eng.md_info()[1] == 1 else 'peer copies'})",
               "hours": hours, "synth_s": synth_s, "transport_note": note}
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


def md_supervise(args):
    """--gpus N > 1: the multi-device run in a child process (this one touches no GPU), under a time
    limit.  RCCL between distinct GPUs is first exercised on the node the driver runs this on; if
    the child fails or hangs over RCCL (transport auto), it is run once more over peer copies and the
    line says so.  A child that refuses the GPU count (exit 2) is final."""
    import subprocess
    argv = [a for a in sys.argv[1:]]

    def child(extra):
        cmd = [sys.executable, os.path.abspath(__file__)] + argv + ["--md-child"] + extra
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, timeout=args.md_timeout, cwd=ROOT)
        except subprocess.TimeoutExpired:
            return None, f"timed out after {args.md_timeout:.0f} s"
        lines = [ln for ln in r.stdout.decode(errors="replace").splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return r.returncode, f"exited {r.returncode}"
        return 0, lines[-1]

    rc, out = child([])
    if rc == 0:
        print(out, flush=True)
        return
    if rc == 2 or args.transport != "auto":
        print(f"bench.py: multi-device run failed ({out})", file=sys.stderr, flush=True)
        sys.exit(rc if rc else 1)
    first = out
    rc, out = child(["--transport", "copy"])
    if rc != 0:
        print(f"bench.py: multi-device run failed over RCCL ({first}) and over peer copies ({out})",
              file=sys.stderr, flush=True)
        sys.exit(rc if rc else 1)
    line = json.loads(out)
    line["transport_note"] = f"the RCCL run {first}; this line is the peer-copy rerun"
    print(json.dumps(line), flush=True)


def main_md(args):
    """--gpus N > 1 without a launcher: one process, one multi-device context over N GPUs."""
    from opentsdb_amd import abi
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
    t_gen = time.perf_counter()
    eng.synth(total_series, T0, args.points, args.period_ms, args.value_kind, args.groups, int_mod, 0x5EED)
    eng.sync()
    t_gen = time.perf_counter() - t_gen
    _, _, mode, per_series = eng.md_info()
    index_ms = eng.timing().index_ms
    q = query(args)
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
    extra = None if args.no_config3 else {"config3_strong": md_config3(args, n)}
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
        "rccl_ranks": ranks,
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


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus not in (1, world):
        print(f"bench.py: --gpus {args.gpus} under a launcher with WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(2)
    if world == 1 and args.gpus > 1 and not args.pmc_child:
        return main_md(args) if args.md_child else md_supervise(args)
    if args.pmc_child_config3:
        return config3_pmc_child(args, local_rank)
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
    # a tiny store first: loads the index kernels' code objects, so index_ms is the load of
    # the real store alone
    eng.synth(256, T0, args.points, args.period_ms, args.value_kind, min(args.groups, 256), 30000, 1)
    t_gen = time.perf_counter()
    int_mod = 30000 if args.value_kind == 2 else 2000
    if args.scaling == "strong":
        from opentsdb_amd.dist import synth_bounds
        b = synth_bounds(args.series, world)
        eng.synth_shard(b[rank], b[rank + 1], args.series, T0, args.points, args.period_ms, args.value_kind,
                        args.groups, int_mod, 0x5EED)
    else:
        eng.synth(args.series, T0, args.points, args.period_ms, args.value_kind, args.groups, int_mod,
                  0x5EED ^ (rank * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF))
    eng.sync()
    t_gen = time.perf_counter() - t_gen
    index_ms = eng.timing().index_ms   # k_index at load (row classification / validation)
    q = query(args)

    def step():
        if dist is None:
            return eng.run(q)
        from opentsdb_amd.dist import run_distributed
        return run_distributed(eng, q, dist, args.groups, device=f"cuda:{local_rank}")

    if args.pmc_child:
        for _ in range(args.steps):
            step()
        eng.sync()
        eng.close()
        return
    for _ in range(args.warmup):
        step()
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    eng.sync()
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
    if dist is not None:   # datapoints of every rank's shard
        import torch
        t = torch.tensor([tm.datapoints], dtype=torch.int64, device=f"cuda:{local_rank}")
        dist.all_reduce(t)
        dps_step = int(t.item())
    else:
        dps_step = tm.datapoints
    value = dps_step / (ms_per_step / 1000.0)
    # dominant kernel: the streaming kernel k_fast when the batch's row class allows it
    # (every tile handed back to k_grid otherwise); hipEvents on the engine stream
    use_fast = min(fast_ms) > 0 and tm.redo_tiles == 0
    # a reference query arrives with freshly scanned Spans (TsdbQuery.java:916-1049): "cold"
    # = the load-time row index + one step, per query
    cold_value = dps_step / ((index_ms + ms_per_step) / 1000.0)
    k_avg = sum(fast_ms if use_fast else kernel_ms) / args.steps
    kname = "k_fast" if use_fast else "k_grid"
    achieved = tm.bytes / (k_avg / 1000.0) / 1e9
    extra = None
    if world == 1 and not args.no_config3:
        eng.close()   # free the headline store before config 3's 18 GB
        extra = {"config3": config3_block(args, local_rank)}
    if rank == 0:
        cpu = None if args.no_cpu_baseline or world > 1 else cpu_baseline(args, args.cpu_seconds)
        traffic, traffic_note = (None, "not collected (--no-pmc or N>1)")
        if not args.no_pmc and world == 1:
            traffic, traffic_note = pmc_traffic(args, f"void tsdb::{kname}")
            if extra is not None:   # config 3: both k_short row classes of a step
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
    if dist is not None:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
