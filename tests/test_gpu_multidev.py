"""One process, several GPUs: the multi-device context (tsdbhip_init_devices, multi.cpp).

The same ctypes Engine drives N devices; every query must return what one GPU returns for the
same batch -- bit for bit where the shards hold whole SpanGroups (TSDB_SHARD_GROUPS), and for
series-sharded stores (TSDB_SHARD_SERIES, partial states gathered to devices[0] and merged in
device order) bit for bit for order statistics / ordered folds / NONE, and within the oracle's
tolerance for the float reductions whose association changes at the shard boundaries.

The development GPU box has one MI355X: N devices are emulated by repeating device 0 (the
device-copy transport), and a one-rank RCCL communicator (ncclCommInitAll over [0]) exercises the
RCCL code path without a peer.  `test_distinct_devices` runs every query kind over 2..N distinct
GPUs with both transports when the machine has them (it skips on a one-GPU box); bench.py's
`--gpus N` drives the same context over N distinct GPUs."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd import engine as E
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400


def q_ds(agg, ds="avg", **kw):
    kw.setdefault("ds_interval_ms", 60000)
    return abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG[ds], **kw)


# (name, query, kind): kind "partials" = decomposable group-by, "sel" = order statistic or
# ordered fold, "none" = per-span, "raw" = raw group-by
QUERIES = [
    ("sum", q_ds("sum"), "partials"),
    ("avg", q_ds("avg", "max"), "partials"),
    ("min", q_ds("min", "sum"), "partials"),
    ("max", q_ds("max", "min"), "partials"),
    ("count", q_ds("count"), "partials"),
    ("dev", q_ds("dev"), "partials"),
    ("first", q_ds("first"), "partials"),
    ("last", q_ds("last"), "partials"),
    ("diff", q_ds("diff"), "partials"),
    ("zimsum", q_ds("zimsum"), "partials"),
    ("mimmax", q_ds("mimmax"), "partials"),
    ("sum-fill-nan", q_ds("sum", "sum", ds_fill=abi.FILL_NAN), "partials"),
    ("avg-rate", q_ds("avg", "avg", rate=True), "partials"),
    ("sum-all", abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["sum"], ds_all=True), "partials"),
    ("sum-p95ds", q_ds("sum", "p95"), "partials"),
    ("p99", q_ds("p99"), "sel"),
    ("median", q_ds("median", "sum"), "sel"),
    ("ordered-sum", q_ds("sum", flags=abi.QF_ORDERED), "sel"),
    ("none", q_ds("none"), "none"),
    ("raw-none", abi.new_query(T0, T0 + 3599, "none"), "none"),
    ("raw-sum", abi.new_query(T0, T0 + 3599, "sum"), "raw"),
    ("raw-p90", abi.new_query(T0, T0 + 3599, "p90"), "raw"),
]
IDS = [n for n, _, _ in QUERIES]


@pytest.fixture(scope="module")
def batch():
    """150 series over 7 groups in interleaved batch order, every 9th series without a group
    (a group-by tag missing: only the NONE aggregator sees it)."""
    b = synth.generate(150, T0, 360, 10000, value_kind=2, n_groups=7, int_mod=30000, seed=0x5EED)
    gid = b.group_id.copy()
    gid[::9] = -1
    return abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, b.val, gid)


@pytest.fixture(scope="module")
def single(batch):
    e = E.Engine(0)
    e.load(batch)
    want = {n: e.run(q) for n, q, _ in QUERIES}
    yield e, want
    e.close()


def bit_same(got, want, ctx):
    assert len(got) == len(want), f"{ctx}: {len(got)} groups vs {len(want)}"
    for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(got, want):
        assert g1 == g2, f"{ctx}: group {g1} != {g2}"
        np.testing.assert_array_equal(t1, t2, err_msg=f"{ctx} g{g1} ts")
        np.testing.assert_array_equal(b1, b2, err_msg=f"{ctx} g{g1} bits")
        np.testing.assert_array_equal(i1, i2, err_msg=f"{ctx} g{g1} is_int")


def md_engine(devices, mode, batch, transport=E.MD_AUTO):
    e = E.Engine(devices=devices, transport=transport)
    e.shard_mode(mode)
    e.load(batch)
    return e


def test_one_device_context_is_bit_identical(batch, single):
    """ndev = 1: the multi-device context over device 0 returns the one-GPU results bit for bit."""
    _, want = single
    e = E.Engine(devices=[0])
    try:
        e.load(batch)
        nd, tr, mode, per = e.md_info()
        assert (nd, mode) == (1, E.SHARD_GROUPS) and int(per.sum()) == batch.n_series
        for n, q, _ in QUERIES:
            bit_same(e.run(q), want[n], f"ndev=1 {n}")
        assert e.timing().total_ms > 0
    finally:
        e.close()


@pytest.mark.parametrize("world", [2, 3, 5])
def test_group_shards_are_bit_identical(batch, single, world):
    """Whole SpanGroups per device: every query type, results concatenated, bit for bit."""
    _, want = single
    e = md_engine([0] * world, E.SHARD_GROUPS, batch)
    try:
        nd, tr, mode, per = e.md_info()
        assert (nd, tr, mode) == (world, E.MD_COPY, E.SHARD_GROUPS)
        assert int(per.sum()) == batch.n_series and (per > 0).sum() >= 2
        for n, q, _ in QUERIES:
            bit_same(e.run(q), want[n], f"groups x{world} {n}")
    finally:
        e.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_series_shards(batch, single, world):
    """Groups straddle devices: partial states gathered and merged in device order (oracle
    tolerance for float reductions); order statistics and ordered folds routed to each group's
    owner (bit for bit, only the straddling groups' rows move); NONE per span (bit for bit); raw
    group-by with the straddling groups evaluated whole on their owners (bit for bit)."""
    _, want = single
    e = md_engine([0] * world, E.SHARD_SERIES, batch)
    try:
        assert e.md_info()[2] == E.SHARD_SERIES
        for n, q, kind in QUERIES:
            if kind == "partials":
                got = e.run(q)
                assert_groups_match(got, O.run_query(batch, q), q_agg(q), ctx=f"series x{world} {n}")
                assert_groups_match(got, want[n], q_agg(q), ctx=f"series x{world} {n} vs one GPU")
            else:
                bit_same(e.run(q), want[n], f"series x{world} {n}")
            if kind == "sel":   # owner routing: far fewer bytes than every span's rows
                _, _, moved = e.md_stats()
                k = 60
                assert 0 < moved < batch.n_series * k * 8 / 2, (n, moved)
        e.run(QUERIES[0][1])
        t = e.timing()
        assert t.exchange_ms > 0 and t.devices_ms > 0   # the owner-routed exchange, the devices' passes
        per, ranks, _ = e.md_stats()
        assert len(per) == world and ranks == 0 and sum(t.datapoints for t in per) == e.timing().datapoints
    finally:
        e.close()


def device_count():
    return E.device_count()   # (not torch's: its own HIP runtime beside RCCL's broke ncclCommInitAll)


@pytest.mark.parametrize("transport", [E.MD_RCCL, E.MD_COPY])
def test_distinct_devices(batch, single, transport):
    """Every query kind over 2..N DISTINCT GPUs (series shards: partial gather, owner-routed
    selection, ordered folds, raw side contexts, NONE), RCCL send / recv and peer copies, against
    the one-GPU results.  Needs a multi-GPU machine."""
    n = device_count()
    if n < 2:
        pytest.skip("one visible GPU: distinct-device exchange needs two or more")
    _, want = single
    for world in sorted({2, min(n, 8)}):
        e = md_engine(list(range(world)), E.SHARD_SERIES, batch, transport=transport)
        try:
            assert e.md_info()[1] == transport
            for name, q, kind in QUERIES:
                got = e.run(q)
                if kind == "partials":
                    assert_groups_match(got, want[name], q_agg(q), ctx=f"distinct x{world} {name}")
                else:
                    bit_same(got, want[name], f"distinct x{world} {name}")
            if transport == E.MD_RCCL:
                assert e.md_stats()[1] == world
        finally:
            e.close()


def q_agg(q):
    return next(k for k, v in abi.AGG.items() if v == q.aggregator)


def test_rccl_gather_one_rank(batch, single):
    """The RCCL transport: ncclCommInitAll over [0], the gather as grouped send / recv."""
    _, want = single
    e = md_engine([0], E.SHARD_SERIES, batch, transport=E.MD_RCCL)
    try:
        assert e.md_info()[1] == E.MD_RCCL
        for n, q, kind in QUERIES:
            if kind == "partials":
                assert_groups_match(e.run(q), O.run_query(batch, q), q_agg(q), ctx=f"rccl {n}")
            elif kind in ("sel", "raw", "none"):
                bit_same(e.run(q), want[n], f"rccl {n}")
        assert e.md_stats()[1] == 1   # a one-rank communicator
    finally:
        e.close()


def test_auto_mode_and_more_devices_than_series(batch):
    """AUTO: 7 uneven groups over 2 devices are not within 10% -> SERIES; 64 groups -> GROUPS.
    Devices without series stay idle."""
    e = E.Engine(devices=[0, 0])
    try:
        e.load(batch)
        assert e.md_info()[2] == E.SHARD_SERIES
        e.synth(2000, T0, 360, 10000, value_kind=2, n_groups=64, int_mod=30000)
        assert e.md_info()[2] == E.SHARD_GROUPS
    finally:
        e.close()
    tiny = synth.generate(3, T0, 60, 60000, value_kind=1, n_groups=2, int_mod=100, seed=3)
    one = E.Engine(0)
    e = md_engine([0] * 8, E.SHARD_SERIES, tiny)
    try:
        one.load(tiny)
        assert (e.md_info()[3] > 0).sum() <= 3
        for agg in ["sum", "p99", "none"]:
            q = q_ds(agg)
            bit_same(e.run(q), one.run(q), f"tiny {agg}")
    finally:
        e.close()
        one.close()


@pytest.mark.parametrize("mode", [E.SHARD_GROUPS, E.SHARD_SERIES])
def test_synth_store(mode):
    """tsdbhip_synth on a multi-device context: each device generates its shard of the store."""
    args = (3000, T0, 360, 10000, 2, 64, 30000)
    one = E.Engine(0)
    e = E.Engine(devices=[0, 0, 0])
    try:
        one.synth(*args)
        e.shard_mode(mode)
        e.synth(*args)
        assert e.n_series() == args[0]
        for agg, ds in [("sum", "avg"), ("max", "sum"), ("dev", "avg"), ("p99", "avg"), ("none", "avg")]:
            q = q_ds(agg, ds)
            got, want = e.run(q), one.run(q)
            if mode == E.SHARD_GROUPS or agg in ("p99", "none", "max"):
                bit_same(got, want, f"synth {mode} {agg}")
            else:
                assert_groups_match(got, want, agg, ctx=f"synth {mode} {agg}")
    finally:
        e.close()
        one.close()


def test_run_multi_fused_on_every_device(batch, single):
    """tsdbhip_run_multi on group shards: each device runs the fused multi-aggregator pass."""
    one, _ = single
    qs = [q_ds(a, "avg") for a in ["sum", "avg", "min", "max", "count", "dev"]]
    want = one.run_multi(qs)
    fused_one = one.timing().fused_queries
    e = md_engine([0, 0, 0], E.SHARD_GROUPS, batch)
    try:
        got = e.run_multi(qs)
        for i, (g, w) in enumerate(zip(got, want)):
            bit_same(g, w, f"run_multi {i}")
        assert e.timing().fused_queries == fused_one
    finally:
        e.close()


MULTI_AGGS = ["sum", "avg", "min", "max", "count", "dev"]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_series_shards_run_multi_fused(batch, single, world):
    """tsdbhip_run_multi on series shards: one fused pass per device (tsdbhip_run_partials_multi)
    and one owner-routed exchange for all the queries; each result as the one-GPU run_multi's
    (the oracle's tolerance: float sums associate per device) and bit for bit for min / max /
    count.  The stage times of the call add up to its wall time."""
    one, _ = single
    qs = [q_ds(a, "avg") for a in MULTI_AGGS]
    want = one.run_multi(qs)
    e = md_engine([0] * world, E.SHARD_SERIES, batch)
    try:
        got = e.run_multi(qs)
        t = e.timing()
        assert t.fused_queries == len(qs)
        for a, g, w in zip(MULTI_AGGS, got, want):
            assert_groups_match(g, w, a, tol=0.0 if a in ("min", "max", "count") else None, ctx=f"x{world} {a}")
            assert_groups_match(g, O.run_query(batch, q_ds(a, "avg")), a, ctx=f"x{world} {a} oracle")
        stages = t.devices_ms + t.xfer_ms + t.select_ms + t.assemble_ms
        assert 0 < stages <= t.total_ms * 1.001, (stages, t.total_ms)
        assert abs(t.exchange_ms - (t.xfer_ms + t.select_ms + t.assemble_ms)) < 1e-9
        # owner routing: the straddling groups' K-slot states and the owners' dense rows move, not
        # every device's G x K partial states
        _, _, moved = e.md_stats()
        G, K = 7, 60
        assert 0 < moved < len(qs) * (world * G * K * 24) / 2, moved
    finally:
        e.close()


@pytest.mark.parametrize("world", [2, 3])
def test_series_shards_day_of_minute_buckets(world):
    """A day of 1m buckets (K = 1440, k_hwin) on series shards: single queries and the fused
    run_multi (k_hwin's MULTI variant on every device) against one GPU."""
    args = (2400, T0, 8640, 10000, 2, 13, 30000)
    one = E.Engine(0)
    e = E.Engine(devices=[0] * world)
    try:
        one.synth(*args)
        e.shard_mode(E.SHARD_SERIES)
        e.synth(*args)
        qs = [abi.new_query(T0, T0 + 86399, a, ds_function=abi.AGG["avg"], ds_interval_ms=60000) for a in MULTI_AGGS]
        want = [one.run(q) for q in qs]
        assert all(len(w[0][1]) == 1440 for w in want)
        got = e.run_multi(qs)
        assert e.timing().fused_queries == len(qs)
        for a, g, w in zip(MULTI_AGGS, got, want):
            assert_groups_match(g, w, a, tol=0.0 if a in ("min", "max", "count") else None, ctx=f"day x{world} {a}")
        for a, q, w in zip(MULTI_AGGS, qs, want):
            assert_groups_match(e.run(q), w, a, tol=0.0 if a in ("min", "max", "count") else None,
                                ctx=f"day x{world} {a} single")
        fused_one = one.run_multi(qs)
        assert one.timing().fused_queries == len(qs)
        for a, g, w in zip(MULTI_AGGS, fused_one, want):
            bit_same(g, w, f"one GPU day run_multi {a}")
    finally:
        e.close()
        one.close()


def test_run_multi_refuses_differing_downsampling(batch):
    """tsdbhip_run_multi's premise (one time range and downsampling) holds on a multi-device
    context as on one GPU, whatever the aggregators: the same refusal, named for run_multi."""
    e = md_engine([0, 0], E.SHARD_SERIES, batch)
    one = E.Engine(0)
    try:
        one.load(batch)
        for aggs in (["sum", "avg"], ["sum", "p99"]):
            qs = [q_ds(aggs[0]), q_ds(aggs[1], ds_interval_ms=300000)]
            for eng in (one, e):
                with pytest.raises(E.EngineError) as ei:
                    eng.run_multi(qs)
                assert ei.value.code == abi.TSDB_E_ILLEGAL_ARGUMENT and "run_multi" in str(ei.value)
    finally:
        e.close()
        one.close()


def test_store_bound_entry_points_refuse(batch):
    e = E.Engine(devices=[0, 0])
    try:
        e.load(batch)
        q = q_ds("sum")
        for call in [lambda: e.partials_layout(q, 7), lambda: e.load_shard(batch, 0, 0, 10), lambda: e.download(),
                     lambda: e.sel_layout(q_ds("p99"), 7)]:
            with pytest.raises(E.EngineError) as ei:
                call()
            assert ei.value.code == abi.TSDB_E_NOT_IMPLEMENTED
        with pytest.raises(E.EngineError):
            E.Engine(devices=[0, 0], transport=E.MD_RCCL)   # RCCL needs distinct devices
    finally:
        e.close()
