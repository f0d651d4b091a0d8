"""GPU parity: libtsdbhip (HIP, gfx950) against the CPU oracle and the reference's
known answers.  Every comparison goes through the C ABI.

Bar (BASELINE.json north_star): timestamps, counts and integer aggregates bit-exact;
floats within REL_TOL (relative) -- cross-series float sums are reduced in a
deterministic tree order on the GPU instead of SpanGroup index order."""
from __future__ import annotations

import math

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.query import TsdbQuery
from oracle import oracle as O
from tests import golden_util as G

pytestmark = pytest.mark.gpu

REL_TOL = 1e-12       # sum / avg / squareSum / interpolated values
DEV_TOL = 1e-9        # dev: Chan merge of per-tile Welford states vs one sequential Welford
EXACT = {"min", "max", "mimmin", "mimmax", "count", "first", "last", "none"}


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def assert_groups_match(got, want, agg, tol=None, ctx=""):
    if tol is None:
        tol = 0.0 if agg in EXACT else (DEV_TOL if agg == "dev" else REL_TOL)
    assert len(got) == len(want), f"{ctx}: {len(got)} groups vs {len(want)}"
    for (gg, ts1, b1, i1), (wg, ts2, b2, i2) in zip(got, want):
        assert gg == wg, f"{ctx}: group id {gg} != {wg}"
        assert len(ts1) == len(ts2), f"{ctx} g{gg}: {len(ts1)} points vs {len(ts2)}"
        np.testing.assert_array_equal(ts1, ts2, err_msg=f"{ctx} g{gg}: timestamps")
        np.testing.assert_array_equal(i1, i2, err_msg=f"{ctx} g{gg}: is_int")
        ints = i2.astype(bool)
        np.testing.assert_array_equal(b1[ints], b2[ints], err_msg=f"{ctx} g{gg}: integer values")
        d1 = b1[~ints].view(np.float64)
        d2 = b2[~ints].view(np.float64)
        n1, n2 = np.isnan(d1), np.isnan(d2)
        np.testing.assert_array_equal(n1, n2, err_msg=f"{ctx} g{gg}: NaN positions")
        if tol == 0.0:
            np.testing.assert_array_equal(b1[~ints][~n1], b2[~ints][~n2], err_msg=f"{ctx} g{gg}: values (bit-exact)")
        else:
            a, b = d1[~n1], d2[~n2]
            err = np.abs(a - b) / np.maximum(1.0, np.abs(b))
            assert err.size == 0 or err.max() <= tol, f"{ctx} g{gg}: max rel err {err.max()} > {tol}"


# ---- reference known answers (downsampled queries) through the engine --------------
QUERIES = G.load("queries.json")
GRID_CASES = QUERIES["cases"]


@pytest.mark.parametrize("case", GRID_CASES, ids=[c["name"] for c in GRID_CASES])
def test_golden_queries_on_gpu(eng, case):
    store = G.store_from(QUERIES["stores"][case["store"]])
    q = G.query_from(case, store, eng.run_batch)
    got = G.groups_as_points(q.run())
    want = case["expect"] if case["multi_group"] else [case["expect"]]
    assert len(got) == len(want)
    for g, w in zip(got, want):
        G.assert_points(g, w, case["tol"], case["check_int"], case["name"])
    # and against the oracle on the same inputs
    qo = G.query_from(case, store, O.run_query)
    batch, _ = q.build_batch()
    assert_groups_match(eng.run_batch(batch, q.to_abi()), O.run_query(batch, q.to_abi()), case["aggregator"],
                        ctx=case["name"])


# ---- synthetic parity matrix ----------------------------------------------------------
T0 = 1356998400


def synth_batch(n_series, n_points, period_ms, kind, groups, int_mod=30000, seed=0x5EED, start=T0):
    return synth.generate(n_series, start, n_points, period_ms, value_kind=kind, n_groups=groups,
                          int_mod=int_mod, seed=seed)


AGGS = ["sum", "avg", "min", "max", "count", "dev", "zimsum", "mimmin", "mimmax", "squareSum", "first", "last",
        "diff", "pfsum"]
DS_FUNS = ["avg", "sum", "min", "max", "count", "dev", "first", "last", "diff", "squareSum", "mult"]


@pytest.fixture(scope="module")
def float_batch():
    return synth_batch(96, 720, 5000, 0, 4)


@pytest.fixture(scope="module")
def mixed_batch():
    return synth_batch(96, 360, 10000, 2, 5)


@pytest.mark.parametrize("agg", AGGS)
def test_synth_groupby_aggregators(eng, float_batch, agg):
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    assert_groups_match(eng.run_batch(float_batch, q), O.run_query(float_batch, q), agg, ctx=agg)


@pytest.mark.parametrize("ds", DS_FUNS)
def test_synth_downsample_functions(eng, mixed_batch, ds):
    q = abi.new_query(T0, T0 + 3599, "max", ds_function=abi.AGG[ds], ds_interval_ms=60000)
    # max is order-insensitive: the per-bucket downsample values must be bit-exact
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), "max", ctx=ds)


@pytest.mark.parametrize("interval", [1000, 7000, 60000, 90000, 600000, 3600000, 86400000])
def test_synth_intervals(eng, mixed_batch, interval):
    q = abi.new_query(T0 + 17, T0 + 3000, "sum", ds_function=abi.AGG["sum"], ds_interval_ms=interval)
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), "sum", ctx=str(interval))


@pytest.mark.parametrize("fill", [abi.FILL_NAN, abi.FILL_ZERO, abi.FILL_NULL])
@pytest.mark.parametrize("agg", ["sum", "avg", "count", "min"])
def test_synth_fill_policies(eng, mixed_batch, fill, agg):
    q = abi.new_query(T0, T0 + 7200, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000, ds_fill=fill)
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), agg, ctx=f"{fill}-{agg}")


def test_scalar_fill_raises(eng, mixed_batch):
    from opentsdb_amd.engine import EngineError
    q = abi.new_query(T0, T0 + 7200, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000, ds_fill=abi.FILL_SCALAR)
    with pytest.raises(EngineError) as ei:
        eng.run_batch(mixed_batch, q)
    with pytest.raises(O.OracleError) as eo:
        O.run_query(mixed_batch, q)
    assert ei.value.java == eo.value.java == "RuntimeException"


@pytest.mark.parametrize("opts", [dict(), dict(counter=True), dict(counter=True, drop_resets=True),
                                  dict(counter=True, counter_max=100000, reset_value=50)])
def test_synth_rate(eng, opts):
    b = synth_batch(40, 360, 10000, 1, 3, int_mod=1000)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000, rate=True, **opts)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "sum", ctx=str(opts))


def test_synth_all_downsample(eng, mixed_batch):
    for qs, qe in [(T0 * 1000, (T0 + 3600) * 1000), ((T0 + 100) * 1000, (T0 + 900) * 1000), (T0, T0 + 3600)]:
        q = abi.new_query(qs, qe, "sum", ds_function=abi.AGG["sum"], ds_all=True)
        assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), "sum", ctx=f"all {qs}")


def test_none_aggregator(eng, mixed_batch):
    q = abi.new_query(T0, T0 + 3599, "none", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), "none", ctx="none")


def test_sparse_series_lerp(eng):
    """Series with missing buckets: LERP / ZIM / MAX / MIN / PREV between their points."""
    rng = np.random.default_rng(7)
    from opentsdb_amd.store import MockStore, make_batch
    st = MockStore()
    for s in range(30):
        ts = np.sort(rng.choice(np.arange(0, 7200, 7), size=rng.integers(5, 200), replace=False))
        for t in ts:
            if s % 3 == 0:
                st.add_float("m", T0 + int(t), float(rng.normal(10, 5)), {"h": f"h{s}", "g": f"g{s % 4}"})
            else:
                st.add_long("m", T0 + int(t), int(rng.integers(-1000, 1000)), {"h": f"h{s}", "g": f"g{s % 4}"})
    for agg in ["sum", "zimsum", "mimmin", "mimmax", "pfsum", "avg", "count", "min", "max"]:
        q = TsdbQuery(st, runner=eng.run_batch)
        q.setStartTime(T0)
        q.setEndTime(T0 + 7199)
        q.setTimeSeries("m", {"g": "*"}, agg, False)
        q.downsample("2m-avg")
        batch, _ = q.build_batch()
        assert_groups_match(eng.run_batch(batch, q.to_abi()), O.run_query(batch, q.to_abi()), agg, ctx=agg)


def test_device_synth_matches_host_synth(eng):
    for args in [(50, 400, 10000, 2, 3, 30000), (20, 3600, 1000, 0, 2, 0), (10, 300, 1500, 1, 1, 300)]:
        n, npts, period, kind, groups, mod = args
        eng.synth(n, T0 + 30, npts, period, kind, groups, max(mod, 1), 0x5EED)
        dev = eng.download()
        host = synth_batch(n, npts, period, kind, groups, int_mod=max(mod, 1), start=T0 + 30)
        np.testing.assert_array_equal(dev.series_row_ptr, host.series_row_ptr)
        np.testing.assert_array_equal(dev.row_base_time, host.row_base_time)
        np.testing.assert_array_equal(dev.row_qual_off, host.row_qual_off)
        np.testing.assert_array_equal(dev.row_val_off, host.row_val_off)
        np.testing.assert_array_equal(dev.qual, host.qual)
        np.testing.assert_array_equal(dev.val, host.val)
        np.testing.assert_array_equal(dev.group_id, host.group_id)


def test_bench_config_scaled_down(eng):
    """BASELINE config 2 shape (1 h @1 s float32, sum:1m-avg, 64 groups) at 1/500 scale,
    generated on the device, checked against the oracle on the downloaded bytes."""
    eng.synth(2000, T0, 3600, 1000, 0, 64, 1, 0x5EED)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    got = eng.run(q)
    host = eng.download()
    assert_groups_match(got, O.run_query(host, q), "sum", ctx="config2/500")
    t = eng.timing()
    assert t.datapoints == 2000 * 3600


def test_malformed_row_raises(eng):
    b = synth_batch(4, 100, 10000, 1, 1, int_mod=1000)
    qual = b.qual.copy()
    qual[1] = (qual[1] & 0xF0) | 0x2      # 3-byte integer: illegal length
    bad = abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, qual, b.val, b.group_id)
    from opentsdb_amd.engine import EngineError
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["sum"], ds_interval_ms=60000)
    with pytest.raises(EngineError) as ei:
        eng.run_batch(bad, q)
    assert ei.value.java == "IllegalDataException"
