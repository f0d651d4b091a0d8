"""GPU parity of percentiles / median as the GROUP-BY aggregator:
AggregationIterator hands PercentileAgg.runDouble / Median.runDouble one value per span at
each union timestamp -- the span's bucket value or its LERP between neighbouring buckets
(src/core/AggregationIterator.java:735-797) -- and runDouble drops NaNs and always uses
LEGACY estimation (src/core/Aggregators.java:689-706; Median :416-430).  Queries without a
downsampler run on the raw path (tests/test_gpu_pct_raw.py).

Results are order statistics of exactly computed per-series values (plus commons-math3's
`lower + d * (upper - lower)`), so the bar is bit-exact against the oracle."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import set_option
from opentsdb_amd.query import TsdbQuery
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400
GSEL = ["p999", "p99", "p95", "p90", "p75", "p50", "ep99r3", "ep99r7", "median"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def mixed_batch():
    return synth.generate(70, T0, 720, 5000, value_kind=2, n_groups=3, int_mod=30000, seed=11)


@pytest.mark.parametrize("agg", GSEL)
def test_pct_group_aggregators(eng, mixed_batch, agg):
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), agg, tol=0.0, ctx=agg)


@pytest.mark.parametrize("ds", ["sum", "max", "min", "count", "dev", "first", "p99", "median"])
def test_pct_group_over_downsample_functions(eng, mixed_batch, ds):
    q = abi.new_query(T0, T0 + 3599, "p95", ds_function=abi.AGG[ds], ds_interval_ms=300000)
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), "p95", tol=0.0, ctx=ds)


def test_pct_group_single_group_many_series(eng):
    # one group of 300 series: segments longer than a wave, ties between integer series
    b = synth.generate(300, T0, 360, 10000, value_kind=1, n_groups=1, int_mod=50, seed=3)
    for agg in ["p99", "p50", "median", "p999"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["max"], ds_interval_ms=60000)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, tol=0.0, ctx=agg)


@pytest.mark.parametrize("win", ["1", "2"])   # (2: the sampled window for any group size)
@pytest.mark.parametrize("fill", [abi.FILL_NAN, abi.FILL_ZERO, abi.FILL_NULL])
def test_pct_group_fill(eng, monkeypatch, fill, win):
    set_option("SEL_WIN", win)
    b = synth.generate(20, T0 + 1800, 200, 10000, value_kind=2, n_groups=2, int_mod=1000, seed=4)
    q = abi.new_query(T0, T0 + 7199, "p90", ds_function=abi.AGG["avg"], ds_interval_ms=300000, ds_fill=fill)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "p90", tol=0.0, ctx=f"fill {fill}")


@pytest.mark.parametrize("opts", [dict(), dict(counter=True), dict(counter=True, drop_resets=True)])
def test_pct_group_rate(eng, opts):
    b = synth.generate(24, T0, 360, 10000, value_kind=1, n_groups=3, int_mod=1000, seed=9)
    for ds in ["avg", "p75"]:
        q = abi.new_query(T0, T0 + 3599, "p50", ds_function=abi.AGG[ds], ds_interval_ms=60000, rate=True, **opts)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "p50", tol=0.0, ctx=f"{ds} {opts}")


def test_pct_group_all(eng, mixed_batch):
    q = abi.new_query(T0 * 1000, (T0 + 3600) * 1000, "p75", ds_function=abi.AGG["sum"], ds_all=True)
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), "p75", tol=0.0, ctx="all")


@pytest.mark.parametrize("win", ["1", "2"])
def test_pct_group_sparse_lerp(eng, monkeypatch, win):
    """Series with missing buckets and different extents: LERP-interpolated members (option SEL_WIN = 2:
    through the sampled window where the batch qualifies)."""
    set_option("SEL_WIN", win)
    rng = np.random.default_rng(17)
    from opentsdb_amd.store import MockStore
    st = MockStore()
    for s in range(40):
        ts = np.sort(rng.choice(np.arange(0, 7200, 7), size=rng.integers(3, 150), replace=False))
        for t in ts:
            if s % 3 == 0:
                st.add_float("m", T0 + int(t), float(rng.normal(10, 5)), {"h": f"h{s}", "g": f"g{s % 3}"})
            else:
                st.add_long("m", T0 + int(t), int(rng.integers(-1000, 1000)), {"h": f"h{s}", "g": f"g{s % 3}"})
    for agg in ["p99", "p50", "median", "ep90r7"]:
        q = TsdbQuery(st, runner=eng.run_batch)
        q.setStartTime(T0)
        q.setEndTime(T0 + 7199)
        q.setTimeSeries("m", {"g": "*"}, agg, False)
        q.downsample("2m-avg")
        batch, _ = q.build_batch()
        assert_groups_match(eng.run_batch(batch, q.to_abi()), O.run_query(batch, q.to_abi()), agg, tol=0.0, ctx=agg)


@pytest.mark.parametrize("win", ["1", "2"])
def test_pct_group_nan_members(eng, monkeypatch, win):
    """Buckets of NaNs (present, value NaN) are dropped by runDouble; a slot whose members
    are all NaN yields NaN (option SEL_WIN = 2: also through the sampled window)."""
    set_option("SEL_WIN", win)
    rng = np.random.default_rng(5)
    rows, gids = [], []
    for s in range(12):
        ts = T0 * 1000 + np.sort(rng.choice(np.arange(0, 3600), 300, replace=False)) * 1000
        f = rng.normal(0, 10, 300)
        f[rng.random(300) < 0.2] = np.nan
        if s in (3, 4, 5):
            f[:] = np.nan
        kind = np.full(300, 2)
        rows.append(synth.encode_rows(ts, np.zeros(300, np.int64), f, kind, np.zeros(300, bool)))
        gids.append(0 if s < 6 else 1)
    b = synth.from_series(rows, gids)
    for agg in ["p90", "median"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["max"], ds_interval_ms=600000)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, tol=0.0, ctx=agg)


def test_pct_group_segment_beyond_lds(eng):
    """One group of 13000 spans: each (group, slot) column exceeds the LDS stage (SEL_CAP =
    12288 values) and is selected in the global-memory key space."""
    eng.synth(13000, T0, 360, 10000, 2, 1, 30000, 0x5EED)
    b = eng.download()
    for agg in ["p99", "median", "p50"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=300000)
        assert_groups_match(eng.run(q), O.run_query(b, q), agg, tol=0.0, ctx=agg)


@pytest.mark.parametrize("cols", ["0", "1"])
def test_pct_group_column_layout(eng, mixed_batch, monkeypatch, cols):
    """The fused percentile pass writes each (group, slot) column contiguously (sel_cols) or one
    row per series (option SEL_COLS = 0): both feed the same select and match the oracle, incl.
    a single group wider than a wave and the LDS-staged select."""
    set_option("SEL_COLS", cols)
    for agg in ["p99", "median", "ep99r7"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), agg, tol=0.0, ctx=agg)
    b = synth.generate(300, T0, 360, 10000, value_kind=1, n_groups=1, int_mod=50, seed=3)
    q = abi.new_query(T0, T0 + 3599, "p50", ds_function=abi.AGG["max"], ds_interval_ms=60000)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "p50", tol=0.0, ctx="one group")


@pytest.mark.parametrize("variant", [{}, {"SEL_WAVE": 0}, {"SEL_WAVE": 0, "SEL_COLS": 0}, {"SEL_REG": 0, "SEL_WAVE": 0}])
def test_pct_group_select_kernels(eng, variant):
    """The select kernels -- k_sel_wave (columns of <= 2048 values), the register-resident block
    select k_sel_reg (512 x 24 keys) and the LDS k_sel_seg -- against the oracle: segments of a
    few values, ~3000 values with clustered integers (ties: several radix digits), negative
    rates, members without a value, both layouts."""
    for k, v in variant.items():
        set_option(k, v)
    if variant:   # (the block kernels also for the small segments k_sel_wave takes by default)
        set_option("SEL_WAVE", "0")
    mixed = synth.generate(70, T0, 720, 5000, value_kind=2, n_groups=3, int_mod=30000, seed=11)
    ties = synth.generate(3000, T0, 360, 10000, value_kind=1, n_groups=1, int_mod=7, seed=5)
    for b, ds, rate in ((mixed, "avg", False), (ties, "max", False), (ties, "avg", False), (ties, "avg", True)):
        for agg in ["p999", "p99", "median", "p50", "ep90r7"]:
            # (rate over u mod 7: negative and positive rates of equal magnitude)
            q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG[ds], ds_interval_ms=60000, rate=rate)
            assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, tol=0.0, ctx=f"{agg} {ds} {variant}")


@pytest.mark.parametrize("n", [256, 1000, 2048, 2049])
@pytest.mark.parametrize("kind", ["ties", "mixed"])
def test_pct_group_wave_select(eng, monkeypatch, n, kind):
    """k_sel_wave (a wave a column, columns of at most 64 x 4 / 16 / 32 values; 2049 takes the
    block kernel) against the oracle at each size class's edge, with clustered integers (long
    runs of equal keys) or mixed integer / float spans (empty slots past the data's end), both
    layouts, and option SEL_WAVE = 0 alike.  (Members without a value: the NaN-member and sparse
    LERP tests above, whose groups are small, so they take k_sel_wave.)"""
    if kind == "ties":
        eng.synth(n, T0 + 60, 300, 20000, 1, 1, 7, 0x60 + n)
    else:
        eng.synth(n, T0 + 60, 300, 20000, 2, 1, 30000, 0x61 + n)
    b = eng.download()
    for wave in ["1", "0"]:
        set_option("SEL_WAVE", wave)
        for cols in ["1", "0"]:
            set_option("SEL_COLS", cols)
            for agg in ["p999", "p99", "median", "p50", "ep90r7"]:
                q = abi.new_query(T0, T0 + 7199, agg, ds_function=abi.AGG["avg"], ds_interval_ms=300000)
                assert_groups_match(eng.run(q), O.run_query(b, q, threads=8), agg, tol=0.0,
                                    ctx=f"{kind} n={n} {agg} wave={wave} cols={cols}")


def test_pct_group_sampled_window(eng, monkeypatch):
    """The sampled-window select (groups of >= 4096 spans on the short streaming tiles): a sample
    pass over every stride-th tile bounds a window around the target ranks of each (group, slot)
    column, the main pass keeps only the values inside it, and the select ranks them with exact
    counts -- bit-exact against the oracle, and taken without falling back on regular data."""
    eng.synth(60_000, T0, 360, 10000, 2, 6, 30000, 0x5EED)
    b = eng.download()
    r0 = eng.debug_sel_window()
    for agg in ["p99", "p999", "ep99r7", "p95", "ep90r7"]:   # (p95 / p90 over 10000: windows too wide, full path)
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        assert_groups_match(eng.run(q), O.run_query(b, q, threads=8), agg, tol=0.0, ctx=f"window {agg}")
    r1 = eng.debug_sel_window()
    assert (r1[0] - r0[0], r1[1] - r0[1]) == (3, 0), f"window runs / misses {r0} -> {r1}"
    # mid ranks keep the full path; option SEL_WIN = 2 takes the window for them too
    q = abi.new_query(T0, T0 + 3599, "median", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    assert_groups_match(eng.run(q), O.run_query(b, q, threads=8), "median", tol=0.0, ctx="median full path")
    assert eng.debug_sel_window()[0] == r1[0]
    set_option("SEL_WIN", "2")   # (windows wider than a column holds: they fall back)
    for agg in ["median", "p75", "p95"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        assert_groups_match(eng.run(q), O.run_query(b, q, threads=8), agg, tol=0.0, ctx=f"window {agg}")
    r2 = eng.debug_sel_window()
    assert r2[0] - r1[0] == 3, f"window runs {r1} -> {r2}"
    # option SEL_WIN = 0: the full path, the same results
    set_option("SEL_WIN", "0")
    q = abi.new_query(T0, T0 + 3599, "p99", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    assert_groups_match(eng.run(q), O.run_query(b, q, threads=8), "p99", tol=0.0, ctx="full path")
    assert eng.debug_sel_window()[0] == r2[0]


@pytest.mark.parametrize("kind", ["ties", "small"])
def test_pct_group_sampled_window_fallback(eng, monkeypatch, kind):
    """Windows that miss (a few distinct values tie across the window: more kept values than a
    (tile, slot) holds) and small groups forced through the window (option SEL_WIN = 2, sparse
    samples): the query falls back to the full path where a column misses -- the oracle's answers
    either way."""
    if kind == "ties":
        eng.synth(20_000, T0, 360, 10000, 1, 2, 3, 0x51)
    else:
        eng.synth(3_000, T0, 360, 10000, 2, 7, 30000, 0x52)
    b = eng.download()
    # (also the full path: ties of more than 256 equal keys resolved to the last bit, a round-5 fix
    # of the 12-bit first digit -- these keys' low 3 bits were left unresolved)
    for win in ["2", "0"]:
        set_option("SEL_WIN", win)
        for agg in ["p99", "median", "p50"]:
            for ds in ["avg", "max"]:
                q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG[ds], ds_interval_ms=60000)
                assert_groups_match(eng.run(q), O.run_query(b, q, threads=8), agg, tol=0.0,
                                    ctx=f"{kind} {agg} {ds} win={win}")
    assert eng.debug_sel_window()[0] > 0
