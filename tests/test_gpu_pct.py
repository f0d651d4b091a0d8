"""GPU parity of percentile / median downsampling (BASELINE config 5's 1h-p99 /
1h-ep99r7): per-bucket order statistics with commons-math3 LEGACY estimation (the
reference's runDouble ignores ep*r3 / ep*r7, src/core/Aggregators.java:690), NaNs skipped,
then the usual group-by.  Downsampled values are bit-exact (checked through the
order-insensitive max / min / count group aggregators); float sums within REL_TOL."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import set_option
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400
SEL = ["p999", "p99", "p95", "p90", "p75", "p50", "ep99r3", "ep99r7", "ep50r3", "ep999r7", "median"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def day_batch():
    # config 5 shape at small scale: 1 day @10 s, float32 (360 values per 1 h bucket)
    return synth.generate(24, T0, 8640, 10000, value_kind=0, n_groups=3, seed=0x5EED)


@pytest.fixture(scope="module")
def mixed_batch():
    return synth.generate(30, T0, 720, 5000, value_kind=2, n_groups=4, int_mod=30000, seed=7)


@pytest.mark.parametrize("fn", SEL)
def test_pct_1h_config5_shape(eng, day_batch, fn):
    q = abi.new_query(T0, T0 + 86399, "max", ds_function=abi.AGG[fn], ds_interval_ms=3600000)
    assert_groups_match(eng.run_batch(day_batch, q), O.run_query(day_batch, q), "max", ctx=fn)


@pytest.mark.parametrize("fn", ["p99", "p50", "ep90r7", "median"])
@pytest.mark.parametrize("interval", [15000, 60000, 600000, 3600000])
def test_pct_bucket_sizes(eng, mixed_batch, fn, interval):
    # 3 .. 720 values per bucket: register sort (<= 512) and LDS sort (> 512)
    q = abi.new_query(T0, T0 + 3599, "min", ds_function=abi.AGG[fn], ds_interval_ms=interval)
    assert_groups_match(eng.run_batch(mixed_batch, q), O.run_query(mixed_batch, q), "min", ctx=f"{fn} {interval}")


@pytest.mark.parametrize("agg", ["sum", "avg", "count", "dev", "zimsum", "mimmax", "first", "last"])
def test_pct_groupby_aggregators(eng, day_batch, agg):
    q = abi.new_query(T0, T0 + 86399, agg, ds_function=abi.AGG["p99"], ds_interval_ms=3600000)
    assert_groups_match(eng.run_batch(day_batch, q), O.run_query(day_batch, q), agg, ctx=agg)


@pytest.mark.parametrize("fill", [abi.FILL_NAN, abi.FILL_ZERO])
def test_pct_fill_and_rate(eng, fill):
    b = synth.generate(20, T0 + 1800, 200, 10000, value_kind=1, n_groups=2, int_mod=1000, seed=3)
    q = abi.new_query(T0, T0 + 7199, "sum", ds_function=abi.AGG["p90"], ds_interval_ms=300000, ds_fill=fill)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "sum", ctx=f"fill {fill}")
    q = abi.new_query(T0, T0 + 7199, "sum", ds_function=abi.AGG["median"], ds_interval_ms=300000, rate=True)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "sum", ctx="rate")


def test_pct_nan_values_and_all(eng):
    rng = np.random.default_rng(5)
    rows, gids = [], []
    for s in range(10):
        ts = T0 * 1000 + np.sort(rng.choice(np.arange(0, 3600), 300, replace=False)) * 1000
        f = rng.normal(0, 10, 300)
        f[rng.random(300) < 0.2] = np.nan
        if s == 3:
            f[:] = np.nan   # buckets of NaNs only -> NaN values (present buckets)
        kind = np.full(300, 2)
        rows.append(synth.encode_rows(ts, np.zeros(300, np.int64), f, kind, np.zeros(300, bool)))
        gids.append(s % 2)
    order = sorted(range(10), key=lambda i: gids[i])
    b = synth.from_series([rows[i] for i in order], [gids[i] for i in order])
    for fn in ["p99", "median", "p50"]:
        for agg in ["max", "count"]:
            q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG[fn], ds_interval_ms=600000)
            assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, ctx=f"{fn} {agg}")
    q = abi.new_query(T0, T0 + 3600, "max", ds_function=abi.AGG["p95"], ds_all=True)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "max", ctx="all")


def test_pct_large_bucket_lds_sort(eng):
    # 1 h @ 1 s: 3600 values per bucket (LDS sort up to PCT_CAP = 4096)
    b = synth.generate(6, T0, 3600, 1000, value_kind=4, n_groups=2, seed=9)
    q = abi.new_query(T0, T0 + 3599, "max", ds_function=abi.AGG["p99"], ds_interval_ms=3600000)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "max", ctx="3600/bucket")


@pytest.mark.parametrize("fn", ["p99", "median", "p50", "ep999r7"])
def test_pct_1d_buckets_over_lds_capacity(eng, fn):
    """1d-p99 / 1d-median over 1 day @10 s: 8640 values per bucket, above PCT_CAP (4096) --
    the large-bucket pass spills them to its global region and radix-selects (the reference
    has no size limit, src/core/Aggregators.java:657-708)."""
    b = synth.generate(40, T0, 8640, 10000, value_kind=2, n_groups=3, int_mod=30000, seed=12)
    q = abi.new_query(T0, T0 + 86399, "max", ds_function=abi.AGG[fn], ds_interval_ms=86400000)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "max", ctx=f"1d-{fn}")
    q = abi.new_query(T0, T0 + 86399, "sum", ds_function=abi.AGG[fn], ds_interval_ms=86400000)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "sum", ctx=f"1d-{fn} sum")


def test_pct_2h_p95_at_1s(eng):
    """2h-p95 @1 s: 7200 values per bucket, full-mantissa doubles, ties-free."""
    b = synth.generate(12, T0, 14400, 1000, value_kind=4, n_groups=2, seed=9)
    for fn in ["p95", "p999", "median"]:
        q = abi.new_query(T0, T0 + 14399, "max", ds_function=abi.AGG[fn], ds_interval_ms=7200000)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "max", ctx=f"2h-{fn}")


def test_pct_large_buckets_with_ties_and_nans(eng):
    """Buckets of 5000-20000 values with 7 distinct values (radix-select ties) and NaNs."""
    rng = np.random.default_rng(21)
    rows, gids = [], []
    for s in range(8):
        n = 5000 + 2000 * s
        ts = T0 * 1000 + np.arange(n, dtype=np.int64) * 1000
        f = rng.integers(0, 7, n).astype(np.float64)
        f[rng.random(n) < 0.05] = np.nan
        kind = np.full(n, 2)
        rows.append(synth.encode_rows(ts, np.zeros(n, np.int64), f, kind, np.zeros(n, bool)))
        gids.append(0)
    b = synth.from_series(rows, gids)
    for fn in ["p99", "p50", "median", "p999"]:
        q = abi.new_query(T0, T0 + 86399, "max", ds_function=abi.AGG[fn], ds_interval_ms=86400000)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "max", ctx=f"ties {fn}")


def test_pct_sharded(eng, day_batch):
    from tests.test_gpu_dist import run_sharded
    from opentsdb_amd.engine import Engine
    es = [eng, Engine(0)]
    try:
        q = abi.new_query(T0, T0 + 86399, "sum", ds_function=abi.AGG["ep99r7"], ds_interval_ms=3600000)
        assert_groups_match(run_sharded(es, day_batch, q, 2), O.run_query(day_batch, q), "sum", ctx="x2")
    finally:
        es[1].close()


@pytest.mark.parametrize("fn", ["p999", "p99", "p95", "ep99r3", "ep99r7", "ep999r7"])
@pytest.mark.parametrize("interval", [60000, 600000, 3600000])
def test_pct_extreme_selection_with_ties(eng, fn, interval):
    # order statistics near either end (selection by extraction): integer values with many
    # ties (5 distinct values) and 6..360 values per bucket
    b = synth.generate(16, T0, 360, 10000, value_kind=1, n_groups=2, int_mod=5, seed=11)
    q = abi.new_query(T0, T0 + 3599, "max", ds_function=abi.AGG[fn], ds_interval_ms=interval)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "max", ctx=f"{fn} {interval}")


@pytest.mark.parametrize("fn", ["median", "p50", "p75", "ep50r7", "p90", "p999"])
def test_pct_mid_ranks_key_kernel(eng, fn):
    """1 h buckets of 4-byte values through k_pct_rows' 32-bit key kernel at any rank: the
    bitwise rank search (median, p50, p75) and extraction (near the ends) on float32 rows with
    ties, NaNs, negative values (and +-0.0 for the median), and on int32 rows with few distinct
    values; buckets
    of 1..360 values (points missing at random), and rows of distinct values."""
    rng = np.random.default_rng(17)
    rows, gids = [], []
    for s in range(20):
        keep = rng.random(3 * 360) < (0.9 if s % 5 else 0.01)
        ts = T0 * 1000 + np.flatnonzero(keep).astype(np.int64) * 10000
        n = len(ts)
        if s >= 14:   # distinct values: the rank search's candidate set ends at any rank
            f = rng.normal(0, 1e3, n) * (1 + s)
            rows.append(synth.encode_rows(ts, np.zeros(n, np.int64), f, np.full(n, 1), np.zeros(n, bool)))
        elif s % 2 == 0:
            f = np.round(rng.normal(0, 20, n) * 2) / 2
            f[rng.random(n) < 0.1] = np.nan
            if fn == "median":   # Collections.sort orders -0.0 before 0.0; commons-math's
                # KthSelector leaves the order of equal zeros to its partitioning (not restated)
                f[rng.random(n) < 0.05] = -0.0
                f[rng.random(n) < 0.05] = 0.0
            rows.append(synth.encode_rows(ts, np.zeros(n, np.int64), f, np.full(n, 1), np.zeros(n, bool)))
        else:
            lv = rng.integers(40000, 40006, n) * (1 if s % 3 else -1)
            rows.append(synth.encode_rows(ts, lv, np.zeros(n), np.zeros(n, np.int64), np.zeros(n, bool)))
        gids.append(s % 3)
    order = sorted(range(20), key=lambda i: gids[i])
    b = synth.from_series([rows[i] for i in order], [gids[i] for i in order])
    for agg in ["max", "min", "count"]:
        q = abi.new_query(T0, T0 + 3 * 3600 - 1, agg, ds_function=abi.AGG[fn], ds_interval_ms=3600000)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, ctx=f"{fn} {agg}")
    q = abi.new_query(T0, T0 + 3 * 3600 - 1, "none", ds_function=abi.AGG[fn], ds_interval_ms=3600000)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "none", tol=0.0, ctx=f"{fn} none")


def _vonly_batch(seed=23):
    """Rows k_index certifies for the values-only key kernel (every row 4-byte values, all float32
    without NaN or all int32, sorted) plus the cases it must hand back to k_pct: an int32 MIN value
    (keys to 0 = absent), and a row whose last offset is past its hour (2-byte qualifiers reach
    4095 s).  Buckets of 1..360 values, rows of any length (partial lanes)."""
    rng = np.random.default_rng(seed)
    rows, gids = [], []
    for s in range(18):
        keep = rng.random(3 * 360) < (0.85 if s % 4 else 0.02)
        ts = T0 * 1000 + np.flatnonzero(keep).astype(np.int64) * 10000
        n = len(ts)
        if s % 2 == 0:   # float32, ties and negatives, no NaN
            f = np.round(rng.normal(0, 50, n) * 4) / 4 + (1 + s) * 0.5
            rows.append(synth.encode_rows(ts, np.zeros(n, np.int64), f, np.full(n, 1), np.zeros(n, bool)))
        else:            # int32 (4-byte vle), few distinct values, both signs
            lv = rng.integers(70000, 70009, n) * (1 if s % 3 else -1) * (1 + s)
            if s == 5:
                lv[rng.random(n) < 0.1] = -(1 << 31)   # int32 MIN: handed back to k_pct
            if s == 7:
                lv[:] = rng.integers(-(1 << 31) + 1, (1 << 31) - 1, n)
            rows.append(synth.encode_rows(ts, lv, np.zeros(n), np.zeros(n, np.int64), np.zeros(n, bool)))
        gids.append(s % 3)
    # series 9: its first hour row carries 20 more int32 points at offsets 3600..3790 s (the
    # next hour's bucket), as a row may under 2-byte qualifiers
    base, q, v = rows[9][0]
    extra_q = b"".join((((3600 + 10 * k) << 4) | 3).to_bytes(2, "big") for k in range(20))
    extra_v = b"".join(int(-90000 - k).to_bytes(4, "big", signed=True) for k in range(20))
    meta = v[-1:] if len(v) % 4 == 1 else b"\x00"
    body = v[:len(v) - len(meta)]
    rows[9][0] = (base, q + extra_q, body + extra_v + meta)
    order = sorted(range(18), key=lambda i: gids[i])
    return synth.from_series([rows[i] for i in order], [gids[i] for i in order])


@pytest.mark.parametrize("fn", ["p99", "p999", "p90", "ep99r7", "p75", "p50", "median"])
def test_pct_values_only_key_rows(eng, fn, monkeypatch):
    """k_pct_rows' values-only key kernel (rows certified at load read 4 B a datapoint, one
    qualifier a row; 6 values a lane when no row exceeds 384, else 8) against the oracle, and
    bit-identical to the qualifier-reading key kernel (option PCT_VONLY = 0)."""
    b = _vonly_batch()
    res = {}
    modes = [("1", "1"), ("1", "0"), ("0", "1")]   # (option PCT_VONLY, option PCT_V6)
    for vonly, v6 in modes:
        set_option("PCT_VONLY", vonly)
        set_option("PCT_V6", v6)
        for agg in ["max", "min", "none"]:
            q = abi.new_query(T0, T0 + 3 * 3600 - 1, agg, ds_function=abi.AGG[fn], ds_interval_ms=3600000)
            got = eng.run_batch(b, q)
            assert_groups_match(got, O.run_query(b, q), agg, tol=0.0, ctx=f"{fn} {agg} vonly={vonly} v6={v6}")
            res[(vonly, v6, agg)] = got
    for agg in ["max", "min", "none"]:
        for m in modes[1:]:
            assert_groups_match(res[modes[0] + (agg,)], res[m + (agg,)], agg, tol=0.0, ctx=f"{fn} {agg} {m}")
