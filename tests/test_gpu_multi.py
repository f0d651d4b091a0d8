"""tsdbhip_run_multi: several group-by aggregators over one downsampling (BASELINE config 3's
avg/min/max/count/dev "fused into one pass"): one decode + downsample pass,
then each query's SpanGroup step -- every result checked against the oracle run of that
query alone, with the usual tolerances."""
from __future__ import annotations

import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import get_option, set_option
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400
AGGS = ["sum", "avg", "min", "max", "count", "dev", "zimsum", "mimmax", "first", "last", "diff", "mult", "squareSum"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("shape", [(600, 360, 10000, 2), (40, 3600, 1000, 0), (30, 1440, 60000, 1)])
def test_multi_matches_single_queries(eng, shape):
    n, pts, period, kind = shape
    b = synth.generate(n, T0, pts, period, value_kind=kind, n_groups=7, int_mod=30000, seed=9)
    eng.load(b)
    end = T0 + pts * period // 1000 - 1
    qs = [abi.new_query(T0, end, a, ds_function=abi.AGG["avg"], ds_interval_ms=60000) for a in AGGS]
    got = eng.run_multi(qs)
    for a, q, g in zip(AGGS, qs, got):
        if a == "mult":
            continue   # products of hundreds of ~50 values overflow: checked on a small batch below
        assert_groups_match(g, O.run_query(b, q), a, ctx=f"{shape} {a}")


def test_multi_with_rate_fill_percentile_ordered(eng):
    b = synth.generate(50, T0, 720, 5000, value_kind=2, n_groups=3, int_mod=1000, seed=4)
    eng.load(b)
    qs = [abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["max"], ds_interval_ms=300000, ds_fill=abi.FILL_NAN),
          abi.new_query(T0, T0 + 3599, "avg", ds_function=abi.AGG["max"], ds_interval_ms=300000, ds_fill=abi.FILL_NAN,
                        rate=True),
          abi.new_query(T0, T0 + 3599, "p90", ds_function=abi.AGG["max"], ds_interval_ms=300000, ds_fill=abi.FILL_NAN),
          abi.new_query(T0, T0 + 3599, "dev", ds_function=abi.AGG["max"], ds_interval_ms=300000, ds_fill=abi.FILL_NAN,
                        flags=abi.QF_ORDERED),
          abi.new_query(T0, T0 + 3599, "mult", ds_function=abi.AGG["max"], ds_interval_ms=300000, ds_fill=abi.FILL_NAN),
          abi.new_query(T0, T0 + 3599, "min", ds_function=abi.AGG["max"], ds_interval_ms=300000, ds_fill=abi.FILL_NAN)]
    got = eng.run_multi(qs)
    for q, g, name, tol in zip(qs, got, ["sum", "avg", "p90", "dev", "mult", "min"], [None, None, 0.0, 0.0, None, None]):
        assert_groups_match(g, O.run_query(b, q), name, tol=tol, ctx=name)


def test_multi_percentile_downsampling(eng):
    b = synth.generate(40, T0, 8640, 10000, value_kind=0, n_groups=2, seed=6)
    eng.load(b)
    qs = [abi.new_query(T0, T0 + 86399, a, ds_function=abi.AGG["p99"], ds_interval_ms=3600000)
          for a in ["sum", "max", "count"]]
    for a, q, g in zip(["sum", "max", "count"], qs, eng.run_multi(qs)):
        assert_groups_match(g, O.run_query(b, q), a, ctx=a)


def test_multi_rejects_different_downsampling(eng):
    b = synth.generate(10, T0, 360, 10000, value_kind=0, n_groups=2, seed=6)
    eng.load(b)
    qs = [abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000),
          abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["max"], ds_interval_ms=60000)]
    with pytest.raises(Exception) as ei:
        eng.run_multi(qs)
    assert ei.value.java == "IllegalArgumentException"


# ---- the fused multi-aggregator pass (run_multi_fused, kcommon.h MultiReg) -------------------
FUSABLE = ["sum", "avg", "min", "max", "count", "dev"]


def run_separate(eng, qs):
    """The same queries with the fused pass switched off (one streaming pass per query)."""
    set_option("MULTI_FUSE", 0)
    try:
        return eng.run_multi(qs)
    finally:
        set_option("MULTI_FUSE", None)


def sparse_batch(seed, n_series=240, n_groups=5, span_s=3600, period_s=10):
    """Series with minutes-long gaps, late starts and early ends on a 10 s grid, int or float
    values: LERP between present buckets, slots before the first / after the last bucket."""
    import numpy as np
    rng = np.random.default_rng(seed)
    series, gids = [], []
    for s in range(n_series):
        grid = np.arange(0, span_s, period_s)
        keep = rng.random(len(grid)) < rng.uniform(0.05, 0.9)
        lo, hi = sorted(rng.integers(0, len(grid), 2))
        keep[:lo] = False
        keep[hi + 1:] = False
        for _ in range(int(rng.integers(0, 4))):     # whole missing minutes
            m = int(rng.integers(0, span_s // 60))
            keep[(grid >= m * 60) & (grid < m * 60 + 60)] = False
        if not keep.any():
            keep[int(rng.integers(0, len(grid)))] = True
        ts = (T0 + grid[keep]) * 1000
        n = len(ts)
        kind = np.zeros(n, int) if s % 2 == 0 else np.ones(n, int)
        lv = rng.integers(-5000, 30000, n)
        fv = np.round(rng.normal(50, 20, n), 3)
        series.append(synth.encode_rows(ts, lv, fv, kind, np.zeros(n, bool)))
        gids.append(s % n_groups)
    order = sorted(range(n_series), key=lambda i: gids[i])
    return synth.from_series([series[i] for i in order], [gids[i] for i in order])


def check_fused(eng, b, qs, ctx, expect_fused=True):
    from tests.test_gpu_fast import assert_bit_equal
    if b is not None:
        eng.load(b)
    got = eng.run_multi(qs)
    fused = eng.timing().fused_queries
    if expect_fused is not None:
        assert fused == (len(qs) if expect_fused else 0), f"{ctx}: fused_queries {fused}"
    sep = run_separate(eng, qs)
    assert eng.timing().fused_queries == 0
    host = b if b is not None else eng.download()
    for q, g, s in zip(qs, got, sep):
        name = abi.AGGREGATOR_NAMES[q.aggregator]
        assert_bit_equal(g, s, f"{ctx} {name}: fused vs separate passes")
        assert_groups_match(g, O.run_query(host, q), name, ctx=f"{ctx} {name}")


def fused_queries(end, ds="avg", interval=60000, fill=abi.FILL_NONE, aggs=FUSABLE, **kw):
    return [abi.new_query(T0, end, a, ds_function=abi.AGG[ds], ds_interval_ms=interval, ds_fill=fill, **kw)
            for a in aggs]


@pytest.mark.parametrize("shape", [(2000, 360, 10000, 2, 30000), (256, 3600, 1000, 0, 1), (300, 2400, 1500, 0, 1),
                                   (256, 360, 10000, 1, 2000)])
def test_fused_multi_dense_shapes(eng, shape):
    """Config 3's shape (k_short, int and float classes), config 2's (k_fast walker), ms
    qualifiers, vle integers."""
    n, pts, period, kind, mod = shape
    b = synth.generate(n, T0, pts, period, value_kind=kind, n_groups=16, int_mod=mod, seed=5)
    end = T0 + pts * period // 1000 - 1
    check_fused(eng, b, fused_queries(end), f"dense {shape}")


@pytest.mark.parametrize("ds", ["avg", "sum", "count", "min", "max", "squareSum"])
def test_fused_multi_sparse_interpolation(eng, ds):
    """Missing buckets: avg/min/max/dev/sum interpolate (LERP), count reads 0.0 (ZIM).  Sums of
    squares of 3-decimal values rarely pass the exactness certificate: those tiles are handed
    back and the queries run one by one (either way the results are the separate passes')."""
    check_fused(eng, sparse_batch(3), fused_queries(T0 + 3599, ds=ds), f"sparse {ds}",
                expect_fused=None if ds == "squareSum" else True)


@pytest.mark.parametrize("fill", [abi.FILL_ZERO, abi.FILL_NAN, abi.FILL_NULL])
def test_fused_multi_fill(eng, fill):
    check_fused(eng, sparse_batch(4), fused_queries(T0 + 3599, ds="max", interval=120000, fill=fill),
                f"fill {fill}")


def test_fused_multi_windows_and_all(eng):
    b = sparse_batch(5)
    check_fused(eng, b, [abi.new_query(T0 + 700, T0 + 2900, a, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
                         for a in FUSABLE], "window")
    # "all" runs on the general kernel only: one pass per query
    check_fused(eng, None, [abi.new_query(T0 + 100, T0 + 3000, a, ds_function=abi.AGG["sum"], ds_all=True)
                            for a in FUSABLE], "0all", expect_fused=False)


def test_fused_multi_subsets_and_duplicates(eng):
    b = synth.generate(500, T0, 360, 10000, value_kind=2, n_groups=9, int_mod=30000, seed=8)
    check_fused(eng, b, fused_queries(T0 + 3599, aggs=["count", "dev"]), "count+dev")
    check_fused(eng, None, fused_queries(T0 + 3599, aggs=["max", "max", "avg", "min", "sum"]), "duplicates")


def test_fused_multi_falls_back(eng):
    """Queries or tiles the fused pass does not take run one pass each, with the same results:
    a rate query, an aggregator outside the fused set, K > 64, and NaN rows (handed back)."""
    b = synth.generate(300, T0, 360, 10000, value_kind=2, n_groups=4, int_mod=30000, seed=2)
    check_fused(eng, b, fused_queries(T0 + 3599) + [abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"],
                                                                  ds_interval_ms=60000, rate=True)],
                "rate", expect_fused=False)
    check_fused(eng, None, fused_queries(T0 + 3599, aggs=["sum", "zimsum"]), "zimsum", expect_fused=False)
    check_fused(eng, None, fused_queries(T0 + 3599, interval=30000, aggs=["sum", "avg"]), "K=120", expect_fused=False)
    import numpy as np
    val = b.val.copy()
    # the first series whose row holds float32 values (2-byte qualifier flags 0xB)
    s = next(i for i in range(b.n_series) if b.qual[int(b.row_qual_off[b.series_row_ptr[i]]) + 1] & 0xF == 0xB)
    off = int(b.row_val_off[b.series_row_ptr[s]]) + 4 * 10
    val[off:off + 4] = np.frombuffer(np.array([np.nan], ">f4").tobytes(), np.uint8)
    nb = abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, val, b.group_id)
    check_fused(eng, nb, fused_queries(T0 + 3599), "nan row", expect_fused=False)
