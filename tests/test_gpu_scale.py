"""GPU parity at the BASELINE configs' real sizes, and the load-time row index.

* k_index (vectorised, one pass, 8 datapoints per lane) against the sequential per-datapoint
  path it replaced (option INDEX_GENERIC = 1), row descriptor by row descriptor, over fuzzed
  cells of every class: 2-byte / 4-byte / mixed qualifiers, vle integers, float32 / float64,
  NaN / -0.0 / Inf, unsorted offsets, malformed lengths, short value arrays, long rows.
* BASELINE config 1 at its exact size (1k series x 1 day @10 s, vle integers, 24 rows per
  series, sum:1m-avg, one group) through the k_fast vle walker, against the oracle.
* BASELINE config 2 at full size (1M series x 1 h @1 s float32, 64 groups): 7.2 GB of
  qualifiers and 14.4 GB of values resident, so every blob offset above 2^31 and 2^32 is
  exercised (the regime of the round-1 sign-extension fault), against the oracle run with 16
  threads on the downloaded bytes.  Reference known answer this config scales:
  test/core/TestTsdbQueryDownsample.java:137-172 (single-series 1m-avg).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import get_option, set_option
from oracle import oracle as O
from tests.test_gpu_fast import assert_bit_equal
from tests.test_gpu_parity import assert_groups_match, T0

pytestmark = pytest.mark.gpu

ROW_QW_MASK, ROW_VL_MASK = 0x7, 0xF00
ROW_ERR, ROW_ALLF, ROW_NAN, ROW_NEGZ, ROW_UNSORTED, ROW_SFIRST, ROW_ALLI, ROW_VLE2 = (
    0x10000, 0x20000, 0x40000, 0x80000, 0x100000, 0x200000, 0x400000, 0x800000)


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def _with_generic(flag: bool):
    class Ctx:
        def __enter__(self):
            self.old = get_option("INDEX_GENERIC")
            set_option("INDEX_GENERIC", 1 if flag else 0)

        def __exit__(self, *a):
            set_option("INDEX_GENERIC", self.old)
    return Ctx()


def fuzz_batch(seed: int, n_series: int = 400):
    """Series of 1-3 hour rows of every cell class, then corruptions."""
    rng = np.random.default_rng(seed)
    series, gids = [], []
    for s in range(n_series):
        style = s % 9
        rows = []
        for h in range(int(rng.integers(1, 4))):
            n = int(rng.choice([1, 2, 7, 63, 64, 65, 360, 511, 512, 513, 1500, 3600]))
            if style == 8:
                n = min(n, 1800)
            ts = np.sort(rng.choice(3600 if style != 3 else 3_600_000, size=n, replace=False)).astype(np.int64)
            base = (T0 + 3600 * h) * 1000
            ts = base + (ts * 1000 if style != 3 else ts)
            ms = np.zeros(n, bool) if style != 3 else np.ones(n, bool)
            if style == 4:          # mixed second / millisecond qualifiers in one row
                ms = rng.random(n) < 0.5
                ts = np.where(ms, ts + rng.integers(1, 999, n), ts)
                ts = np.unique(ts)
                n = len(ts)
                ms = (ts % 1000) != 0
            kind = np.zeros(n, int)
            lv = np.zeros(n, np.int64)
            fv = np.zeros(n)
            if style == 0:          # float32
                kind[:] = 1
                fv = rng.normal(50, 10, n).astype(np.float32).astype(np.float64)
            elif style == 1:        # vle 1-2 byte ints
                lv = rng.integers(-300, 30000, n)
            elif style == 2:        # float64
                kind[:] = 2
                fv = rng.normal(0, 1e6, n)
            elif style == 3:        # ms qualifiers, mixed int sizes
                lv = rng.integers(-(1 << 40), 1 << 40, n) >> rng.integers(0, 40, n)
            elif style == 5:        # int / float mixed
                kind = rng.integers(0, 3, n)
                lv = rng.integers(-(1 << 20), 1 << 20, n)
                fv = rng.normal(0, 100, n)
            elif style == 6:        # special floats
                kind[:] = 1
                fv = rng.normal(0, 1, n).astype(np.float32).astype(np.float64)
                for spec in (np.nan, -0.0, np.inf, -np.inf):
                    if rng.random() < 0.5:
                        fv[int(rng.integers(0, n))] = spec
            elif style == 7:        # 8-byte ints
                lv = rng.integers(-(1 << 62), 1 << 62, n)
            else:                   # 4-byte ints
                lv = rng.integers(-(1 << 30), 1 << 30, n)
            rows += synth.encode_rows(ts, lv, fv, kind, ms)
        series.append(rows)
        gids.append(s % 5)
    b = synth.from_series(series, gids)
    qual, val = b.qual.copy(), b.val.copy()
    qo, vo = b.row_qual_off.astype(np.int64), b.row_val_off.astype(np.int64)
    nr = len(b.row_base_time)
    for r in rng.choice(nr, size=nr // 8, replace=False):
        q0, q1 = int(qo[r]), int(qo[r + 1])
        qw = 4 if (qual[q0] & 0xF0) == 0xF0 else 2
        nq = (q1 - q0) // qw
        c = int(rng.integers(0, 3))
        if c == 0 and nq >= 2:      # swap two qualifiers: unsorted offsets
            i = int(rng.integers(0, nq - 1))
            a = qual[q0 + i * qw:q0 + (i + 1) * qw].copy()
            qual[q0 + i * qw:q0 + (i + 1) * qw] = qual[q0 + (i + 1) * qw:q0 + (i + 2) * qw]
            qual[q0 + (i + 1) * qw:q0 + (i + 2) * qw] = a
        elif c == 1:                # illegal length (3-byte integer)
            i = int(rng.integers(0, nq))
            p = q0 + i * qw + qw - 1
            qual[p] = (qual[p] & 0xF0) | 0x2
        elif c == 2 and vo[r + 1] - vo[r] > 3:   # claim 8-byte values: runs past the value array
            i = int(rng.integers(0, nq))
            p = q0 + i * qw + qw - 1
            qual[p] = (qual[p] & 0xF0) | 0x7
    return abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, qual, val, b.group_id)


def rows_of(eng, batch, generic: bool):
    with _with_generic(generic):
        eng.load(batch)
    return eng.debug_rows(), eng.timing().index_ms


def assert_rows_equal(fast, gen, ctx):
    ndp_f, fl_f, lsb_f, am_f = fast
    ndp_g, fl_g, lsb_g, am_g = gen
    np.testing.assert_array_equal(ndp_f, ndp_g, err_msg=f"{ctx}: ndp")
    bad = (fl_g & ROW_ERR) != 0
    np.testing.assert_array_equal(fl_f & ROW_ERR, fl_g & ROW_ERR, err_msg=f"{ctx}: malformed rows")
    # malformed rows: the value statistics are never read (the row raises IllegalDataException)
    shape = ROW_QW_MASK | ROW_VL_MASK | ROW_ALLF | ROW_ALLI | ROW_VLE2 | ROW_UNSORTED | ROW_SFIRST
    np.testing.assert_array_equal(fl_f & shape, fl_g & shape, err_msg=f"{ctx}: row shape flags")
    ok = ~bad
    np.testing.assert_array_equal(fl_f[ok], fl_g[ok], err_msg=f"{ctx}: flags")
    np.testing.assert_array_equal(lsb_f[ok], lsb_g[ok], err_msg=f"{ctx}: lsb")
    np.testing.assert_array_equal(am_f[ok], am_g[ok], err_msg=f"{ctx}: absmax")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_index_fast_matches_generic_fuzz(eng, seed):
    b = fuzz_batch(seed)
    fast, _ = rows_of(eng, b, False)
    gen, _ = rows_of(eng, b, True)
    assert_rows_equal(fast, gen, f"fuzz {seed}")
    # every class is present
    qw = fast[1] & ROW_QW_MASK
    assert (qw == 2).any() and (qw == 4).any() and (qw == 0).any()
    assert ((fast[1] & ROW_ERR) != 0).any() and ((fast[1] & ROW_UNSORTED) != 0).any()


@pytest.mark.parametrize("args", [(3000, 3600, 1000, 0, 64, 1), (3000, 360, 10000, 2, 8, 30000),
                                  (1000, 8640, 10000, 1, 1, 2000), (500, 4000, 1500, 0, 4, 1)])
def test_index_fast_matches_generic_synth(eng, args):
    n, npts, period, kind, groups, mod = args
    b = synth.generate(n, T0, npts, period, value_kind=kind, n_groups=groups, int_mod=mod)
    fast, _ = rows_of(eng, b, False)
    gen, _ = rows_of(eng, b, True)
    assert_rows_equal(fast, gen, str(args))


def test_index_val2_matches_generic(eng):
    """The int16 value copy of vle rows (second k_index pass) read by k_short / k_fast:
    queries over it are bit-equal whichever index pass wrote it, and match the oracle."""
    b = synth.generate(2000, T0, 360, 10000, value_kind=2, n_groups=8, int_mod=30000, seed=5)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    with _with_generic(True):
        eng.load(b)
    gen = eng.run(q)
    with _with_generic(False):
        eng.load(b)
    fast = eng.run(q)
    assert eng.timing().fast_ms > 0 and eng.timing().redo_tiles == 0
    assert_bit_equal(fast, gen, "val2")
    assert_groups_match(fast, O.run_query(b, q), "sum", ctx="val2 vs oracle")


def test_config1_exact_size(eng):
    """BASELINE config 1 exactly: sum:1m-avg over 1000 series x 1 day @10 s (8.64e6 dp),
    vle integers hash % 2000, 24 hour rows per series, no group-by.  1441 output slots exceed
    the streaming kernel's LDS slot budget, so the general kernel runs it; the result matches
    the oracle within the cross-series float tolerance, the TSDB_QF_ORDERED fold bit for bit,
    and integer aggregates bit for bit."""
    eng.synth(1000, T0, 8640, 10000, 1, 1, 2000, 0x5EED)
    host = eng.download()
    assert len(host.row_base_time) == 24 * 1000
    q = abi.new_query(T0, T0 + 86400, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    got = eng.run(q)
    t = eng.timing()
    assert t.datapoints == 1000 * 8640
    want = O.run_query(host, q, threads=8)
    assert len(want) == 1 and len(want[0][1]) == 1440
    assert_groups_match(got, want, "sum", ctx="config1")
    qo = abi.new_query(T0, T0 + 86400, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000,
                       flags=abi.QF_ORDERED)
    assert_groups_match(eng.run(qo), want, "sum", tol=0.0, ctx="config1 ordered (bit-exact)")
    for agg in ["count", "max", "min"]:
        qa = abi.new_query(T0, T0 + 86400, agg, ds_function=abi.AGG["max"], ds_interval_ms=60000)
        assert_groups_match(eng.run(qa), O.run_query(host, qa, threads=8), agg, tol=0.0, ctx=f"config1 {agg}")


@pytest.mark.parametrize("interval", [600000, 1800000, 3600000])
def test_config1_data_streaming_vle_walker(eng, interval):
    """Config 1's data (24 vle-integer rows per series) at intervals whose slots fit the
    streaming kernel: every tile through k_fast's multi-row vle walker, none handed back,
    against the oracle (default tolerance and TSDB_QF_ORDERED bit-exact) and k_grid (bit-exact)."""
    from tests.test_gpu_fast import run_path
    eng.synth(1000, T0, 8640, 10000, 1, 1, 2000, 0x5EED)
    host = eng.download()
    q = abi.new_query(T0, T0 + 86400, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=interval)
    got, t = run_path(eng, None, q, True)
    assert t.fast_ms > 0 and t.redo_tiles == 0, (t.fast_ms, t.redo_tiles)
    gen, _ = run_path(eng, None, q, False)
    assert_bit_equal(got, gen, f"config1 data {interval}")
    want = O.run_query(host, q, threads=8)
    assert_groups_match(got, want, "sum", ctx=f"config1 data {interval}")
    qo = abi.new_query(T0, T0 + 86400, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=interval,
                       flags=abi.QF_ORDERED)
    assert_groups_match(eng.run(qo), want, "sum", tol=0.0, ctx=f"config1 data {interval} ordered")


def test_config2_full_size(eng):
    """BASELINE config 2 at full size: blobs of 7.2 GB (qualifiers) and 14.4 GB (values), so
    row offsets run far past 2^31 and 2^32; sum:1m-avg over 64 groups against the oracle."""
    eng.synth(1_000_000, T0, 3600, 1000, 0, 64, 1, 0x5EED)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    got = eng.run(q)
    t = eng.timing()
    assert t.datapoints == 3_600_000_000 and t.fast_ms > 0 and t.redo_tiles == 0
    qo = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000, flags=abi.QF_ORDERED)
    got_ordered = eng.run(qo)
    qm = abi.new_query(T0, T0 + 3599, "max", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    got_max = eng.run(qm)
    host = eng.download()
    assert int(host.row_qual_off[-1]) > (1 << 32) and int(host.row_val_off[-1]) > (1 << 33)
    want = O.run_query(host, q, threads=16)
    assert len(want) == 64 and all(len(w[1]) == 60 for w in want)
    assert_groups_match(got, want, "sum", ctx="config2 full")
    assert_groups_match(got_ordered, want, "sum", tol=0.0, ctx="config2 full ordered (bit-exact)")
    assert_groups_match(got_max, O.run_query(host, qm, threads=16), "max", ctx="config2 full max")


def empty_batch():
    return abi.HostBatch(np.zeros(1, np.int64), np.zeros(0, np.uint32), np.zeros(1, np.uint64), np.zeros(1, np.uint64),
                         np.zeros(0, np.uint8), np.zeros(0, np.uint8), np.zeros(0, np.int32))


@pytest.mark.parametrize("kind", ["empty", "out_of_range", "dropped"])
def test_empty_inputs_every_path(eng, kind):
    """No series, series entirely outside the scan range, and every series dropped (group -1):
    every path -- downsampled, percentile downsampling and group-by, ORDERED, NONE, raw union,
    raw percentile, rate -- returns what the oracle returns (no groups / inactive groups)."""
    if kind == "empty":
        b = empty_batch()
    else:
        b = synth.generate(12, T0 + (86400 if kind == "out_of_range" else 0), 360, 10000, value_kind=2, n_groups=3,
                           int_mod=30000)
        if kind == "dropped":
            b = abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, b.val,
                              np.full(b.n_series, -1, np.int32))
    queries = [
        ("sum", dict(ds_function=abi.AGG["avg"], ds_interval_ms=60000)),
        ("max", dict(ds_function=abi.AGG["p99"], ds_interval_ms=600000)),
        ("p95", dict(ds_function=abi.AGG["avg"], ds_interval_ms=60000)),
        ("sum", dict(ds_function=abi.AGG["avg"], ds_interval_ms=60000, flags=abi.QF_ORDERED)),
        ("none", dict(ds_function=abi.AGG["avg"], ds_interval_ms=60000)),
        ("sum", dict(ds_function=abi.AGG["sum"], ds_interval_ms=60000, ds_fill=abi.FILL_NAN)),
        ("sum", dict()),
        ("p99", dict()),
        ("none", dict()),
        ("sum", dict(rate=True, counter=True)),
    ]
    for agg, kw in queries:
        q = abi.new_query(T0, T0 + 3599, agg, **kw)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, tol=0.0, ctx=f"{kind} {agg} {kw}")
