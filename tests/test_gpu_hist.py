"""Histogram path on the MI355X: libtsdbhip's k_hist kernels through the C
ABI (tsdbhip_load_histograms / tsdbhip_hist_run) against the oracle (oracle/refhist.c) and the
reference's own known answers (tests/golden/histogram.json).  Bit-exact: timestamps, percentile
values (SimpleHistogram.percentile's int arithmetic and float bucket midpoints, the long codec's
data * p) and bucket counts."""
from __future__ import annotations

import zlib

import numpy as np
import pytest

from opentsdb_amd import abi
from opentsdb_amd.engine import get_option, set_option
from opentsdb_amd import histogram as H
from opentsdb_amd.engine import Engine, EngineError
from oracle import oracle as O
from tests import hist_util as U

pytestmark = pytest.mark.gpu

G = U.golden()
T0 = 1356998400


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("gq", G["queries"], ids=[q["name"] for q in G["queries"]])
def test_gpu_golden_queries(eng, gq):
    hb = U.store_batch(G["stores"][gq["store"]])
    eng.load_histograms(hb)
    q = U.golden_query(gq)
    got = eng.run_histogram(q, gq["percentiles"], gq["show_buckets"], gq["span_range"])
    U.check_golden(got, gq)
    U.same(got, O.run_hist(hb, q, gq["percentiles"], gq["show_buckets"], gq["span_range"]), gq["name"])


QUERIES = [
    ("raw-sum", dict(agg="sum", ds=None)),
    ("raw-none", dict(agg="none", ds=None)),
    ("10s-sum", dict(agg="sum", ds="10s-sum")),
    ("1m-sum", dict(agg="sum", ds="1m-sum")),
    ("7m-sum", dict(agg="sum", ds="7m-sum")),
    ("1h-sum", dict(agg="sum", ds="1h-sum")),
    ("1m-sum-none", dict(agg="none", ds="1m-sum")),
    ("1m-p99-groupby", dict(agg="p99", ds="1m-sum")),
]
PCTS = [50.0, 95.0, 99.9, 1.0, 100.0, 0.5, 150.0]


def run_both(eng, hb, q, pcts, buckets, span_range=None):
    eng.load_histograms(hb)
    try:
        want = O.run_hist(hb, q, pcts, buckets, span_range)
    except O.OracleError as e:
        with pytest.raises(EngineError) as ee:
            eng.run_histogram(q, pcts, buckets, span_range)
        return e.code, ee.value.code
    got = eng.run_histogram(q, pcts, buckets, span_range)
    U.same(got, want)
    return got


@pytest.mark.parametrize("name,kw", QUERIES, ids=[n for n, _ in QUERIES])
@pytest.mark.parametrize("buckets", [False, True])
def test_gpu_random_simple(eng, name, kw, buckets):
    rng = np.random.default_rng(zlib.crc32(name.encode()) % 1000 + 17 * buckets)
    hb = U.random_store(rng, n_series=7, n_rows=3, period_ms=10000, groups=3, layouts=3)
    got = run_both(eng, hb, U.query(T0 + 600, T0 + 3 * 3600 - 900, kw["agg"], kw["ds"]), PCTS, buckets)
    assert isinstance(got, list) and sum(len(g[0].ts) for g in got) > 0


@pytest.mark.parametrize("seed", range(6))
def test_gpu_random_wild_buckets_and_counts(eng, seed):
    """NaN / +-inf / -0.0 bucket bounds (Float.compare order, canonical NaN keys), overlapping
    buckets, counts above 2^31 and negative (intValue wrap in percentile, long sums), columns
    holding a subset of their series' layout."""
    rng = np.random.default_rng(100 + seed)
    hb = U.random_store(rng, n_series=5, n_rows=2, period_ms=20000, groups=2, layouts=4, wild=True,
                        big_counts=seed % 2 == 1)
    for ds in (None, "1m-sum"):
        run_both(eng, hb, U.query(T0, T0 + 2 * 3600, "sum", ds), PCTS, True)


@pytest.mark.parametrize("seed", range(3))
def test_gpu_malformed_columns_dropped(eng, seed):
    rng = np.random.default_rng(200 + seed)
    hb = U.random_store(rng, n_series=6, n_rows=2, period_ms=15000, groups=2, bad_frac=0.3)
    for ds in (None, "1m-sum", "0all-sum"):
        run_both(eng, hb, U.query(T0, T0 + 7200, "sum", ds), [50.0, 99.0], True)


def test_gpu_long_codec_and_mixed_codecs(eng):
    rng = np.random.default_rng(7)
    # one codec per group (series s is in group s % 2; even series long): no mixing
    hb = U.random_store(rng, n_series=6, n_rows=2, period_ms=10000, groups=2, long_frac=0.0)
    run_both(eng, hb, U.query(T0, T0 + 7200, "sum", "1m-sum"), [0.98, 50.0], True)
    hb = U.random_store(rng, n_series=6, n_rows=2, period_ms=10000, groups=2, long_frac=1.0)
    run_both(eng, hb, U.query(T0, T0 + 7200, "sum", "1m-sum"), [0.98, 50.0], True)
    # codecs mixed inside a group: the reference's aggregate throws (ClassCastException or
    # IllegalArgumentException by receiver); the engine raises IllegalArgumentException
    hb = U.random_store(rng, n_series=8, n_rows=1, period_ms=10000, groups=1, long_frac=0.5)
    r = run_both(eng, hb, U.query(T0, T0 + 3600, "sum", "1m-sum"), [50.0], False)
    if isinstance(r, tuple):
        assert r[0] in (-9, -3) and r[1] == -3


def test_gpu_nonsum_downsampling_null_pointer(eng):
    rng = np.random.default_rng(8)
    hb = U.random_store(rng, n_series=3, n_rows=1, period_ms=10000, sparse=0.0, ms_frac=0.0)
    r = run_both(eng, hb, U.query(T0, T0 + 3600, "sum", "1m-avg"), [50.0], False)
    assert r == (-10, -10)
    run_both(eng, hb, U.query(T0, T0 + 3600, "sum", "10s-max"), [50.0], False)   # one point per interval


def test_gpu_all_downsampling_ms_query(eng):
    """0all with millisecond query bounds (the downsampler's query start / end are TsdbQuery's as
    set): one point per group at the query end (the clone's timestamp)."""
    rng = np.random.default_rng(9)
    hb = U.random_store(rng, n_series=5, n_rows=3, period_ms=10000, groups=2)
    got = run_both(eng, hb, U.query((T0 + 1000) * 1000, (T0 + 9000) * 1000, "sum", "0all-sum"), [50.0, 99.0], True)
    assert [list(g[0].ts) for g in got] == [[(T0 + 9000) * 1000]] * 2
    # seconds: the "all" filter compares ms timestamps with second bounds -- nothing (reference quirk)
    got = run_both(eng, hb, U.query(T0 + 1000, T0 + 9000, "sum", "0all-sum"), [50.0], False)
    assert all(len(g[0].ts) == 0 for g in got)


def test_gpu_duplicate_row_keys_merge(eng):
    """HistogramSpan.addRow: a row whose key repeats with overlapping timestamps merges into the
    existing HistogramRowSeq (the earlier point kept on a tie, HistogramRowSeq.addRow :66-105)."""
    a = [(bytes([6]) + int.to_bytes(t, 2, "big"), U.encode_simple(0, [((1.0, 2.0), t)], 0, 0)) for t in range(0, 3600, 60)]
    b = [(bytes([6]) + int.to_bytes(t, 2, "big"), U.encode_simple(0, [((1.0, 2.0), 1000 + t)], 0, 0))
         for t in range(30, 3600, 120)]
    c = [(bytes([6]) + int.to_bytes(t, 2, "big"), U.encode_simple(0, [((2.0, 3.0), 7)], 0, 0)) for t in range(0, 3600, 600)]
    hb = H.HostHistBatch.from_rows([[(T0, a), (T0 + 3600, a), (T0, b), (T0, c)]], [0], {0: H.HCODEC_SIMPLE})
    for ds in (None, "5m-sum"):
        run_both(eng, hb, U.query(T0, T0 + 7200, "sum", ds), [50.0], True)


def test_gpu_unsorted_row_matches(eng):
    """Mixed second / millisecond qualifiers in one row are iterated in column order
    (HistogramRowSeq does not sort): the raw group-by then follows the aggregation iterator's
    greedy walk (HistogramAggregationIterator.next :240-292, k_hist_walk)."""
    cols = [(bytes([6, 0, 10]), U.encode_simple(0, [((1.0, 2.0), 1)], 0, 0)),
            (bytes([6, 0, 0, 0x13, 0x88]), U.encode_simple(0, [((1.0, 2.0), 2)], 0, 0)),   # 5000 ms
            (bytes([6, 0, 20]), U.encode_simple(0, [((1.0, 2.0), 4)], 0, 0))]
    hb = H.HostHistBatch.from_rows([[(T0, cols)]], [0], {0: H.HCODEC_SIMPLE})
    eng.load_histograms(hb)
    for ds in (None, "1m-sum"):
        q = U.query(T0, T0 + 3600, "sum", ds)
        U.same(eng.run_histogram(q, [50.0], True), O.run_hist(hb, q, [50.0], True))


def _shuffled_rows(hb_rows, rng, frac):
    return [[(base, [cols[i] for i in rng.permutation(len(cols))] if rng.random() < frac else cols)
             for base, cols in rows] for rows in hb_rows]


@pytest.mark.parametrize("seed", [31, 32, 33])
def test_gpu_raw_spans_out_of_order_walk(eng, seed):
    """Raw (no downsampler) group-by over spans some of whose rows hold their columns out of time
    order: the greedy walk across the group's spans -- repeated and receding timestamps, points of
    several spans merged only when they are current together -- against the oracle's literal
    iterator, for sum and none, with queries that cut the spans at both ends."""
    rng = np.random.default_rng(seed)
    series = []
    for s in range(7):
        rows = []
        for r in range(2):
            cols = []
            for off in rng.choice(3600, size=int(rng.integers(3, 40)), replace=False):
                ms = rng.random() < 0.3
                q = bytes([6]) + (int(off) * 1000 + int(rng.integers(0, 999))).to_bytes(4, "big") if ms else \
                    bytes([6]) + int(off).to_bytes(2, "big")
                cols.append((q, U.encode_simple(0, [((1.0, 2.0), int(rng.integers(0, 9))),
                                                    ((2.0, 4.0), int(rng.integers(0, 9)))], 0, int(rng.integers(0, 3)))))
            cols.sort(key=lambda c: c[0])            # HBase's qualifier-byte order: s / ms mixed out of time order
            rows.append((T0 + 3600 * r, cols))
        series.append(rows)
    series = _shuffled_rows(series, rng, 0.3)        # and some rows in no order at all
    hb = H.HostHistBatch.from_rows(series, [s % 3 for s in range(7)], {0: H.HCODEC_SIMPLE})
    for agg in ("sum", "none"):
        for t0, t1 in ((T0, T0 + 7200), (T0 + 600, T0 + 5000)):
            run_both(eng, hb, U.query(t0, t1, agg, None), [50.0, 95.0], True)


def test_gpu_group_filter_and_empty(eng):
    """Spans without a group-by tag (-1) drop out; NONE keeps them; empty store."""
    rng = np.random.default_rng(11)
    hb = U.random_store(rng, n_series=4, n_rows=1, period_ms=30000, groups=2)
    hb.group_id[1] = -1
    for agg in ("sum", "none"):
        run_both(eng, hb, U.query(T0, T0 + 3600, agg, "1m-sum"), [50.0], True)
    empty = H.HostHistBatch.from_rows([], [], {0: H.HCODEC_SIMPLE})
    assert run_both(eng, empty, U.query(T0, T0 + 3600, "sum", None), [50.0], True) == []


def test_gpu_larger_store(eng):
    """100 series x 2 h @ 5 s of 20-bucket histograms (144k columns), 8 groups."""
    rng = np.random.default_rng(12)
    hb = U.random_store(rng, n_series=100, n_rows=2, period_ms=5000, groups=8, layouts=5, nb=(18, 22),
                        sparse=0.05, ms_frac=0.0)
    for ds in ("1m-sum", "15m-sum", None):
        run_both(eng, hb, U.query(T0, T0 + 2 * 3600, "sum", ds), [50.0, 90.0, 99.0], ds == "15m-sum")


@pytest.mark.parametrize("layouts,nb", [(70, (8, 14)), (2, (40, 60))], ids=["dict-over-lds", "wide-columns"])
def test_gpu_accum_fallback_paths(eng, layouts, nb):
    """k_hist_accum's other paths: a dictionary larger than its LDS table (> 512 buckets: global
    hash lookups) and tiles whose columns overflow the 32 KB LDS stage (parsed from global)."""
    rng = np.random.default_rng(300 + layouts)
    hb = U.random_store(rng, n_series=layouts, n_rows=1, period_ms=20000, groups=3, layouts=layouts, nb=nb,
                        ms_frac=0.0)
    for ds in (None, "2m-sum"):
        run_both(eng, hb, U.query(T0, T0 + 3600, "sum", ds), [50.0, 99.0], True)


def raw_simple(buckets, under=0, over=0, codec_id=0):
    """A stored SimpleHistogram column written bucket by bucket in the given order (duplicates
    and out-of-order keys included), as a foreign writer could store it."""
    import struct
    out = bytearray([codec_id]) + struct.pack(">h", len(buckets))
    for lo, up, cnt in buckets:
        out += struct.pack(">ff", lo, up) + H.kryo_varlong(cnt)
    return bytes(out + H.kryo_varlong(under) + H.kryo_varlong(over))


def test_gpu_repeated_bucket_keys_last_count_wins(eng):
    """fromHistogram's TreeMap.put (src/core/SimpleHistogram.java:110-113): a key repeated inside
    one column keeps its LAST count; columns with keys out of order still aggregate by key."""
    cols = [
        raw_simple([(0.0, 1.0, 5), (1.0, 2.0, 7), (0.0, 1.0, 11)], 1, 2),           # (0,1) -> 11
        raw_simple([(1.0, 2.0, 3), (0.0, 1.0, 4)], 0, 1),                          # out of order
        raw_simple([(-0.0, 1.0, 2), (0.0, 1.0, 9), (-0.0, 1.0, 6), (5.0, 6.0, 1)]),  # -0.0 != 0.0
        raw_simple([(0.0, 1.0, 1), (0.0, 1.0, 2), (0.0, 1.0, 3), (0.0, 1.0, 4)]),   # -> 4
    ]
    series = []
    for s in range(2):
        rows = []
        for r in range(2):
            base = T0 + r * 3600
            cells = []
            for k in range(6):
                _, q = H.histogram_qualifier(base + 10 * k + s)
                cells.append((q, cols[(k + r + s) % len(cols)]))
            rows.append((base, cells))
        series.append(rows)
    hb = H.HostHistBatch.from_rows(series, [0, 0], {0: H.HCODEC_SIMPLE})
    for ds in (None, "1m-sum", "1h-sum"):
        run_both(eng, hb, U.query(T0, T0 + 2 * 3600, "sum", ds), [50.0, 90.0, 10.0], True)


@pytest.mark.parametrize("env", [{"HIST_WINDOW": 0}, {"HIST_WS": 1}, {"HIST_WS": 5}, {"HIST_WS": 64},
                                 {"HIST_LAYOUT": 0}],
                         ids=["atomic-kernel", "ws1", "ws5", "ws64", "keyed"])
def test_gpu_accum_window_sizes(eng, env):
    """k_hist_accw keeps a window of consecutive points' counters in LDS; tiles whose points leave
    it flush it, points past its end add to the global counters directly.  Windows of 1, 5 and 64
    points, every bucket through the keyed lookup (no layout table) and the per-column atomic
    kernel give the oracle's answers, raw unions included (developer options)."""
    rng = np.random.default_rng(77)
    hb = U.random_store(rng, n_series=40, n_rows=2, period_ms=5000, groups=5, layouts=4, nb=(10, 16),
                        sparse=0.1, ms_frac=0.2)
    for k, v in env.items():
        set_option(k, v)
    try:
        for agg, ds, b in (("sum", "1m-sum", True), ("sum", None, True), ("none", "2m-sum", False),
                           ("p99", "30s-sum", False), ("sum", "0all-sum", True)):
            run_both(eng, hb, U.query(T0 + 100, T0 + 2 * 3600 - 50, agg, ds), [50.0, 95.0, 99.9], b)
    finally:
        for k in env:
            set_option(k, None)


T_DST = 1457740800   # 2016-03-12 00:00 UTC: America/Denver enters daylight time on Mar 13


@pytest.fixture(scope="module")
def dst_store():
    rng = np.random.default_rng(4242)
    return U.random_store(rng, n_series=9, n_rows=80, period_ms=600000, t0=T_DST, groups=3, layouts=3, nb=(4, 9),
                          sparse=0.15, ms_frac=0.0)


@pytest.mark.parametrize("tz", [None, "America/Denver", "Asia/Kabul"])
@pytest.mark.parametrize("spec", ["1dc-sum", "6hc-sum", "1wc-sum", "1nc-sum", "2dc-sum", "90mc-sum", "7sc-sum",
                                  "1hc-avg"])
def test_gpu_calendar_downsampling(eng, dst_store, tz, spec):
    """HistogramDownsampler with calendar intervals (src/core/HistogramDownsampler.java:219-331):
    intervals from DateTime.previousInterval of each span's first datapoint after the seek, in the
    query's zone, stepped by the calendar unit; the spans' outputs merge over the union of their
    timestamps.  7sc / 2dc / 90mc anchor per span; 1hc-avg over two datapoints raises as the
    reference's null HistogramAggregation does."""
    from opentsdb_amd import tz as T
    zone = T.table(tz) if tz else None
    for agg in ("sum", "none"):
        q = abi.new_query(T_DST + 1800, T_DST + 3 * 86400 + 600, agg, tz=zone)
        d = U.query(0, 1, agg, spec)
        q.ds_function, q.ds_interval_ms, q.ds_all, q.ds_calendar, q.ds_fill = (d.ds_function, d.ds_interval_ms,
                                                                               d.ds_all, d.ds_calendar, d.ds_fill)
        run_both(eng, dst_store, q, [50.0, 99.0], agg == "sum")


@pytest.mark.parametrize("n_dev", [2, 3])
def test_gpu_multi_device_context_runs_histograms(eng, n_dev):
    """A multi-device context (tsdbhip_init_devices; the one-GPU box repeats device 0) shards the
    histogram spans by whole groups over its devices (multi.cpp md_load_histograms): the same
    answers as one device and the oracle, for golden and random stores -- group-by and "none"
    (spans in batch order), per-device bucket dictionaries merged (wild bounds, show_buckets),
    ungrouped spans, more devices than groups."""
    md = Engine(devices=[0] * n_dev)
    try:
        for gq in G["queries"][:6]:
            hb = U.store_batch(G["stores"][gq["store"]])
            md.load_histograms(hb)
            q = U.golden_query(gq)
            got = md.run_histogram(q, gq["percentiles"], gq["show_buckets"], gq["span_range"])
            U.check_golden(got, gq)
        rng = np.random.default_rng(31)
        hb = U.random_store(rng, n_series=20, n_rows=2, period_ms=10000, groups=4, layouts=3)
        for agg, ds in [("sum", "1m-sum"), ("none", None), ("p99", "5m-sum")]:
            q = U.query(T0, T0 + 2 * 3600, agg, ds)
            got = run_both(md, hb, q, PCTS, True)
            U.same(got, run_both(eng, hb, q, PCTS, True))
        for seed in range(3):   # wild bucket bounds: each device's dictionary differs
            rng = np.random.default_rng(500 + seed)
            hb = U.random_store(rng, n_series=9, n_rows=2, period_ms=20000, groups=5, layouts=4, wild=True,
                                big_counts=seed == 1)
            hb.group_id[::4] = -1   # ungrouped spans: dropped by a group-by, their own group under "none"
            for agg, ds in [("sum", None), ("none", "1m-sum"), ("sum", "0all-sum")]:
                q = U.query(T0, T0 + 2 * 3600, agg, ds)
                got = run_both(md, hb, q, PCTS, True)
                U.same(got, run_both(eng, hb, q, PCTS, True))
        hb = U.random_store(np.random.default_rng(9), n_series=2, n_rows=2, period_ms=10000, groups=1, layouts=2)
        q = U.query(T0, T0 + 2 * 3600, "sum", "1m-sum")   # one group: the other devices hold nothing
        U.same(run_both(md, hb, q, PCTS, True), run_both(eng, hb, q, PCTS, True))
    finally:
        md.close()
