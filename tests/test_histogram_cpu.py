"""Histogram path on the CPU: the oracle (oracle/refhist.c) against the
reference's own known answers (tests/golden/histogram.json, transcribed by
tests/golden/make_histogram_golden.py), the host helpers of opentsdb_amd.histogram (the Kryo
encoder, qualifiers, the bucket adaptor's TreeMap lookups) and the C ABI's histogram symbols."""
from __future__ import annotations

import struct

import numpy as np
import pytest

from opentsdb_amd import histogram as H
from oracle import oracle as O
from tests import hist_util as U

G = U.golden()


@pytest.mark.parametrize("case", G["values"], ids=[c["name"] for c in G["values"]])
def test_oracle_value_known_answers(case):
    got = O.hist_value_percentile(bytes.fromhex(case["value"]), case["kind"], case["p"])
    assert got == case["expect"]


@pytest.mark.parametrize("gq", G["queries"], ids=[q["name"] for q in G["queries"]])
def test_oracle_query_known_answers(gq):
    hb = U.store_batch(G["stores"][gq["store"]])
    got = O.run_hist(hb, U.golden_query(gq), gq["percentiles"], gq["show_buckets"], gq["span_range"])
    U.check_golden(got, gq)


def test_encoder_matches_the_tests_kryo_bytes():
    """SimpleHistogram.histogram(true) of testToFromBytes' histogram (TestSimpleHistogram.java:130-168)
    round-trips: the fixture bytes of testPercentileList are what the encoder writes."""
    h = H.SimpleHistogram(0)
    for lo, up, c in [(1.0, 6.0, 5), (6.0, 10.0, 10), (10.0, 20.0, 1), (20.0, 40.0, 0)]:
        h.addBucket(lo, up, c)
    h.overflow = 5
    assert h.histogram(True).hex() == next(v["value"] for v in G["values"] if v["name"] == "testPercentileList p50")


@pytest.mark.parametrize("v", [0, 1, 127, 128, 300, 1 << 35, (1 << 56) - 1, 1 << 56, (1 << 63) - 1, -1, -(1 << 40)])
def test_kryo_varlong_lengths(v):
    b = H.kryo_varlong(v)
    u = v & 0xFFFFFFFFFFFFFFFF
    expect_len = next((n for n in range(1, 9) if u >> (7 * n) == 0), 9)
    assert len(b) == expect_len
    # decode as Kryo Input.readLong(true)
    r = 0
    for j, x in enumerate(b[:8]):
        r |= (x & 0x7F) << (7 * j)
        if not x & 0x80:
            break
    else:
        r |= b[8] << 56
    assert r == u


def test_histogram_qualifier():
    """Internal.getQualifier(ts, 0x06) (src/core/Internal.java:1027-1049)."""
    assert H.histogram_qualifier(1356998430) == (1356998400, bytes([6, 0, 30]))
    assert H.histogram_qualifier(1356998400500) == (1356998400, bytes([6, 0, 0, 1, 0xF4]))


def test_initialize_histogram_bucket_counts():
    """SimpleHistogram.initializeHistogram known answers (TestSimpleHistogram.java:543-592)."""
    assert len(H.SimpleHistogram.initializeHistogram(1.0, 6000.0, 100.0, 2000.0, 0.05)) == 33
    assert len(H.SimpleHistogram.initializeHistogram(100.0, 2000.0, 100.0, 2000.0, 0.05)) == 31
    assert len(H.SimpleHistogram.initializeHistogram(100.0, 6000.0, 100.0, 2000.0, 0.05)) == 32
    assert len(H.SimpleHistogram.initializeHistogram(1.0, 2000.0, 100.0, 2000.0, 0.05)) == 32
    for bad in [(10000.0, 6000.0, 100.0, 2000.0, 0.05), (1.0, 6000.0, 3000.0, 2000.0, 0.05),
                (1.0, 6000.0, 100.0, 2000.0, -0.05), (1.0, 1000.0, 100.0, 2000.0, 0.05),
                (200.0, 100.0, 1500.0, 2000.0, 0.05), (100.0, 6000.0, 100.0, 6000.0, 0.01)]:
        with pytest.raises(ValueError):
            H.SimpleHistogram.initializeHistogram(*bad)


def _two_point_store(first_buckets, second_buckets, under=(7, 300), over=(9, 10)):
    # (an underflow of 300 is a 2-byte varint: an empty histogram is then 6 bytes and decodes)
    """One span, two points (1 s apart) with the given regular buckets."""
    t = 1356998400
    cols = [(bytes([6, 0, 0]), U.encode_simple(0, [((lo, up), c) for lo, up, c in first_buckets], under[0], over[0])),
            (bytes([6, 0, 1]), U.encode_simple(0, [((lo, up), c) for lo, up, c in second_buckets], under[1], over[1]))]
    return H.HostHistBatch.from_rows([[(t, cols)]], [0], {0: H.HCODEC_SIMPLE})


@pytest.mark.parametrize("second", [
    [(1.0, 2.0, 5), (3.0, 4.0, 6)],          # (0, 0) absent, below every bucket: the UNDERFLOW leaf
    [(-3.0, -2.0, 5), (-1.0, -0.5, 6)],      # above every bucket: the OVERFLOW leaf
    [(-3.0, -2.0, 5), (3.0, 4.0, 6)],        # between: not found
    [],                                       # no regular bucket: the UNDERFLOW root
    [(0.0, 0.0, 11), (3.0, 4.0, 6)],         # present
    [(-0.0, 0.0, 11)],                        # -0.0 lower bound: another key
])
def test_bucket_adaptor_zero_key_lookup_matches_treemap(second):
    """HistogramBucketDataPointsAdaptor looks the first point's buckets up in every point's
    getHistogramBucketsIfHas TreeMap, whose HistogramBucket.compareTo treats REGULAR (+0.0, +0.0)
    as equal to UNDERFLOW / OVERFLOW: the oracle restates java.util.TreeMap's red-black tree,
    opentsdb_amd.histogram.bucket_value the closed form the GPU results go through."""
    hb = _two_point_store([(0.0, 0.0, 3), (1.0, 2.0, 4)], second)
    q = U.query(1356998400, 1356998460)
    want = O.run_hist(hb, q, [], True)
    series = {tuple(s.bucket): list(s.values) for s in want[0]}
    zero = series[(H.BK_REG, 0, 0)]
    counts = {(H._fcmp_key(H.f32bits(lo)), H._fcmp_key(H.f32bits(up))): c for lo, up, c in second}
    got = H.bucket_value((H.BK_REG, 0, 0), sorted(counts), counts, 300, 10)
    assert zero == [3, got]


def test_library_exports_histogram_symbols():
    from opentsdb_amd import engine as E
    L = E.lib()
    for s in ("tsdbhip_load_histograms", "tsdbhip_hist_run", "tsdbhip_hist_run_range", "tsdbhip_hist_result_free"):
        assert hasattr(L, s)


def test_oracle_drops_malformed_columns_and_keeps_valid_ones():
    """SaltScanner.processRow drops a column whose decode throws (:771-778): truncated values,
    unknown codec ids, empty values and non-histogram qualifier lengths."""
    rng = np.random.default_rng(5)
    hb = U.random_store(rng, n_series=3, n_rows=1, period_ms=60000, bad_frac=0.5, sparse=0.0, ms_frac=0.0)
    got = O.run_hist(hb, U.query(1356998400, 1357002000), [50.0], False)
    n = sum(len(g[0].ts) for g in got)
    assert 0 < n < 3 * 60


def test_oracle_nonsum_downsampling_raises_null_pointer():
    rng = np.random.default_rng(6)
    hb = U.random_store(rng, n_series=2, n_rows=1, period_ms=10000, sparse=0.0, ms_frac=0.0)
    with pytest.raises(O.OracleError) as e:
        O.run_hist(hb, U.query(1356998400, 1357002000, ds="1m-avg"), [50.0], False)
    assert e.value.code == -10
    # one datapoint per interval: no aggregation, no exception
    O.run_hist(hb, U.query(1356998400, 1357002000, ds="10s-avg"), [50.0], False)


def test_percentile_struct_pack_roundtrip():
    assert struct.unpack(">f", struct.pack(">I", H.f32bits(0.98)))[0] == np.float32(0.98)


def _loop_bucket_series(lo, up, cnt, pres, kind, a, b):
    """The per-point, per-bucket loop over bucket_value (the closed form's definition)."""
    D = len(lo)
    first = [d for d in range(D) if pres[a, d]]
    keys = [(H.BK_UNDER, 0, 0)] + [(H.BK_REG, lo[d], up[d]) for d in first] + [(H.BK_OVER, 0, 0)]
    vals = np.zeros((len(keys), b - a), np.int64)
    for i in range(a, b):
        if kind[i] != H.HCODEC_SIMPLE:
            continue
        counts = {(H._fcmp_key(lo[d]), H._fcmp_key(up[d])): int(cnt[i, d]) for d in range(D) if pres[i, d]}
        regs = sorted(counts)
        for k, key in enumerate(keys):
            vals[k, i - a] = H.bucket_value(key, regs, counts, int(cnt[i, D]), int(cnt[i, D + 1]))
    return keys, vals


@pytest.mark.parametrize("seed", range(6))
def test_bucket_series_vectorised_matches_loop(seed):
    """result_to_series builds every bucket series with array operations; it must equal the
    per-point bucket_value loop, (+0.0, +0.0) lookups and non-simple points included."""
    import ctypes as C
    rng = np.random.default_rng(seed)
    bounds = [0.0, -0.0, 1.0, 2.0, -3.0, 5.5, 1e9]
    pairs = [(H.f32bits(x), H.f32bits(y)) for x in bounds for y in bounds if x <= y]
    pairs = list(dict.fromkeys(pairs))
    D = len(pairs)
    n_groups = 4
    sizes = rng.integers(1, 12, n_groups)
    n_all = int(sizes.sum())
    gptr = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    pres = (rng.random((n_all, D)) < 0.3).astype(np.uint8)
    cnt = rng.integers(0, 1000, (n_all, D + 2)).astype(np.int64)
    kind = np.where(rng.random(n_all) < 0.9, H.HCODEC_SIMPLE, H.HCODEC_SIMPLE + 1).astype(np.uint8)
    kind[gptr[:-1]] = H.HCODEC_SIMPLE
    ts = np.arange(n_all, dtype=np.int64)
    lo = np.array([p[0] for p in pairs], np.uint32)
    up = np.array([p[1] for p in pairs], np.uint32)
    gid = np.arange(n_groups, dtype=np.int32)
    keep = [gid, gptr, ts, lo, up, cnt, pres, kind]
    r = H.HistResult()
    r.n_groups, r.n_pct, r.show_buckets, r.n_buckets = n_groups, 0, 1, D
    for name, a, ct in (("group_id", gid, C.c_int32), ("group_ptr", gptr, C.c_int64), ("ts_ms", ts, C.c_int64),
                        ("bucket_lower", lo, C.c_uint32), ("bucket_upper", up, C.c_uint32),
                        ("count", cnt, C.c_int64), ("present", pres, C.c_uint8), ("codec", kind, C.c_uint8)):
        setattr(r, name, a.ctypes.data_as(C.POINTER(ct)))
    out = H.result_to_series(r, [])
    assert keep and len(out) == n_groups
    for g in range(n_groups):
        keys, vals = _loop_bucket_series(list(lo), list(up), cnt, pres, kind, gptr[g], gptr[g + 1])
        assert [tuple(s.bucket) for s in out[g]] == [(k[0], int(k[1]), int(k[2])) for k in keys]
        for s, v in zip(out[g], vals):
            assert np.array_equal(np.asarray(s.values), v)
