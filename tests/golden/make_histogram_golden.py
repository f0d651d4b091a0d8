"""Transcribes the known answers of the reference's histogram tests into
tests/golden/histogram.json:

- values:   SimpleHistogram.percentile / fromHistogram (test/core/TestSimpleHistogram.java); its merge
            tests as queries whose bucket series are checked on the buckets the test asserts
- queries:  HistogramAggregationIterator.create over HistogramSpans
            (test/core/TestHistogramAggregationIterator.java: every test method),
            HistogramDownsampler over one span (test/core/TestHistogramDownsampler.java: the
            fixed-interval and "all" methods with a non-zero query start), SimpleHistogram.aggregate
            (TestSimpleHistogram merges) and TsdbQuery.runHistogram end to end over the MockBase
            stores of test/core/BaseTsdbTest.java:792-856 (test/core/TestTsdbQueryHistogramQueries.java).

Histogram values are written the way the tests build them: LongHistogramDataPointForTest
(test/core/LongHistogramDataPointForTest.java: [codec id][BE64 value]; its percentile(p) is
value * p, so a query asking for percentile 1.0 returns each point's summed value) or the Kryo
calls of the SimpleHistogram tests (writeShort / writeFloat big-endian, writeLong(v, true) varints).
Columns are the cells TSDB.addHistogramPoint stores: qualifier Internal.getQualifier(ts, 0x06)
(src/core/Internal.java:1027-1049) in the row of base time ts - ts % 3600 (seconds).

Iterator-level tests (HistogramAggregationIterator.create / a bare HistogramDownsampler) are replayed
with explicit span-group bounds ("span_range": tsdbhip_hist_run_range).  A bare downsampler's
timestamp() for "all" is the query start; through the aggregation iterator a point carries the
downsampler clone's timestamp field (HistogramDownsampler.java:179-183), the query end -- the
fixture keeps the test's values and states the timestamp the aggregation iterator reports.

    python tests/golden/make_histogram_golden.py
"""
from __future__ import annotations

import json
import os
import struct

BASE = 1356998400000   # BASE_TIME of the histogram tests (ms)
LONG_ID = 0            # "{\"net.opentsdb.core.LongHistogramDataPointForTestDecoder\": 0}"
SIMPLE, LONG = 1, 2    # TSDB_HCODEC_*


def varlong(v: int) -> bytes:   # Kryo 2.21 Output.writeLong(v, true)
    u = v & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    for _ in range(8):
        if u >> 7 == 0:
            out.append(u)
            return bytes(out)
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u & 0xFF)
    return bytes(out)


def simple(cid, buckets, under, over, count=None) -> bytes:
    b = bytes([cid]) + struct.pack(">h", len(buckets) if count is None else count)
    for lo, up, c in buckets:
        b += struct.pack(">ff", lo, up) + varlong(c)
    return b + varlong(under) + varlong(over)


def longh(v: int) -> bytes:
    return bytes([LONG_ID]) + struct.pack(">q", v)


def qual(ts: int):
    """(base seconds, qualifier) of Internal.getQualifier(ts, 0x06)."""
    if ts & 0xFFFFFFFF00000000:
        base = (ts // 1000) - (ts // 1000) % 3600
        return base, bytes([6]) + struct.pack(">I", ts - base * 1000)
    base = ts - ts % 3600
    return base, bytes([6]) + struct.pack(">H", ts - base)


def series_of(points):
    """[(ts, value bytes)] in time order -> rows [(base, [[qhex, vhex], ...])]."""
    rows = {}
    for ts, v in points:
        base, q = qual(ts)
        rows.setdefault(base, []).append((q, v))
    return [[base, [[q.hex(), v.hex()] for q, v in sorted(cols, key=lambda c: c[0])]] for base, cols in sorted(rows.items())]


def store(series, groups=None, codecs=None):
    return {"codecs": codecs or {str(LONG_ID): LONG}, "series": [series_of(s) for s in series],
            "groups": groups if groups is not None else [0] * len(series)}


def main():
    values, queries, stores = [], [], {}
    SH = "test/core/TestSimpleHistogram.java"
    # ---- SimpleHistogram.percentile ----------------------------------------------------------
    h3 = simple(0, [(1.0, 6.0, 5), (6.0, 10.0, 10), (10.0, 20.0, 1)], 0, 5)
    values.append({"name": "testSinglePercentile p50", "source": f"{SH}:279-303", "value": h3.hex(), "kind": SIMPLE,
                   "p": 50.0, "expect": 8.0})
    values.append({"name": "testSinglePercentile p1000", "source": f"{SH}:279-303", "value": h3.hex(), "kind": SIMPLE,
                   "p": 1000.0, "expect": -1.0})
    h4 = simple(0, [(1.0, 6.0, 5), (6.0, 10.0, 10), (10.0, 20.0, 1), (20.0, 40.0, 0)], 0, 5)
    values.append({"name": "testPercentileList p50", "source": f"{SH}:305-337", "value": h4.hex(), "kind": SIMPLE,
                   "p": 50.0, "expect": 8.0})
    values.append({"name": "testPercentileList p99", "source": f"{SH}:305-337", "value": h4.hex(), "kind": SIMPLE,
                   "p": 99.0, "expect": 15.0})
    values.append({"name": "testIncompletByteArray", "source": f"{SH}:237-254",
                   "value": (bytes([0]) + struct.pack(">h", 4)).hex(), "kind": SIMPLE, "p": 50.0, "expect": None})
    # ---- SimpleHistogram.aggregate (merges) as a query: spans with a point at the same time ---
    def merge_case(name, lines, hists, expect_buckets):
        key = f"merge_{name}"
        stores[key] = store([[(BASE, h)] for h in hists], codecs={"0": SIMPLE})
        queries.append({"name": name, "source": f"{SH}:{lines}", "store": key, "span_range": [BASE, BASE],
                        "start": BASE, "end": BASE + 1000, "aggregator": "sum", "downsample": None,
                        "percentiles": [], "show_buckets": True, "partial_buckets": True,
                        "expect": [{"group": 0, "series": [
                            {"bucket": b, "ts": [BASE], "values": [v]} for b, v in expect_buckets]}]})
    h1 = simple(0, [(1.0, 6.0, 5), (6.0, 10.0, 10), (10.0, 20.0, 1), (20.0, 40.0, 0)], 0, 5)
    h1u = simple(0, [(1.0, 6.0, 5), (6.0, 10.0, 10), (10.0, 20.0, 1), (20.0, 40.0, 0)], 2, 5)
    F = lambda x: struct.unpack(">I", struct.pack(">f", x))[0]   # noqa: E731
    merge_case("testSingleHistogramMerge", "339-373", [h1, h1u],
               [([0, 0, 0], 2), ([1, F(1.0), F(6.0)], 10), ([1, F(6.0), F(10.0)], 20), ([1, F(10.0), F(20.0)], 2),
                ([2, 0, 0], 10)])
    merge_case("testMultipleHistogramMerge", "375-412", [h1, h1, h1],
               [([1, F(1.0), F(6.0)], 15), ([1, F(6.0), F(10.0)], 30), ([1, F(10.0), F(20.0)], 3),
                ([2, 0, 0], 15)])
    ha = simple(0, [(5.0, 7.0, 3), (7.0, 10.0, 5), (15.0, 20.0, 2)], 0, 0)
    hb = simple(0, [(5.0, 7.0, 3), (7.0, 10.0, 5), (10.0, 15.0, 2), (15.0, 20.0, 1)], 0, 0)
    merge_case("testMissingBucketsHistogramAggregation", "526-541", [ha, hb], [([1, F(10.0), F(15.0)], 2)])

    # ---- HistogramAggregationIterator ----------------------------------------------------------
    AI = "test/core/TestHistogramAggregationIterator.java"

    def it_case(name, lines, spans, start, end, ds, expect):
        key = f"it_{name}"
        stores[key] = store([[(t, longh(v)) for t, v in sp] for sp in spans])
        queries.append({"name": name, "source": f"{AI}:{lines}", "store": key, "span_range": [start, end],
                        "start": 0, "end": 0, "aggregator": "sum", "downsample": ds, "percentiles": [1.0],
                        "show_buckets": False,
                        "expect": [{"group": 0, "series": [{"percentile": 1.0, "ts": [t for t, _ in expect],
                                                            "values": [float(v) for _, v in expect]}]}]})
    ten = [(BASE + 5000 * i, i) for i in range(10)]
    it_case("testOneHistogramSpanWithNoDownsampler", "49-81", [ten], BASE, BASE + 50000, None, ten)
    it_case("testOneHistogramSpanWithDownsampler_10secs", "83-132", [ten], BASE, BASE + 50000, "10s-sum",
            [(BASE + 10000 * k, 4 * k + 1) for k in range(5)])
    it_case("testOneHistogramSpanNoDownSamplerSkipEarlyDataPoints", "134-167", [ten], BASE + 5000, BASE + 50000, None,
            ten[1:])
    it_case("testOneHistogramSpanNoDownSamplerOutofRange", "169-188", [ten], BASE + 50000, BASE + 100000, None, [])
    it_case("testOneHistogramSpanNoDownSamplerLaterDataPoints", "190-222", [ten], BASE, BASE + 25000, None, ten[:6])
    it_case("testOneHistogramSpanDownSamplerLaterDataPoints", "224-264", [ten], BASE, BASE + 25000, "10s-sum",
            [(BASE, 1), (BASE + 10000, 5), (BASE + 20000, 9)])
    it_case("testTwoHistogramSpanNoDownSamplerSameTimestamp", "266-308", [ten, ten], BASE, BASE + 50000, None,
            [(t, 2 * v) for t, v in ten])
    it_case("testTwoHistogramSpanDownSamplerSameTimestamp", "310-353", [ten, ten], BASE, BASE + 50000, "10s-sum",
            [(BASE + 10000 * i, 2 * (i * 2 + i * 2 + 1)) for i in range(5)])
    it_case("testTwoHistogramSpanNoDownSamplerDiffTimestamp", "355-401",
            [[(BASE + 5000 * i, i) for i in range(0, 10, 2)], [(BASE + 5000 * i, i) for i in range(1, 10, 2)]],
            BASE, BASE + 50000, None, ten)
    it_case("testTwoHistogramSpanNoDownSamplerMergeSome", "403-457",
            [ten, [(BASE + 5000 * i, i) for i in range(1, 5)] + [(BASE + 5000 * (5 + i), 5 + i) for i in range(5, 10)]],
            BASE, BASE + 100000, None,
            [(BASE + 5000 * i, 2 * i) for i in range(5)] + [(BASE + 5000 * i, i) for i in range(5, 15)])
    it_case("testTwoHistogramSpanNoDownSamplerOneHasMore", "459-500",
            [ten, [(BASE + 5000 * i, i) for i in range(1, 5)]], BASE, BASE + 100000, None,
            [(BASE + 5000 * i, 2 * i) for i in range(5)] + [(BASE + 5000 * i, i) for i in range(5, 10)])
    it_case("testTwoHistogramSpanNoDownSamplerOneOutofRange", "502-540",
            [ten, [(BASE + 5000 * i, i) for i in range(1, 5)]], BASE + 25000, BASE + 50000, None,
            [(BASE + 5000 * (5 + i), 5 + i) for i in range(5)])

    # ---- HistogramDownsampler (one span, through the aggregation iterator from 0) --------------
    DS = "test/core/TestHistogramDownsampler.java"

    def ds_case(name, lines, pts, spec, qs, qe, expect):
        key = f"ds_{name}"
        stores[key] = store([[(t, longh(v)) for t, v in pts]])
        queries.append({"name": name, "source": f"{DS}:{lines}", "store": key, "span_range": [0, 1 << 62],
                        "start": qs, "end": qe, "aggregator": "sum", "downsample": spec, "percentiles": [1.0],
                        "show_buckets": False,
                        "expect": [{"group": 0, "series": [{"percentile": 1.0, "ts": [t for t, _ in expect],
                                                            "values": [float(v) for _, v in expect]}]}]})
    six = [(BASE, 40), (BASE + 2000000, 50), (BASE + 3600000, 40), (BASE + 3605000, 50), (BASE + 7200000, 40),
           (BASE + 9200000, 50)]
    ds_case("testDownsampler", "112-136", six, "1000s-sum", 0, 0,
            [(BASE - 400000, 40), (BASE + 1600000, 50), (BASE + 3600000, 90), (BASE + 6600000, 40),
             (BASE + 8600000, 50)])
    eleven = [(BASE + 5000 * i, 1 << i) for i in range(11)]
    ds_case("testDownsampler_10seconds", "138-190", eleven, "10s-sum", 0, 0,
            [(BASE, 3), (BASE + 10000, 12), (BASE + 20000, 48), (BASE + 30000, 192), (BASE + 40000, 768),
             (BASE + 50000, 1024)])
    six2 = [(BASE + 5000, 1), (BASE + 15000, 2), (BASE + 25000, 4), (BASE + 35000, 8), (BASE + 45000, 16),
            (BASE + 55000, 32)]
    ds_case("testDownsampler_15seconds", "192-229", six2, "15s-sum", 0, 0,
            [(BASE, 1), (BASE + 15000, 6), (BASE + 30000, 8), (BASE + 45000, 48)])
    # value 14 at timestamp() = BASE + 15000 (the query start); the aggregation iterator's point
    # carries the clone's timestamp, the query end BASE + 45000
    ds_case("testDownsampler_allFilterOnQuery", "262-294", six2, "0all-sum", BASE + 15000, BASE + 45000,
            [(BASE + 45000, 14)])
    ds_case("testDownsampler_allFilterOnQueryOutOfRangeEarly", "295-325", six2, "0all-sum", BASE + 65000,
            BASE + 75000, [])
    ds_case("testDownsampler_allFilterOnQueryOutOfRangeLate", "326-356", six2, "0all-sum", BASE - 15000,
            BASE - 5000, [])

    # ---- TsdbQuery.runHistogram (MockBase stores of BaseTsdbTest) -----------------------------
    TQ = "test/core/TestTsdbQueryHistogramQueries.java"
    ms_pts = [[(1356998400000 + 500 * i, longh(i)) for i in range(1, 301)],
              [(1356998400000 + 500 * (301 - i), longh(i)) for i in range(300, 0, -1)]]
    s_pts = [[(1356998400 + 30 * i, longh(i)) for i in range(1, 301)],
             [(1356998400 + 30 * (301 - i), longh(i)) for i in range(300, 0, -1)]]
    stores["tq_ms_web01"] = store(ms_pts[:1])                    # host=web01 filter: one span
    stores["tq_ms_all"] = store(ms_pts, groups=[0, 0])           # no group-by: one group
    stores["tq_ms_groups"] = store(ms_pts, groups=[0, 1])        # host=*: web01, web02
    stores["tq_s_web01"] = store(s_pts[:1])
    stores["tq_s_all"] = store(s_pts, groups=[0, 0])
    # runWithOnlyAnnotation: the row at 1357002000 is flushed (storage.flushRow)
    stores["tq_s_web01_flushed"] = store([[p for p in s_pts[0] if not (1357002000 <= p[0] < 1357005600)]])
    stores["tq_empty"] = store([])

    def tq(name, lines, key, agg, pcts, expect, tol=1e-4):
        queries.append({"name": name, "source": f"{TQ}:{lines}", "store": key, "span_range": None,
                        "start": 1356998400, "end": 1357041600, "aggregator": agg, "downsample": None,
                        "percentiles": pcts, "show_buckets": False, "tol": tol, "expect": expect})

    def pseries(p, ts, vals):
        return {"percentile": p, "ts": ts, "values": vals}
    ts_ms = [1356998400000 + 500 * i for i in range(1, 301)]
    ts_s = [(1356998400 + 30 * i) * 1000 for i in range(1, 301)]
    tq("runSingleTsMsSinglePercentile", "111-141", "tq_ms_web01", "sum", [0.98],
       [{"group": 0, "series": [pseries(0.98, ts_ms, [v * 0.98 for v in range(1, 301)])]}])
    tq("runSingleTsMsDoulePercentile", "143-190", "tq_ms_web01", "sum", [0.98, 0.95],
       [{"group": 0, "series": [pseries(0.98, ts_ms, [v * 0.98 for v in range(1, 301)]),
                                pseries(0.95, ts_ms, [v * 0.95 for v in range(1, 301)])]}])
    tq("runSingleTsMsTwoAggSum", "192-221", "tq_ms_all", "sum", [0.98],
       [{"group": 0, "series": [pseries(0.98, ts_ms, [301 * 0.98] * 300)]}])
    tq("runSingleTsMsAggNone", "223-271", "tq_ms_all", "none", [0.98],
       [{"group": 0, "series": [pseries(0.98, ts_ms, [v * 0.98 for v in range(1, 301)])]},
        {"group": 1, "series": [pseries(0.98, ts_ms, [v * 0.98 for v in range(300, 0, -1)])]}])
    tq("runSingleTsMsAggSumTwoGroups", "273-322", "tq_ms_groups", "sum", [0.98],
       [{"group": 0, "series": [pseries(0.98, ts_ms, [v * 0.98 for v in range(1, 301)])]},
        {"group": 1, "series": [pseries(0.98, ts_ms, [v * 0.98 for v in range(300, 0, -1)])]}])
    tq("runWithAnnotation", "324-357", "tq_s_web01", "sum", [0.98],
       [{"group": 0, "series": [pseries(0.98, ts_s, [v * 0.98 for v in range(1, 301)])]}])
    kept = [i for i in range(1, 301) if not (1357002000 <= 1356998400 + 30 * i < 1357005600)]
    tq("runWithOnlyAnnotation", "359-398", "tq_s_web01_flushed", "sum", [0.98],
       [{"group": 0, "series": [pseries(0.98, [(1356998400 + 30 * i) * 1000 for i in kept], [v * 0.98 for v in kept])]}])
    tq("runTSUIDQuery", "400-429", "tq_s_web01", "sum", [0.98],
       [{"group": 0, "series": [pseries(0.98, ts_s, [v * 0.98 for v in range(1, 301)])]}])
    tq("runTSUIDsAggSum", "431-460", "tq_s_all", "sum", [0.98],
       [{"group": 0, "series": [pseries(0.98, ts_s, [301 * 0.98] * 300)]}])
    tq("runTSUIDQueryNoData", "462-480", "tq_empty", "sum", [0.98], [])

    out = {"values": values, "stores": stores, "queries": queries}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "histogram.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{path}: {len(values)} values, {len(queries)} queries, {len(stores)} stores")


if __name__ == "__main__":
    main()
