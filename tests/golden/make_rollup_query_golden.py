"""Transcribes the known answers of test/core/TestTsdbQueryRollup.java (the rollup read
path) into tests/golden/rollup_queries.json.

Each case holds the writes the test makes (its storeLongRollup / storeFloatRollup /
storeCount / storePoint loops expanded into explicit addAggregatePoint calls, plus the raw
series of beforeLocal where the query falls back to raw data), the query of its setQuery,
and the answer its assertions state: per group the (timestamp, value) points, a group with
no points, no group at all, or the exception class.  Nothing here runs the reference; the
expected values restate the tests' own loops.

    python tests/golden/make_rollup_query_golden.py
"""
from __future__ import annotations

import json
import os

METRIC, METRIC_B = "sys.cpu.user", "sys.cpu.system"
TAGS = {"host": "web01"}
TAGS2 = {"host": "web02"}
AGG_IDS = {"sum": 0, "count": 1, "max": 2, "min": 3}
INTERVALS = [["10m", "6h"], ["1h", "1d"], ["1d", "1n"]]
T0 = 1356998400
SRC = "test/core/TestTsdbQueryRollup.java"


def store_long_rollup(w, start, end, two, offset, interval_s, agg):   # :858-900
    a, b, i = start, start + (interval_s if offset else 0), 0
    while a <= end:
        i += interval_s
        w.append(["agg", METRIC, TAGS, a, "long", i, "10m", agg])
        if two:
            w.append(["agg", METRIC_B, TAGS, b, "long", i, "10m", agg])
        a += interval_s * 2 if offset else interval_s
        b += interval_s * 2 if offset else interval_s
    a, b = start, start + (interval_s if offset else 0)
    while a <= end:
        i -= interval_s
        w.append(["agg", METRIC, TAGS2, a, "long", i, "10m", agg])
        if two:
            w.append(["agg", METRIC_B, TAGS2, b, "long", i, "10m", agg])
        a += interval_s * 2 if offset else interval_s
        b += interval_s * 2 if offset else interval_s


def store_count(w, start, end, two, offset, interval_s, value):   # :902-944
    for tags in (TAGS, TAGS2):
        a, b = start, start + (interval_s if offset else 0)
        while a <= end:
            w.append(["agg", METRIC, tags, a, "long", value, "10m", "count"])
            if two:
                w.append(["agg", METRIC_B, tags, b, "long", value, "10m", "count"])
            a += interval_s * 2 if offset else interval_s
            b += interval_s * 2 if offset else interval_s


def f32(x):
    import struct
    return struct.unpack(">f", struct.pack(">f", x))[0]


def store_float_rollup(w, start, end, two, offset, interval_s, agg):   # :946-989
    a, b, i = start, start + (interval_s if offset else 0), f32(0.5)
    while a <= end:
        i = f32(i + interval_s)
        w.append(["agg", METRIC, TAGS, a, "float", i, "10m", agg])
        if two:
            w.append(["agg", METRIC_B, TAGS, b, "float", i, "10m", agg])
        a += interval_s * 2 if offset else interval_s
        b += interval_s * 2 if offset else interval_s
    a, b = start, start + (interval_s if offset else 0)
    while a <= end:
        i = f32(i - interval_s)
        w.append(["agg", METRIC, TAGS2, a, "float", i, "10m", agg])
        if two:
            w.append(["agg", METRIC_B, TAGS2, b, "float", i, "10m", agg])
        a += interval_s * 2 if offset else interval_s
        b += interval_s * 2 if offset else interval_s


def store_point(w, ts, value, agg):   # :991-995
    w.append(["agg", METRIC, TAGS, ts, "long", value, "10m", agg])


def raw_series(w):   # BaseTsdbTest.storeLongTimeSeriesSeconds(false, false) :610-640
    ts = T0
    for i in range(1, 301):
        ts += 30
        w.append(["raw", METRIC, TAGS, ts, "long", i])
    ts = T0
    for i in range(300, 0, -1):
        ts += 30
        w.append(["raw", METRIC, TAGS2, ts, "long", i])


def query(ds, agg, tags=TAGS, group_by=None, rate=False, end=1357041600, start=T0):   # setQuery :997-1011
    return {"start": start, "end": end, "metric": METRIC, "ds": ds, "aggregator": group_by or agg,
            "tags": dict(tags), "rate": rate}


def series(ts0, step, n, v0, dv):
    return [[(ts0 + k * step) * 1000, v0 + k * dv] for k in range(n)]


def cases():
    out = []

    def add(name, lines, writes, q, expect, tol=1e-4, **kw):
        c = {"name": name, "source": f"{SRC}:{lines}", "writes": writes, "query": q, "expect": expect, "tol": tol}
        c.update(kw)
        out.append(c)

    # :101-135 15m has no rollup table (10m does not divide it): raw data
    w = []
    raw_series(w)
    store_long_rollup(w, T0, 1357041600, False, False, 600, "sum")
    pts = [[(T0 + k * 900) * 1000, 435 + 900 * k] for k in range(10)] + [[(T0 + 10 * 900) * 1000, 300]]
    add("run15mSumLongSingleTS", "101-135", w, query("15m-sum", "sum"), {"groups": [pts]}, 1e-5)

    w = []
    store_long_rollup(w, T0, 1357041599, False, False, 600, "sum")
    add("run30mSumLongSingleTS", "138-167", w, query("30m-sum", "sum"),
        {"groups": [series(T0, 1800, 24, 3600, 5400)]}, 0)

    w = []
    store_long_rollup(w, T0, 1357041599, False, False, 600, "sum")
    add("run10mZimSumLongSingleTS", "170-201", w, query("10m-zimsum", "zimsum"),
        {"groups": [series(T0, 600, 72, 600, 600)]})

    w = []
    store_long_rollup(w, T0, 1357041599, False, False, 600, "sum")
    add("run10mMaxLongSingleTSNotFound", "203-218", w, query("10m-max", "max"), {"groups": []})

    w = []
    store_long_rollup(w, T0, 1357041600, False, False, 600, "sum")
    add("run10mSumLongSingleTS", "220-250", w, query("10m-sum", "sum"), {"groups": [series(T0, 600, 73, 600, 600)]})

    add("run10mSumLongSingleTSInMS", "252-262",
        [["agg", METRIC, TAGS, 1356998400000, "long", 0, "10m", "sum"]], None, {"write_error": "IllegalArgumentException"})

    w = []
    store_long_rollup(w, T0, 1357041600, False, False, 600, "sum")
    add("run10mSumLongSingleTSRate", "264-293", w, query("10m-sum", "sum", rate=True),
        {"groups": [series(T0 + 600, 600, 72, 1.0, 0.0)]}, 1e-5)

    w = []
    store_float_rollup(w, T0, 1357041600, True, False, 600, "sum")
    add("run10mSumFloatSingleTS", "295-324", w, query("10m-sum", "sum"),
        {"groups": [series(T0, 600, 73, 600.5, 600)]}, 1e-5)

    w = []
    store_float_rollup(w, T0, 1357041600, False, False, 600, "sum")
    add("run10mSumFloatSingleTSRate", "326-355", w, query("10m-sum", "sum", rate=True),
        {"groups": [series(T0 + 600, 600, 72, 1.0, 0.0)]}, 1e-5)

    w = []
    store_long_rollup(w, T0, 1357041600, True, False, 600, "sum")
    add("run10mSumLongDoubleTSFilter", "357-388", w, query("10m-sum", "sum"),
        {"groups": [series(T0, 600, 73, 600, 600)]})

    w = []
    store_long_rollup(w, T0, 1357041600, True, False, 600, "sum")
    add("run10mSumLongDoubleTS", "390-420", w, query("10m-sum", "sum", tags={}),
        {"groups": [series(T0, 600, 73, 43800, 0)]})

    w = []
    for agg in ("sum", "max", "min"):
        store_long_rollup(w, T0, 1357041600, True, False, 600, agg)
    add("run10mSumLongDoubleTSFilterOtherAggs", "422-457", w, query("10m-sum", "sum"),
        {"groups": [series(T0, 600, 73, 600, 600)]})

    for agg, lines in (("max", "459-489"), ("min", "491-521")):
        w = []
        store_long_rollup(w, T0, 1357041600, False, False, 600, agg)
        add(f"run10m{agg.capitalize()}LongSingleTS", lines, w, query(f"10m-{agg}", agg),
            {"groups": [series(T0, 600, 73, 600, 600)]})

    w = []
    store_long_rollup(w, T0, 1357041600, False, False, 600, "sum")
    store_count(w, T0, 1357041600, False, False, 600, 2)
    add("run10mAvgLongSingleTS", "523-554", w, query("10m-avg", "avg"), {"groups": [series(T0, 600, 73, 300, 300)]})

    w = []
    store_long_rollup(w, T0, 1357041600, False, False, 600, "sum")
    add("run10mAvgLongSingleTSMissingCount", "556-576", w, query("10m-avg", "avg"), {"groups": [[]]})

    w = []
    store_count(w, T0, 1357041600, False, False, 600, 1)
    add("run10mAvgLongSingleTSMissingSum", "578-597", w, query("10m-avg", "avg"), {"groups": [[]]})

    w = []
    store_point(w, 1356998400, 20, "sum")
    store_point(w, 1356998400, 2, "count")
    store_point(w, 1356999000, 40, "sum")
    store_point(w, 1356999600, 60, "sum")
    store_point(w, 1356999600, 3, "count")
    store_point(w, 1357000200, 80, "sum")
    store_point(w, 1357000200, 4, "count")
    three = [[1356998400000, 10], [1356999600000, 20], [1357000200000, 20]]
    add("run10mAvgLongSingleTSMissingACount", "599-635", w, query("10m-avg", "avg"), {"groups": [three]})

    w = []
    store_point(w, 1356998400, 20, "sum")
    store_point(w, 1356998400, 2, "count")
    store_point(w, 1356999000, 5, "count")
    store_point(w, 1356999600, 60, "sum")
    store_point(w, 1356999600, 3, "count")
    store_point(w, 1357000200, 80, "sum")
    store_point(w, 1357000200, 4, "count")
    add("run10mAvgLongSingleTSMissingASum", "637-673", w, query("10m-avg", "avg"), {"groups": [three]})

    w = []
    store_point(w, 1356998400, 20, "sum")
    store_point(w, 1356999000, 5, "count")
    store_point(w, 1356999600, 60, "sum")
    store_point(w, 1357000200, 4, "count")
    add("run10mAvgLongSingleTSMissingToZero", "675-702", w, query("10m-avg", "avg"), {"groups": [[]]})

    w = []
    for ts, v, a in ((1356998400, 20, "sum"), (1356998400, 2, "count"), (1356999000, 40, "sum"),
                     (1356999000, 5, "count"), (1357084800, 60, "sum"), (1357085400, 4, "count"),
                     (1357171200, 90, "sum"), (1357171200, 3, "count"), (1357171800, 100, "sum"),
                     (1357171800, 5, "count")):
        store_point(w, ts, v, a)
    add("run10mAvgLongSingleTSMissingToZeroOneSpan", "704-752", w, query("10m-avg", "avg", end=1359590400),
        {"groups": [[[1356998400000, 10], [1356999000000, 8], [1357171200000, 30], [1357171800000, 20]]]})

    w = []
    for ts, v, a in ((1356998400, 20, "sum"), (1356999000, 5, "count"), (1357084800, 60, "sum"),
                     (1357084800, 3, "count"), (1357085400, 80, "sum"), (1357085400, 4, "count"),
                     (1357171200, 3, "count"), (1357171800, 100, "sum")):
        store_point(w, ts, v, a)
    add("run10mAvgLongSingleTSMissingToZeroBookends", "754-796", w, query("10m-avg", "avg", end=1359590400),
        {"groups": [[[1357084800000, 20], [1357085400000, 20]]]})

    w = [["agg", METRIC, TAGS, 1357026600, "long", 2147483647, "10m", "sum"],
         ["agg", METRIC, TAGS, 1357026600, "float", 42.5, "10m", "sum"]]
    add("runDupes", "798-823", w, query("10m-sum", "sum"), {"error": "IllegalDataException"}, fix_duplicates=False)
    add("runDupesFixed", "798-823", w, query("10m-sum", "sum"), {"first": [1357026600000, 42.5]},
        fix_duplicates=True)

    w = [["column", "10m", METRIC, TAGS, 1356998400, "73756d3a0000", "2a"]]
    add("oldStringPrefix", "825-852", w, query("10m-sum", "sum"), {"groups": [[[1356998400000, 42]]]}, 1e-3)
    return out


def main():
    doc = {"about": __doc__.strip().splitlines()[0], "agg_ids": AGG_IDS, "intervals": INTERVALS,
           "cases": cases()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rollup_queries.json")
    with open(path, "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(path, len(doc["cases"]), "cases")


if __name__ == "__main__":
    main()
