"""Generates the golden-vector fixtures in tests/golden/*.json.

Every case below is a transcription of a known answer held by the reference's own
unit tests (file:line cited per case, relative to the reference tree).  The Java code
cannot run in this pipeline (no JDK), so these fixtures are the
link between the oracle / the GPU engine and the reference's behaviour.  Inputs are
written out explicitly; expected values follow the same arithmetic the Java test
states (Python float == Java double for these expressions).

Run:  python tests/golden/make_golden.py     (rewrites the JSON files next to it)
"""
from __future__ import annotations

import json
import math
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
LONG_MAX = (1 << 63) - 1


def f32(x):
    """Java float arithmetic result as a double."""
    return struct.unpack(">f", struct.pack(">f", x))[0]


def L(ts, v):
    return [ts, 1, int(v)]


def D(ts, v):
    return [ts, 0, float(v)]


def arr(points, generator=False):
    return {"op": "array", "points": points, "generator": generator}


def ds(src, spec, start=0, end=0, qs=0, qe=LONG_MAX):
    return {"op": "downsample", "src": src, "spec": spec, "start": start, "end": end, "qs": qs, "qe": qe}


def ds_raw(src, fn, interval, fill="none", start=0, end=0):
    return {"op": "downsample_raw", "src": src, "fn": fn, "interval": interval, "fill": fill,
            "start": start, "end": end}


def rate(src, counter=False, counter_max=LONG_MAX, reset=0, drop=False):
    return {"op": "rate", "src": src, "counter": counter, "counter_max": counter_max, "reset": reset, "drop": drop}


def agg(srcs, start, end, fn="sum", interp=None, is_rate=False):
    return {"op": "aggregate", "srcs": srcs, "start": start, "end": end, "fn": fn, "interp": interp,
            "rate": is_rate}


ITER = []


def case(name, ref, view, expect=None, tol=0.0, seek=None, error=None, check_int=True):
    c = {"name": name, "ref": ref, "view": view, "seek": seek, "tol": tol, "check_int": check_int}
    if error:
        c["error"] = error
    else:
        c["expect"] = expect
    ITER.append(c)


# ---------------------------------------------------------------------------
# TestDownsampler (test/core/TestDownsampler.java)
B = 1356998400000
DS_DATA = [L(B, 40), L(B + 2000000, 50), L(B + 3600000, 40), L(B + 3605000, 50), L(B + 7200000, 40),
           L(B + 9200000, 50)]
exp = [D(B - 400000, 40), D(B + 1600000, 50), D(B + 3600000, 45), D(B + 6600000, 40), D(B + 8600000, 50)]
case("TestDownsampler.testDownsampler", "test/core/TestDownsampler.java:80-105",
     ds(arr(DS_DATA), "1000s-avg"), exp, 1e-7)
case("TestDownsampler.testDownsamplerDeprecated", "test/core/TestDownsampler.java:107-131",
     ds_raw(arr(DS_DATA), "avg", 1000000), exp, 1e-7)
TEN = [D(B + 5000 * i, 2 ** i) for i in range(11)]
exp10 = [D(B, 3), D(B + 10000, 12), D(B + 20000, 48), D(B + 30000, 192), D(B + 40000, 768), D(B + 50000, 1024)]
case("TestDownsampler.testDownsampler_10seconds", "test/core/TestDownsampler.java:174-214",
     ds(arr(TEN), "10s-sum"), exp10, 1e-7)
case("TestDownsampler.testDownsamplerDeprecated_10seconds", "test/core/TestDownsampler.java:133-172",
     ds_raw(arr(TEN), "sum", 10000), exp10, 1e-7)
FIFTEEN = [L(B + 5000, 1), L(B + 15000, 2), L(B + 25000, 4), L(B + 35000, 8), L(B + 45000, 16), L(B + 55000, 32)]
exp15 = [D(B, 1), D(B + 15000, 6), D(B + 30000, 8), D(B + 45000, 48)]
case("TestDownsampler.testDownsampler_15seconds", "test/core/TestDownsampler.java:248-279",
     ds(arr(FIFTEEN), "15s-sum"), exp15, 1e-7)
case("TestDownsampler.testDownsamplerDeprecated_15seconds", "test/core/TestDownsampler.java:216-246",
     ds_raw(arr(FIFTEEN), "sum", 15000), exp15, 1e-7)
case("TestDownsampler.testDownsampler_allFullRange", "test/core/TestDownsampler.java:281-307",
     ds(arr(FIFTEEN), "0all-sum", qs=0, qe=LONG_MAX), [D(0, 63)], 1e-7)
case("TestDownsampler.testDownsampler_allFilterOnQuery", "test/core/TestDownsampler.java:309-335",
     ds(arr(FIFTEEN), "0all-sum", qs=B + 15000, qe=B + 45000), [D(B + 15000, 14)], 1e-7)
case("TestDownsampler.testDownsampler_allFilterOnQueryOutOfRangeEarly", "test/core/TestDownsampler.java:337-361",
     ds(arr(FIFTEEN), "0all-sum", qs=B + 65000, qe=B + 75000), [], 0)
case("TestDownsampler.testDownsampler_allFilterOnQueryOutOfRangeLate", "test/core/TestDownsampler.java:363-387",
     ds(arr(FIFTEEN), "0all-sum", qs=B - 15000, qe=B - 5000), [], 0)
case("TestDownsampler.testDownsampler_noData", "test/core/TestDownsampler.java:829-836",
     ds(arr([]), "1d-sum"), [], 0)
case("TestDownsampler.testDownsampler_1day", "test/core/TestDownsampler.java:847-868",
     ds_raw(arr([L(B, 1), L(B + 43200000, 2), L(B + 86400000, 4), L(B + 129600000, 8)]), "sum", 86400000),
     [D(B, 3), D(1357084800000, 12)], 1e-6)
case("TestDownsampler.testSeek", "test/core/TestDownsampler.java:1321-1342",
     ds_raw(arr(DS_DATA), "avg", 1000000), [D(B + 3600000, 45), D(B + 6600000, 40), D(B + 8600000, 50)],
     1e-7, seek=B + 3600000)
case("TestDownsampler.testSeek_skipPartialInterval", "test/core/TestDownsampler.java:1384-1409",
     ds_raw(arr(DS_DATA), "avg", 1000000), [D(B + 6600000, 40), D(B + 8600000, 50)], 1e-7, seek=B + 3800000)
case("TestDownsampler.testSeek_abandoningIncompleteInterval(first)", "test/core/TestDownsampler.java:1436-1453",
     ds_raw(arr([L(B + 100 + 1000 * i, 40) for i in range(11)]), "sum", 10000),
     [D(B, 400), D(B + 10000, 40)], 1e-7, seek=B)

# ---------------------------------------------------------------------------
# TestFillingDownsampler (test/core/TestFillingDownsampler.java)
b5 = 500
GAPS = [D(b5 + 25 * k, 1.0) for k in (4, 5, 7, 12, 15, 24, 25, 26, 27)]
nan = float("nan")
vals = [nan, 3.0, nan, 2.0, nan, nan, 4.0, nan, nan]
case("TestFillingDownsampler.testNaNMissingInterval", "test/core/TestFillingDownsampler.java:45-78",
     ds(arr(GAPS), "100ms-sum-nan", start=b5, end=b5 + 36 * 25, qs=0, qe=0),
     [D(b5 + 100 * i, v) for i, v in enumerate(vals)], 0)
case("TestFillingDownsampler.testZeroMissingInterval", "test/core/TestFillingDownsampler.java:80-112",
     ds(arr(GAPS), "100ms-sum-zero", start=b5, end=b5 + 36 * 25, qs=0, qe=0),
     [D(b5 + 100 * i, 0.0 if v != v else v) for i, v in enumerate(vals)], 0)
b1 = 1000
case("TestFillingDownsampler.testWithoutMissingIntervals", "test/core/TestFillingDownsampler.java:114-141",
     ds(arr([D(b1 + 25 * i, 12.0 - i) for i in range(12)]), "100ms-sum-nan", start=b1, end=b1 + 12 * 25, qs=0, qe=0),
     [D(b1, 42.0), D(b1 + 100, 26.0), D(b1 + 200, 10.0)], 0)
bt = 1425335895000
OOB = [D(bt - 60000 * 5 + 320, 53.), D(bt - 60000 * 2 + 8839, 16.), D(bt + 849, 9.), D(bt + 3849, 8.),
       D(bt + 6210, 7.), D(bt + 42216, 6.), D(bt + 60000 + 167, 5.), D(bt + 60000 + 28593, 4.),
       D(bt + 120000 + 30384, 37.), D(bt + 240000 + 1530, 86.)]
case("TestFillingDownsampler.testWithOutOfBoundsData", "test/core/TestFillingDownsampler.java:143-171",
     ds(arr(OOB), "1m-sum-nan", start=bt, end=bt + 120000, qs=0, qe=0),
     [D(1425335880000, 30.), D(1425335940000, 9.)], 0)
case("TestFillingDownsampler.testWithOutOfBoundsDataEarly", "test/core/TestFillingDownsampler.java:173-188",
     ds(arr(OOB[:2]), "1m-sum-nan", start=bt, end=bt + 120000, qs=0, qe=0),
     [D(1425335880000, nan), D(1425335940000, nan)], 0)
case("TestFillingDownsampler.testWithOutOfBoundsDataLate", "test/core/TestFillingDownsampler.java:190-205",
     ds(arr(OOB[-2:]), "1m-sum-nan", start=bt, end=bt + 120000, qs=0, qe=0),
     [D(1425335880000, nan), D(1425335940000, nan)], 0)
case("TestFillingDownsampler.testDownsampler_allFullRange", "test/core/TestFillingDownsampler.java:207-225",
     ds(arr(FIFTEEN), "0all-sum-nan", start=B + 5000, end=B + 55000, qs=0, qe=LONG_MAX), [D(0, 63)], 0)
case("TestFillingDownsampler.testDownsampler_allFilterOnQuery", "test/core/TestFillingDownsampler.java:227-245",
     ds(arr(FIFTEEN), "0all-sum-nan", start=B + 5000, end=B + 55000, qs=B + 15000, qe=B + 45000),
     [D(B + 15000, 14)], 0)
case("TestFillingDownsampler.testDownsampler_allFilterOnQueryOutOfRangeEarly",
     "test/core/TestFillingDownsampler.java:247-264",
     ds(arr(FIFTEEN), "0all-sum-nan", start=B + 5000, end=B + 55000, qs=B + 65000, qe=B + 75000), [], 0)
case("TestFillingDownsampler.testDownsampler_allFilterOnQueryOutOfRangeLate",
     "test/core/TestFillingDownsampler.java:266-283",
     ds(arr(FIFTEEN), "0all-sum-nan", start=B + 5000, end=B + 55000, qs=B - 15000, qe=B - 5000), [], 0)

# ---------------------------------------------------------------------------
# TestRateSpan (test/core/TestRateSpan.java)
RS = [D(1356998400000, 40.0), L(1356998400000 + 2000000, 50), L(1357002000000, 40),
      D(1357002000000 + 5000, 50.0), L(1357005600000, 40), D(1357005600000 + 2000000, 50.0)]
RATE_DP = [D(1356998400000, 40.0 / 1356998400), D(1356998400000 + 2000000, 10.0 / 2000.0),
           D(1357002000000, -10.0 / (1357002000 - 1356998400 - 2000)), D(1357002000000 + 5000, 10.0 / 5.0),
           D(1357005600000, -10.0 / (1357005600 - 1357002005)), D(1357005600000 + 2000000, 10.0 / 2000.0)]
case("TestRateSpan.testNext_iterateAll", "test/core/TestRateSpan.java:93-107", rate(arr(RS)), RATE_DP, 1e-7)
case("TestRateSpan.testSeek", "test/core/TestRateSpan.java:129-144", rate(arr(RS)),
     [D(1357002000000, 40.0 / 1357002000)] + RATE_DP[3:], 1e-7, seek=1357002000000)
case("TestRateSpan.testNext_counter", "test/core/TestRateSpan.java:185-201", rate(arr(RS), True, 70, 0),
     [D(1356998400000, 40.0 / 1356998400), D(1356998400000 + 2000000, 10.0 / 2000.0),
      D(1357002000000, (40.0 + 20) / 1600.0), D(1357002000000 + 5000, 10.0 / 5.0),
      D(1357005600000, (40.0 + 20) / 3595), D(1357005600000 + 2000000, 10.0 / 2000.0)], 1e-7)
case("TestRateSpan.testNext_counterLongMax", "test/core/TestRateSpan.java:203-227",
     rate(arr([L(1356998430000, LONG_MAX - 55), L(1356998460000, LONG_MAX - 25), L(1356998490000, 5)]),
          True, LONG_MAX, 0),
     [D(1356998430000, float(LONG_MAX - 55) / 1356998430.0), D(1356998460000, 1), D(1356998490000, 1)], 1e-7)
case("TestRateSpan.testNext_counterWithResetValue", "test/core/TestRateSpan.java:229-256",
     rate(arr([L(1356998400000, 40), L(1356998401000, 50), L(1356998402000, 40)]), True, 70, 1),
     [D(1356998400000, 40 / 1356998400.0), D(1356998401000, 10), D(1356998402000, 0)], 1e-7)
case("TestRateSpan.testNext_counterDroResets", "test/core/TestRateSpan.java:258-286",
     rate(arr([L(1356998400000, 40), L(1356998401000, 50), L(1356998402000, 40), L(1356998403000, 50)]),
          True, 70, 1, True),
     [D(1356998400000, 40 / 1356998400.0), D(1356998401000, 10), D(1356998403000, 10)], 1e-7)
case("TestRateSpan.testNext_counterDroResetsNothingAfter", "test/core/TestRateSpan.java:288-313",
     rate(arr([L(1356998400000, 40), L(1356998401000, 50), L(1356998402000, 40)]), True, 70, 1, True),
     [D(1356998400000, 40 / 1356998400.0), D(1356998401000, 10)], 1e-7)
case("TestRateSpan.testNext_decreasingTimestamps", "test/core/TestRateSpan.java:146-154",
     rate(arr([L(1357002000000 + 5000, 50), L(1357002000000 + 4000, 50)])), error="IllegalStateException")
case("TestRateSpan.testMoveToNextRate_duplicatedTimestamps", "test/core/TestRateSpan.java:156-167",
     rate(arr([L(1356998400000, 40), L(1356998400000 + 2000000, 50), L(1356998400000 + 2000000, 50)])),
     error="IllegalStateException")
case("TestRateSpan.testCalculateDelta_bigLongValues", "test/core/TestRateSpan.java:169-183",
     rate(arr([L(1356998400000, LONG_MAX - 100), L(1356998500000, LONG_MAX - 20)])),
     [D(1356998400000, float(LONG_MAX - 100) / 1356998400.0), D(1356998500000, 0.8)], 1e-7)

# ---------------------------------------------------------------------------
# TestAggregationIterator (test/core/TestAggregationIterator.java)
P1 = [L(B, 40), L(B + 10000, 50), L(B + 30000, 70)]
P2 = [L(B + 10000, 37), L(B + 20000, 48)]
D5 = [D(B + t, 1) for t in (0, 7000, 10000, 15000, 20000, 25000, 30000, 35000, 40000, 45000, 50000)]
S0, E0 = 1356998400 * 1000, 1356998500 * 1000
case("TestAggregationIterator.testAggregate_singleSpan", "test/core/TestAggregationIterator.java:73-87",
     agg([arr(P1)], S0, E0), P1, 0)
case("TestAggregationIterator.testAggregate_doubleSpans", "test/core/TestAggregationIterator.java:89-112",
     agg([arr(P1), arr(P2)], S0, E0), [L(B, 40), L(B + 10000, 87), L(B + 20000, 108), L(B + 30000, 70)], 0)
case("TestAggregationIterator.testAggregate_manySpansWithDownsampling",
     "test/core/TestAggregationIterator.java:114-144",
     agg([ds_raw(arr(D5), "avg", 10000) for _ in range(7)], B + 1000, B + 100000),
     [D(B + 10000 * i, 7) for i in range(1, 6)], 0)
case("TestAggregationIterator.testDownsample_afterAggregation", "test/core/TestAggregationIterator.java:146-179",
     ds_raw(agg([ds_raw(arr(D5), "avg", 10000) for _ in range(7)], B + 1000, B + 100000), "sum", 15000),
     [D(B, 7), D(B + 15000, 7), D(B + 30000, 14), D(B + 45000, 7)], 0)
case("TestAggregationIterator.testAggregate_emptySpan", "test/core/TestAggregationIterator.java:199-216",
     agg([arr([]), arr(P1)], B, E0), P1, 0)
case("TestAggregationIterator.pfsum", "test/core/TestAggregationIterator.java:290-318",
     agg([arr([L(B, 40), L(B + 30000, 70)]), arr(P2)], S0, E0, "sum", interp="prev"),
     [L(B, 40), L(B + 10000, 77), L(B + 20000, 88), L(B + 30000, 70)], 0)

# ---------------------------------------------------------------------------
# TestAggregators (test/core/TestAggregators.java)
AGGS = []


def acase(name, ref, fn, kind, values, expect, tol=0.0, error=None):
    c = {"name": name, "ref": ref, "fn": fn, "kind": kind, "values": values, "tol": tol}
    if error:
        c["error"] = error
    else:
        c["expect"] = expect
    AGGS.append(c)


r1000 = list(range(1, 1001))
for fn, v in [("p50", 500), ("p75", 750), ("p90", 900), ("p95", 950), ("p99", 990), ("p999", 999),
              ("ep50r3", 500), ("ep75r3", 750), ("ep90r3", 900), ("ep95r3", 950), ("ep99r3", 990), ("ep999r3", 999),
              ("ep50r7", 500), ("ep75r7", 750), ("ep90r7", 900), ("ep95r7", 950), ("ep99r7", 990), ("ep999r7", 999)]:
    acase(f"TestAggregators.testPercentiles[{fn}]", "test/core/TestAggregators.java:148-169", fn, "long", r1000, v)
acase("TestAggregators.testStdDevKnownValues", "test/core/TestAggregators.java:80-93", "dev", "long",
      list(range(10000)), 2886.7513315143719, 1.0)
acase("TestAggregators.testStdDevNoDeviation", "test/core/TestAggregators.java:106-111", "dev", "long", [3, 3, 3], 0, 1.0)
acase("TestAggregators.testStdDevFewDataInputs", "test/core/TestAggregators.java:113-119", "dev", "long", [1, 2], 0.5, 1.0)
acase("TestAggregators.testFirst(long)", "test/core/TestAggregators.java:171-188", "first", "long", list(range(10)), 0)
acase("TestAggregators.testFirst(double)", "test/core/TestAggregators.java:171-188", "first", "double",
      [0.5 + i for i in range(10)], 0.5, 1e-4)
acase("TestAggregators.testLast(long)", "test/core/TestAggregators.java:190-207", "last", "long", list(range(10)), 9)
acase("TestAggregators.testLast(double)", "test/core/TestAggregators.java:190-207", "last", "double",
      [0.5 + i for i in range(10)], 9.5, 1e-4)
acase("TestAggregators.testMedian[1]", "test/core/TestAggregators.java:209-235", "median", "long", [5, 2, -1, 400, 3], 3)
acase("TestAggregators.testMedian[2]", "test/core/TestAggregators.java:209-235", "median", "long",
      [5, 2, -1, 400, 3, -42], 3)
acase("TestAggregators.testMedian[3]", "test/core/TestAggregators.java:209-235", "median", "long", [42], 42)
acase("TestAggregators.testMedian[empty]", "test/core/TestAggregators.java:209-235", "median", "long", [], None,
      error="IllegalStateException")
acase("TestAggregators.testMedian[4]", "test/core/TestAggregators.java:209-235", "median", "double",
      [5.1, 2.434, -1.99, 400.69487, 3.15168], 3.15168, 1e-4)
acase("TestAggregators.testMedian[5]", "test/core/TestAggregators.java:209-235", "median", "double",
      [5.1, 2.434, -1.99, 400.69487, 3.15168, -42], 3.15168, 1e-4)
acase("TestAggregators.testMedian[6]", "test/core/TestAggregators.java:209-235", "median", "double", [42.5], 42.5, 1e-4)
acase("TestAggregators.testMedian[empty double]", "test/core/TestAggregators.java:209-235", "median", "double", [],
      "nan")
acase("TestAggregators.testSquareSumFewDataInputs", "test/core/TestAggregators.java:256-264", "squareSum", "long",
      [1, 2], 5)

# ---------------------------------------------------------------------------
# Codec (test/core/TestInternal.java, test/core/TestCompactionQueue.java)
CODEC = {
    "build_qualifier": [
        # [timestamp, flags, expected bytes hex, ref]
        [1356998403, 7, "0037", "test/core/TestInternal.java:617-621"],
        [1357001999, 7, "e0f7", "test/core/TestInternal.java:623-627"],
        [1356998403, 5, "0035", "test/core/TestInternal.java:629-633"],
        [1357001999, 5, "e0f5", "test/core/TestInternal.java:635-639"],
        [1356998403, 3, "0033", "test/core/TestInternal.java:641-645"],
        [1357001999, 3, "e0f3", "test/core/TestInternal.java:647-651"],
        [1356998403, 1, "0031", "test/core/TestInternal.java:653-657"],
        [1357001999, 1, "e0f1", "test/core/TestInternal.java:659-663"],
        [1356998403, 0, "0030", "test/core/TestInternal.java:665-669"],
        [1357001999, 0, "e0f0", "test/core/TestInternal.java:671-675"],
        [1356998403, 0xF, "003f", "test/core/TestInternal.java:677-682"],
        [1357001999, 0xF, "e0ff", "test/core/TestInternal.java:684-689"],
        [1356998403, 0xB, "003b", "test/core/TestInternal.java:691-696"],
        [1357001999, 0xB, "e0fb", "test/core/TestInternal.java:698-703"],
        [1356998400008, 7, "f0000207", "test/core/TestInternal.java:705-709"],
    ],
    "offset_from_qualifier": [
        # [qualifier hex, offset, expected ms, ref]
        ["0037", 0, 3000, "test/core/TestInternal.java:547-551"],
        ["f0000047", 0, 1, "test/core/TestInternal.java:553-557"],
        ["f0000207", 0, 8, "test/core/TestInternal.java:559-563"],
        ["f0000207f0000307", 4, 12, "test/core/TestInternal.java:565-570"],
        ["00370047", 2, 4000, "test/core/TestInternal.java:586-590"],
        ["0037f00002070047", 2, 8, "test/core/TestInternal.java:598-603"],
    ],
    "compaction": [
        # TestCompactionQueue.twoCellRow: two 8-byte longs 4, 5 at qualifiers 0x0007, 0x0017
        {"ref": "test/core/TestCompactionQueue.java:282-302",
         "cells": [["0007", "0000000000000004"], ["0017", "0000000000000005"]],
         "qualifier": "00070017", "value": "0000000000000004000000000000000500"},
    ],
}

# ---------------------------------------------------------------------------
# Scan bounds (test/core/TestTsdbQueryDownsample.java:49-125)
SCAN = [
    {"ref": "test/core/TestTsdbQueryDownsample.java:49-63", "interval": 60000, "start": 1356998400,
     "end": 1357041600, "scan_start": 1356998400, "scan_end": 1357045200},
    {"ref": "test/core/TestTsdbQueryDownsample.java:65-82", "interval": 900000, "start": 1427415547 - 43200,
     "end": 1427415547, "scan_start": 1427371200, "scan_end": 1427418000},
    {"ref": "test/core/TestTsdbQueryDownsample.java:84-102", "interval": 86400000, "start": 1427415547 - 43200,
     "end": 1427415547, "scan_start": 1427328000, "scan_end": 1427500800},
    {"ref": "test/core/TestTsdbQueryDownsample.java:104-125", "interval": 60000, "start": 1356998400000,
     "end": 1357041600000, "scan_start": 1356998400, "scan_end": 1357045200},
]

# ---------------------------------------------------------------------------
# End-to-end TsdbQuery over the MockBase-equivalent store
QUERIES = []
STORES = {}
STORE_KEYS = {}
M = "sys.cpu.user"
MB = "sys.cpu.nice"
W1 = {"host": "web01"}
W2 = {"host": "web02"}


def put(points, metric, tags, ts, kind, value):
    points.append([metric, tags, ts, kind, value])


def store_long_seconds(two_metrics, offset):  # BaseTsdbTest.java:610-639
    p = []
    ts = 1356998400
    for i in range(1, 301):
        ts += 30
        put(p, M, W1, ts, "long", i)
        if two_metrics:
            put(p, MB, W1, ts, "long", i)
    ts = 1356998415 if offset else 1356998400
    for i in range(300, 0, -1):
        ts += 30
        put(p, M, W2, ts, "long", i)
        if two_metrics:
            put(p, MB, W2, ts, "long", i)
    return p


def store_long_ms():  # BaseTsdbTest.java:641-663
    p = []
    ts = 1356998400000
    for i in range(1, 301):
        ts += 500
        put(p, M, W1, ts, "long", i)
        put(p, MB, W1, ts, "long", i)
    ts = 1356998400000
    for i in range(300, 0, -1):
        ts += 500
        put(p, M, W2, ts, "long", i)
        put(p, MB, W2, ts, "long", i)
    return p


def store_long_missing():  # BaseTsdbTest.java:674-701
    p = []
    ts = 1356998400
    for i in range(300):
        if i % 3 != 0:
            put(p, M, W1, ts, "long", i + 1)
        ts += 10
    ts = 1356998400
    for i in range(300, 0, -1):
        if i % 2 != 0:
            put(p, M, W2, ts, "long", i)
        ts += 10
    return p


def java_float_range(start, stop_incl, step, down=False):
    """for (float i = start; i <= stop (or > stop); i += step) with float arithmetic."""
    out = []
    i = f32(start)
    while (i > stop_incl) if down else (i <= stop_incl):
        out.append(i)
        i = f32(i - step) if down else f32(i + step)
    return out


def store_float_seconds(two_metrics, offset):  # BaseTsdbTest.java:703-731
    p = []
    ts = 1356998400
    for i in java_float_range(1.25, 76, 0.25):
        ts += 30
        put(p, M, W1, ts, "float", i)
        if two_metrics:
            put(p, MB, W1, ts, "float", i)
    ts = 1356998415 if offset else 1356998400
    for i in java_float_range(75, 0, 0.25, down=True):
        ts += 30
        put(p, M, W2, ts, "float", i)
        if two_metrics:
            put(p, MB, W2, ts, "float", i)
    return p


def store_mixed_seconds():  # BaseTsdbTest.java:758-772
    p = []
    ts = 1356998400
    for i in java_float_range(1.25, 76, 0.25):
        ts += 30
        if math.fmod(i, 2) == 0:
            put(p, M, W1, ts, "long", int(i))
        else:
            put(p, M, W1, ts, "float", i)
    return p


def store_mixed_ms_and_s():  # BaseTsdbTest.java:774-791
    p = []
    timestamp = 1356998400000
    for i in java_float_range(1.25, 76, 0.25):
        timestamp += 500
        ts = timestamp
        if ts % 1000 == 0:
            ts //= 1000
        if math.fmod(i, 2) == 0:
            put(p, M, W1, ts, "long", int(i))
        else:
            put(p, M, W1, ts, "float", i)
    return p


def qcase(name, ref, points, start, end, tags, fn, expect, *, rate=False, ro=None, ds=None, tol=0.0,
          check_int=True, expect_groups=None):
    key = json.dumps(points)
    sname = STORE_KEYS.setdefault(key, f"store{len(STORE_KEYS)}")
    STORES[sname] = points
    c = {"name": name, "ref": ref, "store": sname, "start": start, "end": end, "metric": M, "tags": tags,
         "aggregator": fn, "rate": rate, "rate_options": ro, "downsample": ds, "tol": tol, "check_int": check_int}
    c["expect"] = expect if expect_groups is None else expect_groups
    c["multi_group"] = expect_groups is not None
    QUERIES.append(c)


T0 = 1356998400
T1 = 1357041600
qcase("TestTsdbQueryQueries.runLongSingleTS", "test/core/TestTsdbQueryQueries.java:66-88",
      store_long_seconds(True, False), T0, T1, W1, "sum",
      [L(1356998430000 + 30000 * i, i + 1) for i in range(300)])
qcase("TestTsdbQueryQueries.runLongSingleTSMs", "test/core/TestTsdbQueryQueries.java:90-110",
      store_long_ms(), T0, T1, W1, "sum", [L(1356998400500 + 500 * i, i + 1) for i in range(300)])
qcase("TestTsdbQueryQueries.runLongTwoAggSum", "test/core/TestTsdbQueryQueries.java:125-144",
      store_long_seconds(True, False), T0, T1, {}, "sum", [L(1356998430000 + 30000 * i, 301) for i in range(300)])
qcase("TestTsdbQueryQueries.runLongTwoAggSumMs", "test/core/TestTsdbQueryQueries.java:146-165",
      store_long_ms(), T0, T1, {}, "sum", [L(1356998400500 + 500 * i, 301) for i in range(300)])
qcase("TestTsdbQueryQueries.runLongTwoGroup", "test/core/TestTsdbQueryQueries.java:167-201",
      store_long_seconds(True, False), T0, T1, {"host": "*"}, "sum", None,
      expect_groups=[[L(1356998430000 + 30000 * i, i + 1) for i in range(300)],
                     [L(1356998430000 + 30000 * i, 300 - i) for i in range(300)]])
qcase("TestTsdbQueryQueries.runLongSingleTSRate", "test/core/TestTsdbQueryQueries.java:203-221",
      store_long_seconds(True, False), T0, T1, W1, "sum",
      [D(1356998460000 + 30000 * i, f32(0.033)) for i in range(299)], rate=True, tol=0.001, check_int=True)
qcase("TestTsdbQueryQueries.runLongSingleTSRateMs", "test/core/TestTsdbQueryQueries.java:223-241",
      store_long_ms(), T0, T1, W1, "sum", [D(1356998401000 + 500 * i, 2.0) for i in range(299)], rate=True,
      tol=0.001)
FV = java_float_range(1.25, 76, 0.25)
qcase("TestTsdbQueryQueries.runFloatSingleTS", "test/core/TestTsdbQueryQueries.java:243-263",
      store_float_seconds(True, False), T0, T1, W1, "sum",
      [D(1356998430000 + 30000 * i, 1.25 + 0.25 * i) for i in range(300)], tol=0.001)
qcase("TestTsdbQueryQueries.runFloatTwoAggSum", "test/core/TestTsdbQueryQueries.java:287-306",
      store_float_seconds(True, False), T0, T1, {}, "sum", [D(1356998430000 + 30000 * i, 76.25) for i in range(300)],
      tol=0.00001)
qcase("TestTsdbQueryQueries.runFloatTwoGroup", "test/core/TestTsdbQueryQueries.java:364-397",
      store_float_seconds(True, False), T0, T1, {"host": "*"}, "sum", None, tol=0.0001,
      expect_groups=[[D(1356998430000 + 30000 * i, 1.25 + 0.25 * i) for i in range(300)],
                     [D(1356998430000 + 30000 * i, 75 - 0.25 * i) for i in range(300)]])
qcase("TestTsdbQueryQueries.runFloatSingleTSRate", "test/core/TestTsdbQueryQueries.java:399-417",
      store_float_seconds(True, False), T0, T1, W1, "sum",
      [D(1356998460000 + 30000 * i, f32(0.00833)) for i in range(299)], rate=True, tol=0.00001)


def mixed_expect(ts0, step):  # TestTsdbQueryQueries.runMixedSingleTS loop (:475-490)
    out = []
    fv, iv = 1.25, 76
    for k in range(300):
        ts = ts0 + step * k
        if k == 299:
            out.append(L(ts, iv))
        else:
            out.append(D(ts, fv))
            fv += 0.25
    return out


qcase("TestTsdbQueryQueries.runMixedSingleTS", "test/core/TestTsdbQueryQueries.java:462-492",
      store_mixed_seconds(), T0, T1, W1, "avg", mixed_expect(1356998430000, 30000), tol=0.001)
qcase("TestTsdbQueryQueries.runMixedSingleTSMsAndS", "test/core/TestTsdbQueryQueries.java:494-524",
      store_mixed_ms_and_s(), T0, T1, W1, "avg", mixed_expect(1356998400500, 500), tol=0.001)


def rate_pts(vals, start=1356998400):
    p = []
    ts = start
    for v in vals:
        ts += 30
        put(p, M, W1, ts, "long", v)
    return p


qcase("TestTsdbQueryQueries.runRateCounterDefault", "test/core/TestTsdbQueryQueries.java:1125-1149",
      rate_pts([LONG_MAX - 55, LONG_MAX - 25, 5]), T0, T1, W1, "sum",
      [D(1356998460000, 1.0), D(1356998490000, 1.0)], rate=True, ro=[True, LONG_MAX, 0, False], tol=0.001)
qcase("TestTsdbQueryQueries.runRateCounterDefaultNoOp", "test/core/TestTsdbQueryQueries.java:1151-1173",
      rate_pts([30, 60, 90]), T0, T1, W1, "sum", [D(1356998460000, 1.0), D(1356998490000, 1.0)], rate=True,
      ro=[True, LONG_MAX, 0, False], tol=0.001)
qcase("TestTsdbQueryQueries.runRateCounterMaxSet", "test/core/TestTsdbQueryQueries.java:1175-1197",
      rate_pts([45, 75, 5]), T0, T1, W1, "sum", [D(1356998460000, 1.0), D(1356998490000, 1.0)], rate=True,
      ro=[True, 100, 0, False], tol=0.001)
qcase("TestTsdbQueryQueries.runRateCounterAnomally", "test/core/TestTsdbQueryQueries.java:1199-1219",
      rate_pts([45, 75, 25]), T0, T1, W1, "sum", [D(1356998460000, 1.0), D(1356998490000, 0.0)], rate=True,
      ro=[True, 10000, 35, False], tol=0.001)
qcase("TestTsdbQueryQueries.runRateCounterAnomallyDrop", "test/core/TestTsdbQueryQueries.java:1221-1243",
      rate_pts([45, 75, 25, 55]), T0, T1, W1, "sum", [D(1356998460000, 1.0), D(1356998520000, 1.0)], rate=True,
      ro=[True, 10000, 35, True], tol=0.001)


def interp_expect(ts0, step, reset_ts):  # runInterpolationSeconds loop (:1371-1388)
    out = []
    v = 1
    ts = ts0
    for _ in range(600):
        out.append(L(ts, v))
        if ts == reset_ts:
            v = 1
        elif v == 1 or v == 302:
            v = 301
        else:
            v = 302
        ts += step
    return out


p = []
ts = 1356998400
for i in range(1, 301):
    ts += 30
    put(p, M, W1, ts, "long", i)
ts = 1356998415
for i in range(300, 0, -1):
    ts += 30
    put(p, M, W2, ts, "long", i)
qcase("TestTsdbQueryQueries.runInterpolationSeconds", "test/core/TestTsdbQueryQueries.java:1351-1390",
      p, T0, T1, {}, "sum", interp_expect(1356998430000, 15000, 1357007400000))
p = []
ts = 1356998400000
for i in range(1, 301):
    ts += 500
    put(p, M, W1, ts, "long", i)
ts = 1356998400250
for i in range(300, 0, -1):
    ts += 500
    put(p, M, W2, ts, "long", i)
qcase("TestTsdbQueryQueries.runInterpolationMs", "test/core/TestTsdbQueryQueries.java:1392-1431",
      p, T0, T1, {}, "sum", interp_expect(1356998400500, 250, 1356998550000))
p = []
ts = 1356998400000
for i in range(1, 121):
    ts += 500 if i <= 100 else 5000
    put(p, M, W1, ts, "long", i)
ts = 1356998400250
for i in range(300, 0, -1):
    ts += 500
    put(p, M, W2, ts, "long", i)
exp = []
for i in range(151):
    if i == 0:
        v = 301.0
    elif i < 50:
        v = 602.0
    else:
        v = 701 + (i - 50) * 0.2 - i * 4
    exp.append(D(1356998400000 + 1000 * i, v))
qcase("TestTsdbQueryQueries.runInterpolationMsDownsampled", "test/core/TestTsdbQueryQueries.java:1433-1514",
      p, T0, T1, {}, "sum", exp, ds=["1000ms", "sum", "none"], tol=1e-7)

# TestTsdbQueryDownsample
exp = []
for i in range(151):
    v = 1.0 if i == 0 else (300.0 if i >= 150 else i * 2 + 0.5)
    exp.append(D(1356998400000 + 60000 * i, v))
qcase("TestTsdbQueryDownsample.runLongSingleTSDownsample", "test/core/TestTsdbQueryDownsample.java:137-172",
      store_long_seconds(True, False), T0, T1, W1, "sum", exp, ds=["60000ms", "avg", "none"], tol=0.00001)
exp = [D(1356998460000 + 60000 * i, 0.025 if (i == 0 or i >= 149) else 2 / 60.0) for i in range(150)]
qcase("TestTsdbQueryDownsample.runLongSingleTSDownsampleAndRate", "test/core/TestTsdbQueryDownsample.java:211-248",
      store_long_seconds(True, False), T0, T1, W1, "sum", exp, ds=["60000ms", "avg", "none"], rate=True, tol=0.001)
exp = [D(1356998400000 + 60000 * i, 1.0 if i in (0, 150) else 2.0) for i in range(151)]
qcase("TestTsdbQueryDownsample.runLongSingleTSDownsampleCount", "test/core/TestTsdbQueryDownsample.java:436-462",
      store_long_seconds(True, False), T0, T1, W1, "sum", exp, ds=["60000ms", "count", "none"], tol=0.00001)
qcase("TestTsdbQueryDownsample.runLongSingleTSDownsampleAll", "test/core/TestTsdbQueryDownsample.java:464-495",
      store_long_seconds(True, False), T0 * 1000, T1 * 1000, W1, "sum", [D(1356998400000, 45150)],
      ds=["0all", "sum", "none"], tol=0.00001)
qcase("TestTsdbQueryDownsample.runLongSingleTSDownsampleAllSubSet",
      "test/core/TestTsdbQueryDownsample.java:497-528",
      store_long_seconds(True, False), 1356998500000, 1356998600000, W1, "sum", [D(1356998500000, 15)],
      ds=["0all", "sum", "none"], tol=0.00001)
exp = [D(1356998460000 + 60000 * i, f32(0.016666) if i == 0 else (f32(-0.016666) if i == 149 else 0.0))
       for i in range(150)]
qcase("TestTsdbQueryDownsample.runFloatSingleTSDownsampleAndRateAndCount",
      "test/core/TestTsdbQueryDownsample.java:563-598",
      store_float_seconds(True, False), T0, T1, W1, "sum", exp, ds=["60000ms", "count", "none"], rate=True,
      tol=0.00001)


def wnulls_expect(values, missing):
    """runTSDownsampleWithMissingData (:860-909): 100 valid values, then the fill value,
    (end - start + 3600) / 30 points from the scan start."""
    n = (1357041600 - 1356998400 + 3600) // 30
    out = []
    for i in range(n):
        out.append(D(1356998400000 + 30000 * i, values[i] if i < 100 else missing))
    return out


def alt(fn_even, fn_odd, n=100):
    out = []
    for k in range(n):
        out.append(fn_even(k // 2) if k % 2 == 0 else fn_odd(k // 2))
    return out


NULLS = [
    ("runSumAvgLongSingleTSDownsampleWNulls", "sum", "avg", "nan", [301.5] * 100, ":677-689"),
    ("runAvgSumLongSingleTSDownsampleWNulls", "avg", "sum", "nan",
     alt(lambda j: 152.0 + 3 * j, lambda j: 301.5), ":691-712"),
    ("runAvgAvgLongSingleTSDownsampleWNulls", "avg", "avg", "zero", [150.75] * 100, ":714-726"),
    ("runSumSumLongSingleTSDownsampleWNulls", "sum", "sum", "nan",
     alt(lambda j: 304.0 + 6 * j, lambda j: 603.0), ":728-750"),
    ("runSumMinLongSingleTSDownsampleWNulls", "sum", "min", "nan", alt(lambda j: 301.0, lambda j: 300.0), ":839-857"),
]


def minmin_values():  # runMinMinLongSingleTSDownsampleWNulls validator (:752-794)
    out = []
    ee, ec, oe, oc = -4.0, 6.0, -1.0, 6.0
    even = False
    for _ in range(100):
        even = not even
        if even:
            ee += ec
            if abs(ee - 152.0) < 1e-4:
                ee, ec = 149.0, -6.0
            out.append(ee)
        else:
            oe += oc
            if abs(oe - 155.0) < 1e-4:
                oe, oc = 145.0, -6.0
            out.append(oe)
    return out


def minsum_values():  # runMinSumLongSingleTSDownsampleWNulls validator (:796-837)
    out = []
    ee, ec, oe, oc = -7.0, 12.0, -1.0, 12.0
    even = False
    for _ in range(100):
        even = not even
        if even:
            ee += ec
            if abs(ee - 209.0) < 1e-4:
                ee, ec = 197.0, -6.0
            out.append(ee)
        else:
            oe += oc
            if abs(oe - 311.0) < 1e-4:
                oe, oc = 292.0, -12.0
            out.append(oe)
    return out


NULLS += [("runMinMinLongSingleTSDownsampleWNulls", "min", "min", "zero", minmin_values(), ":752-794"),
          ("runMinSumLongSingleTSDownsampleWNulls", "min", "sum", "nan", minsum_values(), ":796-837")]
for name, qa, da, fill, values, lines in NULLS:
    missing = float("nan") if fill == "nan" else 0.0
    qcase(f"TestTsdbQueryDownsample.{name}", f"test/core/TestTsdbQueryDownsample.java{lines}",
          store_long_missing(), T0, T1, {}, qa, wnulls_expect(values, missing), ds=["30000ms", da, fill], tol=0.0001)

# TestTsdbQueryAggregators (test/core/TestTsdbQueryAggregators.java)
qcase("TestTsdbQueryAggregators.runZimSum", "test/core/TestTsdbQueryAggregators.java:43-61",
      store_long_seconds(False, False), T0, T1, {}, "zimsum", [L(1356998430000 + 30000 * i, 301) for i in range(300)])
qcase("TestTsdbQueryAggregators.runZimSumFloat", "test/core/TestTsdbQueryAggregators.java:63-81",
      store_float_seconds(False, False), T0, T1, {}, "zimsum", [D(1356998430000 + 30000 * i, 76.25) for i in range(300)],
      tol=0.001)
exp = []
v1, v2 = 1, 300
for c in range(600):
    exp.append(L(1356998430000 + 15000 * c, v1 if c % 2 == 0 else v2))
    if c % 2 == 0:
        v1 += 1
    else:
        v2 -= 1
qcase("TestTsdbQueryAggregators.runZimSumOffset", "test/core/TestTsdbQueryAggregators.java:83-111",
      store_long_seconds(False, True), T0, T1, {}, "zimsum", exp)
exp = []
v, dec = 1, False
for i in range(300):
    exp.append(L(1356998430000 + 30000 * i, v))
    v = v - 1 if dec else v + 1
    if v == 151:
        v, dec = 150, True
qcase("TestTsdbQueryAggregators.runMin", "test/core/TestTsdbQueryAggregators.java:201-232",
      store_long_seconds(False, False), T0, T1, {}, "min", exp)
exp = []
v, dec, counter = 1, False, 0
for i in range(600):
    exp.append(L(1356998430000 + 15000 * i, v))
    if counter % 2 != 0:
        v = v - 1 if dec else v + 1
    elif v == 151:
        v, dec = 150, True
        counter -= 1
    counter += 1
qcase("TestTsdbQueryAggregators.runMinOffset", "test/core/TestTsdbQueryAggregators.java:267-300",
      store_long_seconds(False, True), T0, T1, {}, "min", exp)
exp = []
v, dec, counter = 1, True, 0
for i in range(600):
    ts = 1356998430000 + 15000 * i
    exp.append(L(ts, v))
    if v == 1:
        v = 300
    elif ts == 1357007400000:
        v = 1
    elif counter % 2 == 0:
        v = v - 1 if dec else v + 1
    if v == 150:
        v, dec = 151, False
        counter -= 1
    counter += 1
qcase("TestTsdbQueryAggregators.runMaxOffset", "test/core/TestTsdbQueryAggregators.java:400-439",
      store_long_seconds(False, True), T0, T1, {}, "max", exp)


def main():
    out = {
        "iterators.json": {"source": "reference unit tests (iterator level)", "cases": ITER},
        "aggregators.json": {"source": "test/core/TestAggregators.java", "cases": AGGS},
        "codec.json": CODEC,
        "scan_bounds.json": {"cases": SCAN},
        "queries.json": {"source": "end-to-end TsdbQuery over MockBase", "stores": STORES, "cases": QUERIES},
    }
    for fname, obj in out.items():
        with open(os.path.join(HERE, fname), "w") as f:
            json.dump(obj, f, separators=(",", ":"), allow_nan=True)
        print(fname, len(obj.get("cases", [])) if isinstance(obj, dict) else "")


if __name__ == "__main__":
    main()
