"""Transcribes known answers of the reference's expression-function tests
into tests/golden/expression.json.

Inputs are the tests' SeekableViewsForTest.generator series (test/core/SeekableViewsForTest.java:
84-210: integers start + i * (long) increment, doubles by repeated addition of the increment), at
START_TIME 1356998400000, INTERVAL 60000, NUM_POINTS 5; expected outputs are the values the tests
assert (their loops evaluated here), with the test's tolerance.

  test/query/expression/TestScale.java ......... evaluateFactor* (6)
  test/query/expression/TestAbsolute.java ...... evaluate*GroupBy* (4)
  test/query/expression/TestAlias.java ......... evaluate* (3)
  test/query/expression/TestMovingAverage.java . evaluateWindow* (9) and evaluateGroupBy
  test/query/expression/TestSumSeries.java / TestDiffSeries.java / TestMultiplySeries.java /
  TestDivideSeries.java ........................ *OneSeriesEach (4)
  test/query/expression/TestTimeShift.java ..... parseParam, shiftDataPoint
  test/query/expression/TestHighestMax.java / TestHighestCurrent.java .. evaluate* (which series,
                                                 in which order; the tests then check that the
                                                 series come back unchanged)

    python tests/golden/make_expression_golden.py
"""
from __future__ import annotations

import json
import os

START, INTERVAL, N = 1356998400000, 60000, 5
D = "test/query/expression/"


def gen(is_int, start, inc, n=N, t0=START, period=INTERVAL):
    out, v = [], (int(start) if is_int else float(start))
    for i in range(n):
        out.append([t0 + i * period, v])
        v = v + (int(inc) if is_int else inc)
    return out


def main():
    cases = []

    def add(name, src, fn, inputs, params, expect, tol=0.0, **kw):
        cases.append({"name": name, "source": D + src, "fn": fn, "inputs": inputs, "params": params,
                      "expect": expect, "tol": tol, **kw})

    ts = [START + i * INTERVAL for i in range(N)]
    a = gen(True, 1, 1)
    # Scale: results[i] over the group-bys {dps, dps2}; ints stay ints for integral factors
    add("evaluateFactor1GroupByLong", "TestScale.java:82-118", "scale", [[a, gen(True, 10, 1)]], ["1"],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, v] for t, v in zip(ts, range(10, 15))]])
    add("evaluateFactor1GroupByDouble", "TestScale.java:120-156", "scale", [[a, gen(False, 10, 1.5)]], ["1"],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, 10 + 1.5 * i] for i, t in enumerate(ts)]], tol=0.001)
    add("evaluateFactor1point5GroupBy", "TestScale.java:158-195", "scale", [[a, gen(True, 10, 1)]], ["1.5"],
        [[[t, 1.5 * (i + 1)] for i, t in enumerate(ts)], [[t, 15 + 1.5 * i] for i, t in enumerate(ts)]], tol=0.001)
    add("evaluateFactor1024GroupBy", "TestScale.java:197-233", "scale", [[a, gen(True, 10, 1)]], ["1024"],
        [[[t, 1024 * (i + 1)] for i, t in enumerate(ts)], [[t, 10240 + 1024 * i] for i, t in enumerate(ts)]])
    add("evaluateFactor0GroupByLong", "TestScale.java:273-306", "scale", [[a, gen(True, 10, 1)]], ["0"],
        [[[t, 0] for t in ts], [[t, 0] for t in ts]])
    add("evaluateFactorNegative1GroupByLong", "TestScale.java:307-343", "scale", [[a, gen(True, 10, 1)]], ["-1"],
        [[[t, -(i + 1)] for i, t in enumerate(ts)], [[t, -10 - i] for i, t in enumerate(ts)]])
    # Absolute
    add("evaluatePositiveGroupByLong", "TestAbsolute.java:83-119", "absolute", [[a, gen(True, 10, 1)]], [],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, v] for t, v in zip(ts, range(10, 15))]])
    add("evaluatePositiveGroupByDouble", "TestAbsolute.java:120-156", "absolute", [[a, gen(False, 10, 1)]], [],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, 10.0 + i] for i, t in enumerate(ts)]], tol=0.001)
    add("evaluateFactorNegativeGroupByLong", "TestAbsolute.java:157-193", "absolute", [[a, gen(True, -10, -1)]], [],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, v] for t, v in zip(ts, range(10, 15))]])
    add("evaluateNegativeGroupByDouble", "TestAbsolute.java:194-230", "absolute", [[a, gen(False, -10, -1)]], [],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, 10.0 + i] for i, t in enumerate(ts)]], tol=0.001)
    # Alias: renamed, and the absolute value of every point (Alias.java's loop is Absolute's)
    add("aliasGroupByLong", "TestAlias.java:96-132", "alias", [[a, gen(True, 10, 1)]], ["My Alias"],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, v] for t, v in zip(ts, range(10, 15))]], alias_name="My Alias")
    add("aliasGroupByDouble", "TestAlias.java:134-171", "alias", [[a, gen(False, 10, 1)]], ["My Alias"],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, 10.0 + i] for i, t in enumerate(ts)]], tol=0.001,
        alias_name="My Alias")
    add("aliasSubQuerySeries", "TestAlias.java:172-208", "alias", [[a], [gen(True, -10, -1)]], ["My Alias"],
        [[[t, v] for t, v in zip(ts, range(1, 6))], [[t, v] for t, v in zip(ts, range(10, 15))]], alias_name="My Alias")
    # MovingAverage over [START, START + INTERVAL * N] (the mocked TSQuery)
    win = {
        "evaluateWindow1dps": ("1", "TestMovingAverage.java:81-99", [1, 2, 3, 4, 5]),
        "evaluateWindow2dps": ("2", "TestMovingAverage.java:101-123", [0, 1.5, 2.5, 3.5, 4.5]),
        "evaluateWindow5dps": ("5", "TestMovingAverage.java:125-145", [0, 0, 0, 0, 3.0]),
        "evaluateWindow6dps": ("6", "TestMovingAverage.java:147-162", [0, 0, 0, 0, 0]),
        "evaluateWindow1min": ("'1min'", "TestMovingAverage.java:164-185", [0, 2, 3, 4, 5]),
        "evaluateWindow2min": ("'2min'", "TestMovingAverage.java:187-208", [0, 0, 2.5, 3.5, 4.5]),
        "evaluateWindow3min": ("'3min'", "TestMovingAverage.java:210-232", [0, 0, 0, 3, 4]),
        "evaluateWindow4min": ("'4min'", "TestMovingAverage.java:234-252", [0, 0, 0, 0, 3.5]),
        "evaluateWindow5min": ("'5min'", "TestMovingAverage.java:254-269", [0, 0, 0, 0, 0]),
    }
    for name, (p, src, vals) in win.items():
        add(name, src, "movingAverage", [[a]], [p], [[[t, float(v)] for t, v in zip(ts, vals)]], tol=0.001,
            start=START, end=START + INTERVAL * N)
    add("evaluateGroupBy", "TestMovingAverage.java:271-303", "movingAverage", [[a, gen(True, 10, 1)]], ["1"],
        [[[t, float(v)] for t, v in zip(ts, range(1, 6))], [[t, float(v)] for t, v in zip(ts, range(10, 15))]],
        tol=0.001, start=START, end=START + INTERVAL * N)
    # series combinations: one series per sub-query (same empty tags: one joined set)
    b = gen(True, 10, 1)
    add("sumOneSeriesEach", "TestSumSeries.java:80-104", "sumSeries", [[a], [b]], [],
        [[[t, 11.0 + 2 * i] for i, t in enumerate(ts)]], tol=0.001)
    add("diffOneSeriesEach", "TestDiffSeries.java:80-102", "diffSeries", [[a], [b]], [],
        [[[t, -9.0] for t in ts]], tol=0.001)
    add("multiplyOneSeriesEach", "TestMultiplySeries.java:80-103", "multiplySeries", [[a], [b]], [],
        [[[t, float(v)] for t, v in zip(ts, [10, 22, 36, 52, 70])]], tol=0.001)
    add("divideOneSeriesEach", "TestDivideSeries.java:80-103", "divideSeries", [[a], [b]], [],
        [[[t, v] for t, v in zip(ts, [0.1, 0.181, 0.25, 0.307, 0.357])]], tol=0.001)
    # TimeShift.parseParam / shift(DataPoint, ms)
    parse = [["+1week ", 7 * 86400000], ["+1days ", 86400000], ["+1hr ", 3600000], ["+1min ", 60000],
             ["+1sec ", 1000], ["+1 week ", 7 * 86400000], ["+1 days ", 86400000], ["+1 hr ", 3600000],
             ["+1 min ", 60000], ["+1 sec ", 1000], ["+1week", 7 * 86400000], ["+1days", 86400000],
             ["+1hr", 3600000], ["+1min", 60000], ["+1sec", 1000], ["+1 week", 7 * 86400000],
             ["+1 days", 86400000], ["+1 hr", 3600000], ["+1 min", 60000], ["+1 sec", 1000]]
    shift = {"source": D + "TestTimeShift.java:72-80",
             "points": [[1356998400000, 40], [1356998400000 + 2000000, 50]],
             "cases": [[0, 60000, 1356998460000], [1, 7 * 86400000, 1357605200000], [1, 130 * 86400000, 1368232400000]]}
    # highestMax / highestCurrent: dps = ints 1..5 (METRIC), the TSQuery over [START, START + 5 I]
    topn = []
    end = START + INTERVAL * N

    def gen_mixed(start, inc):   # generator(..., false, start, inc, wholes_as_integer=true)
        out, v = [], float(start)
        for i in range(N):
            out.append([START + i * INTERVAL, int(v) if v == int(v) else v])
            v += inc
        return out

    for fn, src in [("highestMax", "TestHighestMax.java"), ("highestCurrent", "TestHighestCurrent.java")]:
        def addt(name, lines, inputs, params, expect=None, raises=None):
            topn.append({"name": f"{fn}.{name}", "source": D + src + ":" + lines, "fn": fn, "inputs": inputs,
                         "params": params, "start": START, "end": end, "expect_index": expect, "raises": raises})
        b = gen(True, 10, 1)
        addt("evaluateTopN1with2SeriesLong", "83-108", [[a, b]], ["1"], [1])
        addt("evaluateTopN2with2SeriesLong", "111-147", [[a, b]], ["2"], [1, 0])
        addt("evaluateTopN100with2SeriesLong", "150-185", [[a, b]], ["100"], [1, 0])
        addt("evaluateTopN100with2SubQuerySeriesLong", "188-224", [[a], [b]], ["100"], [1, 0])
        addt("evaluateTopN2with2SeriesDouble", "227-263", [[a, gen(False, 10, 1.5)]], ["2"], [1, 0])
        addt("evaluateTopN1with2SeriesLongDoubleMixed", "266-298", [[a, gen_mixed(10, 1.5)]], ["1"], [1])
        if fn == "highestCurrent":
            addt("evaluateTopN1with2SeriesDiffSpan", "301-328", [[a, gen(True, 10, 1, n=3)]], ["1"], [0])
        addt("evaluateNullResults", "337-341", [], ["1"], [])
        addt("evaluateEmptyResults", "349-354", [[]], ["1"], [])
        for nm, prm in [("evaluateNullParams", None), ("evaluateEmptyParams", []), ("evaluateTopnNull", [None]),
                        ("evaluateTopnEmpty", [""]), ("evaluateTopnZero", ["0"]),
                        ("evaluateTopnNotaNumber", ["not a number"])]:
            addt(nm, "343-380", [[a]], prm, None, "IllegalArgumentException")
    out = {"cases": cases, "timeshift_parse": {"source": D + "TestTimeShift.java:47-70", "cases": parse},
           "timeshift_shift": shift, "topn": topn}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "expression.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{path}: {len(cases)} cases, {len(parse)} parseParam answers, {len(topn)} top-n cases")


if __name__ == "__main__":
    main()
