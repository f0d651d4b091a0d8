"""Transcribes the known answers of the reference's /api/query/exp join tests (SURVEY.md 8f row
f4) into tests/golden/expression_iter.json:

  test/query/expression/TestUnionIterator.java ........ 37 tests (22 iteration, 13 flattenTags, 2 ctor)
  test/query/expression/TestIntersectionIterator.java . 36 tests (21 iteration, 13 flattenTags, 2 ctor)
  test/query/expression/TestExpressionIterator.java ... 34 tests (expressions over INTERSECTION /
                                                        UNION joins, fills, nested expressions,
                                                        per-series iteration, the constructor checks)

Inputs: the MockBase stores of test/query/expression/BaseTimeSyncedIteratorTest.java (metrics A and
B, tags D / E / Z, UIDs 'A'..'Z' -> 00 00 0A.. as test/core/BaseTsdbTest.java:102-110 assigns them),
queried as its queryAB_Dstar / queryAB_AggAll / queryA_DD do (sum, group by D or by nothing, start
1388534400).  Each query result is written out as the tests' iterators see it: per sub-query the
group-by series in group-key order, their points (spans summed per timestamp -- every group of
these stores has aligned spans), the group's tags and aggregated tags (SpanGroup.computeTags) and
the sub-query's filter tagks.  Points a test writes with tsdb.addPoint AFTER runQueries are not
in the results (the spans were scanned already); those tests keep their extra-point names.

Expected outputs are the values the tests assert, their loops evaluated here (tolerance 0.0001 as
the tests use), or the exception the test expects.

    python tests/golden/make_expression_iter_golden.py
"""
from __future__ import annotations

import json
import os

D = "test/query/expression/"
BASE = D + "BaseTimeSyncedIteratorTest.java"
T0 = 1431561600
TS0 = T0 * 1000
NAN = "NaN"


def uid(letter):   # test/core/BaseTsdbTest.java:102-110
    return [0, 0, 10 + ord(letter) - ord("A")]


def pts(*vals, start=T0, step=60):
    return [[start + i * step, v] for i, v in enumerate(vals)]


# ---- the stores (BaseTimeSyncedIteratorTest.java) -------------------------------------------
STORES = {
    "empty": {"src": "BaseTsdbTest.setDataPointStorage", "series": []},
    "twoSeriesAggedE": {"src": BASE + ":147-178", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "D", "E": "F"}, pts(1, 2, 3)],
        ["B", {"D": "D", "E": "E"}, pts(11, 12, 13)], ["B", {"D": "D", "E": "F"}, pts(11, 12, 13)]]},
    "twoSeriesAggedEandExtraTagK": {"src": BASE + ":184-217", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "D", "E": "F"}, pts(1, 2, 3)],
        ["B", {"D": "D", "E": "E", "Z": "A"}, pts(11, 12, 13)], ["B", {"D": "D", "E": "F", "Z": "B"}, pts(11, 12, 13)]]},
    "oneAggedTheOtherTagged": {"src": BASE + ":223-248", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "E", "E": "F"}, pts(1, 2, 3)],
        ["B", {"D": "D", "E": "E"}, pts(11, 12, 13)]]},
    "threeSameENoB": {"src": BASE + ":253-276", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "F", "E": "E"}, pts(4, 5, 6)],
        ["A", {"D": "G", "E": "E"}, pts(7, 8, 9)]]},
    "oneExtraSameE": {"src": BASE + ":281-319", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "F", "E": "E"}, pts(4, 5, 6)],
        ["B", {"D": "D", "E": "E"}, pts(11, 12, 13)], ["B", {"D": "F", "E": "E"}, pts(14, 15, 16)],
        ["B", {"D": "G", "E": "E"}, pts(17, 18, 19)]]},
    "timeOffset": {"src": BASE + ":326-352", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2)], ["A", {"D": "F", "E": "E"}, pts(4, 5)],
        ["B", {"D": "D", "E": "E"}, pts(13, 14, start=T0 + 120)], ["B", {"D": "F", "E": "E"}, pts(16, 17, start=T0 + 120)]]},
    "threeSameE": {"src": BASE + ":357-401", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "F", "E": "E"}, pts(4, 5, 6)],
        ["A", {"D": "G", "E": "E"}, pts(7, 8, 9)],
        ["B", {"D": "D", "E": "E"}, pts(11, 12, 13)], ["B", {"D": "F", "E": "E"}, pts(14, 15, 16)],
        ["B", {"D": "G", "E": "E"}, pts(17, 18, 19)]]},
    "threeAMissingE": {"src": BASE + ":407-447", "series": [
        ["A", {"D": "D"}, pts(1, 2, 3)], ["A", {"D": "F"}, pts(4, 5, 6)], ["A", {"D": "G"}, pts(7, 8, 9)],
        ["B", {"D": "D", "E": "E"}, pts(11, 12, 13)], ["B", {"D": "F", "E": "E"}, pts(14, 15, 16)],
        ["B", {"D": "G", "E": "E"}, pts(17, 18, 19)]]},
    "threeDifE": {"src": BASE + ":452-495", "series": [
        ["A", {"D": "D", "E": "A"}, pts(1, 2, 3)], ["A", {"D": "F", "E": "B"}, pts(4, 5, 6)],
        ["A", {"D": "G", "E": "C"}, pts(7, 8, 9)],
        ["B", {"D": "D", "E": "D"}, pts(11, 12, 13)], ["B", {"D": "F", "E": "F"}, pts(14, 15, 16)],
        ["B", {"D": "G", "E": "G"}, pts(17, 18, 19)]]},
    "threeDisjointSameE": {"src": BASE + ":501-547", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "F", "E": "E"}, pts(4, 5, 6)],
        ["A", {"D": "G", "E": "E"}, pts(7, 8, 9)],
        ["B", {"D": "D", "E": "E"}, pts(11, 12, 13)], ["B", {"D": "Q", "E": "E"}, pts(14, 15, 16)],
        ["B", {"D": "G", "E": "E"}, pts(17, 18, 19)]]},
    "reduceToOne": {"src": BASE + ":553-599", "series": [
        ["A", {"D": "D", "E": "E"}, pts(1, 2, 3)], ["A", {"D": "F", "E": "E"}, pts(4, 5, 6)],
        ["A", {"D": "G", "E": "E"}, pts(7, 8, 9)],
        ["B", {"D": "P", "E": "E"}, pts(11, 12, 13)], ["B", {"D": "Q", "E": "E"}, pts(14, 15, 16)],
        ["B", {"D": "G", "E": "E"}, pts(17, 18, 19)]]},
    "threeSameEGaps": {"src": BASE + ":605-649", "series": [
        ["A", {"D": "D", "E": "E"}, [[T0, 1], [T0 + 120, 3]]], ["A", {"D": "F", "E": "E"}, [[T0, 4], [T0 + 60, 5]]],
        ["A", {"D": "G", "E": "E"}, [[T0 + 60, 8], [T0 + 120, 9]]],
        ["B", {"D": "D", "E": "E"}, [[T0 + 120, 13]]], ["B", {"D": "F", "E": "E"}, [[T0 + 60, 15]]],
        ["B", {"D": "G", "E": "E"}, [[T0 + 120, 19]]]]},
}

# queryAB_Dstar / queryAB_AggAll / queryA_DD (BaseTimeSyncedIteratorTest.java:48-112): sum,
# `D=*` groups by D, no tags -> one group, `D=D` filters and groups by D
QUERIES = {
    "AB_Dstar": {"src": BASE + ":48-70", "subs": [["A", "D", None], ["B", "D", None]]},
    "AB_AggAll": {"src": BASE + ":75-95", "subs": [["A", None, None], ["B", None, None]]},
    "A_DD": {"src": BASE + ":100-112", "subs": [["A", "D", "D"]]},
}


def compute_tags(span_tags):   # SpanGroup.computeTags (src/core/SpanGroup.java:350-389)
    tag_set, discards = {}, set()
    for tags in span_tags:
        for k in sorted(tags, key=uid):
            if k in discards:
                continue
            if k not in tag_set:
                tag_set[k] = tags[k]
            elif tag_set[k] != tags[k]:
                discards.add(k)
                del tag_set[k]
    return tag_set, sorted(discards, key=uid)


def run_query(store, query):
    """The TSQuery's DataPoints[] per sub-query: groups in group-key order, points summed."""
    out = []
    for metric, groupby, literal in QUERIES[query]["subs"]:
        spans = [s for s in STORES[store]["series"] if s[0] == metric and (literal is None or s[1].get(groupby) == literal)]
        groups = {}
        for s in spans:
            key = s[1].get(groupby) if groupby else ""
            groups.setdefault(key, []).append(s)
        series = []
        for key in sorted(groups, key=lambda k: uid(k) if k else []):
            g = groups[key]
            tss = [p[0] for p in g[0][2]]
            assert all([p[0] for p in s[2]] == tss for s in g), "unaligned group"
            points = [[t * 1000, sum(s[2][i][1] for s in g)] for i, t in enumerate(tss)]
            tags, agg = compute_tags([s[1] for s in g])
            series.append({"points": points, "tags": tags, "agg": agg})
        out.append({"metric": metric, "filter_tagks": [groupby] if groupby else [], "series": series})
    return out


def steps(n, fn):
    """n synchronised steps of a test loop: fn(k) -> the asserted arrays at step k."""
    return [{"ts": TS0 + k * 60000, **fn(k)} for k in range(n)]


def main():
    cases = []

    def add(name, src, **kw):
        if "store" in kw and "query" in kw and kw["query"]:
            kw["results"] = run_query(kw["store"], kw["query"])
        cases.append({"name": name, "source": D + src, "tol": 1e-4, **kw})

    # ---- UnionIterator -------------------------------------------------------------------
    U = "TestUnionIterator.java"
    J = dict(kind="union", fill=NAN)   # runQueries sets NOT_A_NUMBER on every sub iterator

    add("union.ctorNullResults", U + ":74-77", kind="union", error="NullPointerException", null_results=True)
    add("union.ctorEmptyResults", U + ":79-85", kind="union", store="empty", query=None, use_qt=True,
        inc_agg=True, series_size=0, has_next=False)
    add("union.twoAndThreeSeries", U + ":87-122", store="oneExtraSameE", query="AB_Dstar", use_qt=False, inc_agg=False,
        series_size=3, steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 0], "1": [11 + k, 14 + k, 17 + k]}), **J)
    add("union.twoAndThreeSeriesExtraDP", U + ":124-164", store="oneExtraSameE", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=3,
        steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 0], "1": [11 + k, 14 + k, 17 + k]}), **J)
    add("union.threeSeriesUnionToFour", U + ":166-206", store="threeDisjointSameE", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=4,
        steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 7 + k, 0], "1": [11 + k, 0, 17 + k, 14 + k]}), **J)
    add("union.threeSeriesUnionToExtraDPs", U + ":208-262", store="reduceToOne", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=5,
        steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 7 + k, 0, 0], "1": [0, 0, 17 + k, 11 + k, 14 + k]}), **J)
    add("union.threeSeriesAgged", U + ":264-295", store="threeSameE", query="AB_AggAll", use_qt=False, inc_agg=False,
        series_size=1, steps=steps(3, lambda k: {"0": [12 + 3 * k], "1": [42 + 3 * k]}), **J)
    nan_steps = [
        {"ts": TS0, "0": [1, 4, NAN], "1": [NAN, NAN, NAN]},
        {"ts": TS0 + 60000, "0": [NAN, 5, 8], "1": [NAN, 15, NAN]},
        {"ts": TS0 + 120000, "0": [3, NAN, 9], "1": [13, NAN, 19]}]
    add("union.threeSeriesWithNaNs", U + ":297-376", store="threeSameEGaps", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=3, steps=nan_steps, **J)
    offset_steps = [
        {"ts": TS0, "0": [1, 4], "1": [NAN, NAN]}, {"ts": TS0 + 60000, "0": [2, 5], "1": [NAN, NAN]},
        {"ts": TS0 + 120000, "0": [NAN, NAN], "1": [13, 16]}, {"ts": TS0 + 180000, "0": [NAN, NAN], "1": [14, 17]}]
    add("union.twoSeriesTimeOffset", U + ":378-461", store="timeOffset", query="AB_Dstar", use_qt=False, inc_agg=False,
        series_size=2, steps=offset_steps, **J)
    add("union.threeSeriesUsingResultTags", U + ":463-510", store="threeDifE", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=6,
        steps=steps(3, lambda k: {"0": [1 + k, 0, 4 + k, 0, 7 + k, 0], "1": [0, 11 + k, 0, 14 + k, 0, 17 + k]}), **J)
    add("union.threeSeriesUsingQueryTags", U + ":512-548", store="threeDifE", query="AB_Dstar", use_qt=True,
        inc_agg=False, series_size=3,
        steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 7 + k], "1": [11 + k, 14 + k, 17 + k]}), **J)
    add("union.commonAggregatedTag", U + ":550-581", store="twoSeriesAggedE", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=1, steps=steps(3, lambda k: {"0": [2 + 2 * k], "1": [22 + 2 * k]}), **J)
    add("union.extraAggTagIgnored", U + ":583-614", store="twoSeriesAggedEandExtraTagK", query="AB_Dstar",
        use_qt=False, inc_agg=False, series_size=1,
        steps=steps(3, lambda k: {"0": [2 + 2 * k], "1": [22 + 2 * k]}), **J)
    add("union.extraAggTag", U + ":616-650", store="twoSeriesAggedEandExtraTagK", query="AB_Dstar", use_qt=False,
        inc_agg=True, series_size=2, steps=steps(3, lambda k: {"0": [2 + 2 * k, 0], "1": [0, 22 + 2 * k]}), **J)
    for nm, src, qt, ag in [("onlyOneResultSet", ":652-688", False, False),
                            ("onlyOneResultSetQueryTags", ":690-726", True, False),
                            ("onlyOneResultSetAggTags", ":728-764", False, True)]:
        add("union." + nm, U + src, store="threeSameENoB", query="AB_Dstar", use_qt=qt, inc_agg=ag, series_size=3,
            steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 7 + k], "1": [0, 0, 0]}), **J)
    add("union.oneAggedOneTagged", U + ":766-800", store="oneAggedTheOtherTagged", query="AB_AggAll", use_qt=False,
        inc_agg=True, series_size=2, steps=steps(3, lambda k: {"0": [2 + 2 * k, 0], "1": [0, 11 + k]}), **J)
    add("union.oneAggedOneTaggedUseQueryTagsWoutQueryTags", U + ":802-833", store="oneAggedTheOtherTagged",
        query="AB_AggAll", use_qt=True, inc_agg=False, series_size=1,
        steps=steps(3, lambda k: {"0": [2 + 2 * k], "1": [11 + k]}), **J)
    add("union.singleSeries", U + ":835-858", store="oneExtraSameE", query="A_DD", use_qt=False, inc_agg=False,
        series_size=1, steps=steps(3, lambda k: {"0": [1 + k]}), **J)
    add("union.setAMissingE", U + ":860-902", store="threeAMissingE", query="AB_Dstar", use_qt=False, inc_agg=False,
        series_size=6,
        steps=steps(3, lambda k: {"0": [1 + k, 0, 4 + k, 0, 7 + k, 0], "1": [0, 11 + k, 0, 14 + k, 0, 17 + k]}), **J)
    add("union.setAMissingEQueryTags", U + ":904-940", store="threeAMissingE", query="AB_Dstar", use_qt=True,
        inc_agg=False, series_size=3,
        steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 7 + k], "1": [11 + k, 14 + k, 17 + k]}), **J)
    add("union.noData", U + ":942-952", store="empty", query="AB_Dstar", use_qt=False, inc_agg=False, series_size=0,
        has_next=False, **J)
    add("union.nextException", U + ":954-964", store="threeDisjointSameE", query="AB_Dstar", use_qt=False,
        inc_agg=False, next_calls=4, error="IllegalDataException", **J)

    # ---- IntersectionIterator ------------------------------------------------------------
    I = "TestIntersectionIterator.java"
    K = dict(kind="intersection", fill=NAN)
    add("intersection.ctorNullResults", I + ":71-74", kind="intersection", error="NullPointerException",
        null_results=True)
    add("intersection.ctorEmptyResults", I + ":76-82", kind="intersection", store="empty", query=None, use_qt=True,
        inc_agg=True, series_size=0, has_next=False)
    for nm, src in [("twoAndThreeSeries", ":84-116"), ("twoAndThreeSeriesExtraDPinKickedSeries", ":118-157")]:
        add("intersection." + nm, I + src, store="oneExtraSameE", query="AB_Dstar", use_qt=False, inc_agg=False,
            series_size=2, steps=steps(3, lambda k: {"0": [1 + k, 4 + k], "1": [11 + k, 14 + k]}), **K)
    add("intersection.threeSeriesIntersectToTwo", I + ":159-191", store="threeDisjointSameE", query="AB_Dstar",
        use_qt=False, inc_agg=False, series_size=2,
        steps=steps(3, lambda k: {"0": [1 + k, 7 + k], "1": [11 + k, 17 + k]}), **K)
    for nm, src in [("threeSeriesIntersectToExtraDPsinKicked", ":193-231"), ("threeSeriesIntersectToOne", ":233-261")]:
        add("intersection." + nm, I + src, store="reduceToOne", query="AB_Dstar", use_qt=False, inc_agg=False,
            series_size=1, steps=steps(3, lambda k: {"0": [7 + k], "1": [17 + k]}), **K)
    add("intersection.threeSeriesAggedIntoOne", I + ":263-294", store="threeSameE", query="AB_AggAll", use_qt=False,
        inc_agg=False, series_size=1, steps=steps(3, lambda k: {"0": [12 + 3 * k], "1": [42 + 3 * k]}), **K)
    add("intersection.threeSeriesFullIntersetWithNaNs", I + ":296-375", store="threeSameEGaps", query="AB_Dstar",
        use_qt=False, inc_agg=False, series_size=3, steps=nan_steps, **K)
    add("intersection.twoSeriesTimeOffset", I + ":377-460", store="timeOffset", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=2, steps=offset_steps, **K)
    add("intersection.noIntersectionUsingResultTags", I + ":462-467", store="threeDifE", query="AB_Dstar",
        use_qt=False, inc_agg=False, error="IllegalDataException", **K)
    add("intersection.intersectUsingQueryTags", I + ":469-505", store="threeDifE", query="AB_Dstar", use_qt=True,
        inc_agg=False, series_size=3,
        steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 7 + k], "1": [11 + k, 14 + k, 17 + k]}), **K)
    add("intersection.commonAggregatedTag", I + ":507-538", store="twoSeriesAggedE", query="AB_Dstar", use_qt=False,
        inc_agg=False, series_size=1, steps=steps(3, lambda k: {"0": [2 + 2 * k], "1": [22 + 2 * k]}), **K)
    add("intersection.extraAggTagIgnored", I + ":540-571", store="twoSeriesAggedEandExtraTagK", query="AB_Dstar",
        use_qt=False, inc_agg=False, series_size=1,
        steps=steps(3, lambda k: {"0": [2 + 2 * k], "1": [22 + 2 * k]}), **K)
    add("intersection.extraAggTagNoIntersection", I + ":573-578", store="twoSeriesAggedEandExtraTagK",
        query="AB_Dstar", use_qt=False, inc_agg=True, error="IllegalDataException", **K)
    add("intersection.onlyOneResultSet", I + ":580-585", store="threeSameENoB", query="AB_Dstar", use_qt=False,
        inc_agg=True, error="IllegalDataException", **K)
    add("intersection.oneAggedOneTaggedNoIntersection", I + ":587-592", store="oneAggedTheOtherTagged",
        query="AB_AggAll", use_qt=False, inc_agg=True, error="IllegalDataException", **K)
    add("intersection.oneAggedOneTaggedUseQueryTagsWoutQueryTags", I + ":594-625", store="oneAggedTheOtherTagged",
        query="AB_AggAll", use_qt=True, inc_agg=False, series_size=1,
        steps=steps(3, lambda k: {"0": [2 + 2 * k], "1": [11 + k]}), **K)
    add("intersection.singleSeries", I + ":627-650", store="oneExtraSameE", query="A_DD", use_qt=False, inc_agg=False,
        series_size=1, steps=steps(3, lambda k: {"0": [1 + k]}), **K)
    add("intersection.setAMissingE", I + ":652-657", store="threeAMissingE", query="AB_Dstar", use_qt=False,
        inc_agg=False, error="IllegalDataException", **K)
    add("intersection.setAMissingEQueryTags", I + ":659-695", store="threeAMissingE", query="AB_Dstar", use_qt=True,
        inc_agg=False, series_size=3,
        steps=steps(3, lambda k: {"0": [1 + k, 4 + k, 7 + k], "1": [11 + k, 14 + k, 17 + k]}), **K)
    add("intersection.noData", I + ":697-707", store="empty", query="AB_Dstar", use_qt=False, inc_agg=False,
        series_size=0, has_next=False, **K)
    add("intersection.nextException", I + ":709-719", store="threeDisjointSameE", query="AB_Dstar", use_qt=False,
        inc_agg=False, next_calls=4, error="IllegalDataException", **K)

    # ---- flattenTags (both classes) ----------------------------------------------------------
    U1, U2, U3 = [0, 0, 1], [0, 0, 2], [0, 0, 3]
    tags12 = [[U1, U1], [U2, U2]]
    flat = [   # (name, use_qt, inc_agg, tags, agg, query_tags, sub present, expect / error), both tests' order
        ("flattenTags", False, False, tags12, [U3], [U1], True, U1 + U1 + U2 + U2),
        ("flattenTagsWithAgg", False, True, tags12, [U3], [U1], True, U1 + U1 + U2 + U2 + U3),
        ("flattenTagsQueryTags", True, False, tags12, [U3], [U1], True, U1 + U1),
        ("flattenTagsQueryTagsWithAgg", True, True, tags12, [U3], [U1], True, U1 + U1 + U3),
        ("flattenEmptyTags", False, False, [], [U3], [U1], True, []),
        ("flattenEmptyTagsWithAggEmpty", False, True, tags12, [], [U1], True, U1 + U1 + U2 + U2),
        ("flattenTagsQueryTagsEmpty", True, False, tags12, [U3], [], True, []),
        ("flattenTagsQueryTagsEmptyWithAgg", True, True, tags12, [U3], [], True, U3),
        ("flattenTagsNullAggTagsNotRequested", False, False, tags12, None, [U1], True, U1 + U1 + U2 + U2),
        ("flattenTagsNullAggTags", False, True, tags12, None, [U1], True, "NullPointerException"),
        ("flattenTagsNullSubNotRequested", False, False, tags12, [U3], [U1], False, U1 + U1 + U2 + U2),
        ("flattenTagsNullSub", True, False, tags12, [U3], [U1], False, "NullPointerException"),
    ]
    ulines = {"flattenTags": ":966-971", "flattenTagsWithAgg": ":973-979", "flattenTagsQueryTags": ":981-986",
              "flattenTagsQueryTagsWithAgg": ":988-993", "flattenEmptyTags": ":995-1001",
              "flattenEmptyTagsWithAggEmpty": ":1003-1009", "flattenTagsQueryTagsEmpty": ":1013-1019",
              "flattenTagsQueryTagsEmptyWithAgg": ":1021-1027", "flattenTagsNullAggTagsNotRequested": ":1036-1041",
              "flattenTagsNullAggTags": ":1043-1047", "flattenTagsNullSubNotRequested": ":1049-1054",
              "flattenTagsNullSub": ":1056-1060"}
    ilines = {"flattenTags": ":721-726", "flattenTagsWithAgg": ":728-734", "flattenTagsQueryTags": ":736-741",
              "flattenTagsQueryTagsWithAgg": ":743-748", "flattenEmptyTags": ":750-756",
              "flattenEmptyTagsWithAggEmpty": ":758-764", "flattenTagsQueryTagsEmpty": ":768-774",
              "flattenTagsQueryTagsEmptyWithAgg": ":776-782", "flattenTagsNullAggTagsNotRequested": ":789-794",
              "flattenTagsNullAggTags": ":796-799", "flattenTagsNullSubNotRequested": ":801-806",
              "flattenTagsNullSub": ":808-811"}
    for union, pre, src_file, lines in [(True, "union.", U, ulines), (False, "intersection.", I, ilines)]:
        for nm, qt, ag, tg, agg, qtags, sub, exp in flat:
            e = {"error": exp} if isinstance(exp, str) else {"expect": exp}
            add(pre + nm, src_file + lines[nm], kind="flatten", union=union, use_qt=qt, inc_agg=ag, tags=tg, agg=agg,
                query_tags=qtags, sub=sub, **e)
        # null tag map: the union returns an empty key, the intersection throws
        add(pre + "flattenTagsNullTags", src_file + (":1029-1034" if union else ":784-787"), kind="flatten",
            union=union, use_qt=union, inc_agg=False, tags=None, agg=[U3], query_tags=[U1], sub=True,
            **({"expect": []} if union else {"error": "NullPointerException"}))

    # ---- ExpressionIterator (remapResults: sub iterators "a" / "b", fill ZERO) ----------------
    E = "TestExpressionIterator.java"
    X = dict(kind="expr", store="oneExtraSameE", query="AB_Dstar", vars={"a": 0, "b": 1}, use_qt=False,
             inc_agg=False, op="INTERSECTION")

    def ex(name, src, **kw):
        d = dict(X)
        d.update(kw)
        add("expression." + name, E + src, **d)

    ex("ctor", ":31-40", expression="a + b", ctor_only=True, names=["a", "b"])
    ex("ctorNoVariables", ":42-45", expression="1 + 1", error="IllegalArgumentException", ctor_only=True)
    ex("ctorNullExpression", ":47-50", expression=None, error="IllegalArgumentException", ctor_only=True)
    ex("ctorBadExpression", ":52-55", expression=" a / ", error="JexlException", ctor_only=True)
    ex("ctorEmptyExpression", ":57-60", expression="", error="IllegalArgumentException", ctor_only=True)
    ex("ctorNullOperator", ":62-65", expression="a + b", op=None, error="IllegalArgumentException", ctor_only=True)
    two = lambda f: steps(3, lambda k: {"values": f(k)})  # noqa: E731
    dd_ff = {"tags_d": ["D", "F"], "agg_empty": True}
    ex("aPlusBWithTwoSeries", ":67-106", expression="a + b", series_size=2,
       steps=two(lambda k: [12 + 2 * k, 18 + 2 * k]), **dd_ff)
    ex("aMinusBWithTwoSeries", ":108-143", expression="a - b", series_size=2, steps=two(lambda k: [-10, -10]), **dd_ff)
    ex("aTimesBWithTwoSeries", ":145-193", expression="a * b", series_size=2,
       steps=two(lambda k: [[11, 56], [24, 75], [39, 96]][k]), **dd_ff)
    ex("aDivideBWithTwoSeries", ":195-243", expression="a / b", series_size=2,
       steps=two(lambda k: [[0.0909, 0.2857], [0.1666, 0.3333], [0.2307, 0.375]][k]), **dd_ff)
    ex("aModBWithTwoSeries", ":245-281", expression="a % b", series_size=2, steps=two(lambda k: [1 + k, 4 + k]),
       **dd_ff)
    ex("aDivideByZeroWithTwoSeries", ":283-319", expression="a / 0", series_size=2, steps=two(lambda k: [0, 0]),
       **dd_ff)
    ex("doubleVariableAndPrecedence", ":321-369", expression="a + (b * b)", series_size=2,
       steps=two(lambda k: [[122, 200], [146, 230], [172, 262]][k]), **dd_ff)
    ex("doubleVariableAndPrecedenceChanged", ":371-419", expression="(a + b) * b", series_size=2,
       steps=two(lambda k: [[132, 252], [168, 300], [208, 352]][k]), **dd_ff)
    ex("aPlusScalarDropB", ":421-457", expression="a + 1", series_size=2, steps=two(lambda k: [2 + k, 5 + k]), **dd_ff)
    ex("missingRequiredVariable", ":459-471", expression="a + b + c", error="IllegalArgumentException")
    gaps = dict(store="threeSameEGaps", series_size=3, tags_d=["D", "F", "G"], agg_empty=True)
    ex("aPlusBMissingPointsDefaultFillZero", ":473-528", expression="a + b",
       steps=two(lambda k: [[1, 4, 0], [0, 20, 8], [16, 0, 28]][k]), **gaps)
    ex("aPlusBMissingPointsFillOne", ":530-587", expression="a + b", fills={"a": 1, "b": 1},
       steps=two(lambda k: [[2, 5, 2], [2, 20, 9], [16, 2, 28]][k]), **gaps)
    ex("aPlusBMissingPointsFillInfectiousNaN", ":589-648", expression="a + b", fills={"a": NAN, "b": NAN},
       steps=two(lambda k: [[NAN, NAN, NAN], [NAN, 20, NAN], [16, NAN, 28]][k]), **gaps)
    ex("aPlusBResultsOffsetDefaultFill", ":650-706", store="timeOffset", expression="a + b", series_size=2,
       steps=steps(4, lambda k: {"values": [[1, 4], [2, 5], [13, 16], [14, 17]][k]}), **dd_ff)
    ex("aPlusBOneAggedOneTaggedUseQueryTagsWoutQueryTags", ":708-747", store="oneAggedTheOtherTagged",
       query="AB_AggAll", use_qt=True, expression="a + b", series_size=1, steps=two(lambda k: [13 + 3 * k]),
       agg_tags=["D", "E"])
    ex("singleNestedExpression", ":749-793", expression="x * 2", vars={"x": "ei"},
       nested=[{"id": "ei", "expression": "a + b", "vars": {"a": 0, "b": 1}, "op": "INTERSECTION"}],
       series_size=2, steps=two(lambda k: [24 + 4 * k, 36 + 4 * k]), **dd_ff)
    ex("doubleNestedExpression", ":795-844", expression="e2 * 2", vars={"e2": "e2"},
       nested=[{"id": "e1", "expression": "a + b", "vars": {"a": 0, "b": 1}, "op": "INTERSECTION"},
               {"id": "e2", "expression": "e1 * 2", "vars": {"e1": "e1"}, "op": "INTERSECTION"}],
       series_size=2, steps=two(lambda k: [48 + 8 * k, 72 + 8 * k]), **dd_ff)
    ex("noIntersectionFound", ":846-858", store="threeDifE", expression="a + b", error="IllegalDataException")
    for nm, src in [("addResultsMissingId", ":860-868"), ("addResultsMissingSubQuery", ":870-878"),
                    ("addResultsMissingResults", ":880-888")]:
        # not remapped: iterators.get("a") is null -> addResults throws
        ex(nm, src, expression="a + b + c", error="IllegalArgumentException", null_iterator="a")
    ex("unionOneExtraSeries", ":890-933", op="UNION", expression="a + b", series_size=3,
       steps=two(lambda k: [12 + 2 * k, 18 + 2 * k, 17 + k]), agg_empty=True, tags_d=["D", "F"])
    ex("unionOffset", ":935-991", op="UNION", store="timeOffset", expression="a + b", series_size=2,
       steps=steps(4, lambda k: {"values": [[1, 4], [2, 5], [13, 16], [14, 17]][k]}), **dd_ff)
    ex("unionNoIntersection", ":993-1023", op="UNION", store="threeDifE", expression="a + b", series_size=6,
       steps=two(lambda k: [1 + k, 11 + k, 4 + k, 14 + k, 7 + k, 17 + k]))
    ex("unionSingleSeriesIteration", ":1025-1055", op="UNION", expression="a + b", mode="index",
       index_series=[[[TS0 + k * 60000, v] for k, v in enumerate(vals)]
                     for vals in ([12, 14, 16], [18, 20, 22], [17, 18, 19])])
    ex("intersectionSingleSeriesIteration", ":1057-1083", expression="a + b", mode="index",
       index_series=[[[TS0 + k * 60000, v] for k, v in enumerate(vals)] for vals in ([12, 14, 16], [18, 20, 22])])
    ex("aGreaterThanb", ":1085-1120", expression="a > b", series_size=2, steps=two(lambda k: [0, 0]),
       agg_empty=True)
    ex("aLessThanb", ":1122-1157", expression="a < b", series_size=2, steps=two(lambda k: [1, 1]), agg_empty=True)

    out = {"about": __doc__.split("\n\n")[0], "uids": "letter X -> [0, 0, 10 + X - 'A']",
           "stores": STORES, "queries": QUERIES, "cases": cases}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "expression_iter.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(cases)} cases -> {path}")


if __name__ == "__main__":
    main()
