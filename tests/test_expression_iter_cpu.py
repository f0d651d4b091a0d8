"""The /api/query/exp join-iterator oracle (oracle/expr_iter.py) against the 107 known answers
transcribed from TestUnionIterator, TestIntersectionIterator and TestExpressionIterator
(tests/golden/make_expression_iter_golden.py -> tests/golden/expression_iter.json)."""
from __future__ import annotations

import math

import numpy as np
import pytest

from oracle import expr_iter as X
from tests import golden_util as G

GOLD = G.load("expression_iter.json")
CASES = GOLD["cases"]


def uid(letter: str) -> bytes:
    return bytes([0, 0, 10 + ord(letter) - ord("A")])


def num(v):
    return math.nan if v == "NaN" else float(v)


def results_of(case):
    """[(filter tagks, [DataPoints])] per sub-query."""
    out = []
    for sub in case.get("results") or []:
        dps = [X.DataPoints([tuple(p) for p in s["points"]], {uid(k): uid(v) for k, v in s["tags"].items()},
                            [uid(a) for a in s["agg"]], metric=uid(sub["metric"])) for s in sub["series"]]
        out.append(({uid(k) for k in sub["filter_tagks"]}, dps))
    return out


def iterators(case, names, fill):
    res = results_of(case)
    its = {}
    for nm, idx in names.items():
        qt, dps = res[idx] if idx < len(res) else (set(), [])
        its[nm] = X.TimeSyncedIterator(nm, qt, dps, fill)
    return its


def close(got, want, tol, ctx):
    w = num(want)
    if math.isnan(w):
        assert math.isnan(got), f"{ctx}: {got} != NaN"
    else:
        assert abs(got - w) <= tol, f"{ctx}: {got} != {w}"


def run_join(case):
    fill = num(case["fill"]) if "fill" in case else 0.0
    if case.get("null_results"):
        with pytest.raises(X.JavaError) as ei:
            (X.UnionIterator if case["kind"] == "union" else X.IntersectionIterator)("it", None, True, True)
        assert ei.value.java == case["error"]
        return
    names = {str(i): i for i in range(len(case.get("results") or []))}
    its = iterators(case, names, fill)
    cls = X.UnionIterator if case["kind"] == "union" else X.IntersectionIterator
    if "error" in case and "next_calls" not in case:
        with pytest.raises(X.JavaError) as ei:
            cls("it", its, case["use_qt"], case["inc_agg"])
        assert ei.value.java == case["error"]
        return
    it = cls("it", its, case["use_qt"], case["inc_agg"])
    if "next_calls" in case:
        with pytest.raises(X.JavaError) as ei:
            for _ in range(case["next_calls"]):
                it.next()
        assert ei.value.java == case["error"]
        return
    assert it.series_size == case["series_size"]
    if "has_next" in case:
        assert it.has_next() == case["has_next"]
    res = it.results()
    for k, st in enumerate(case.get("steps", [])):
        assert it.has_next(), f"step {k}"
        it.next()
        for var, want in st.items():
            if var == "ts":
                continue
            arr = res[var]
            assert len(arr) == len(want)
            for j, w in enumerate(want):
                assert arr[j].ts == st["ts"], (k, var, j)
                close(arr[j].to_double(), w, case["tol"], f"step {k} set {var}[{j}]")
    if "steps" in case:
        assert not it.has_next()


def run_flatten(case):
    tags = None if case["tags"] is None else {bytes(k): bytes(v) for k, v in case["tags"]}
    agg = None if case["agg"] is None else [bytes(a) for a in case["agg"]]
    qt = [bytes(q) for q in case["query_tags"]]
    call = lambda: X.flatten_tags(case["union"], case["use_qt"], case["inc_agg"], tags, agg, qt, case["sub"])  # noqa: E731
    if "error" in case:
        with pytest.raises(X.JavaError) as ei:
            call()
        assert ei.value.java == case["error"]
    else:
        assert call() == bytes(case["expect"])


def build_expression(case):
    """The test's ExpressionIterator (sub iterators remapped to "a" / "b": fill ZERO unless set)."""
    fills = {k: num(v) for k, v in (case.get("fills") or {}).items()}
    built = {}
    for spec in case.get("nested", []):
        e = X.ExpressionIterator(spec["id"], spec["expression"], spec["op"], case["use_qt"], case["inc_agg"])
        for var, src in spec["vars"].items():
            e.add_results(var, built[src] if isinstance(src, str) else iterators(case, {var: src}, 0.0)[var])
        e.compile()
        built[spec["id"]] = e
    exp = X.ExpressionIterator("ei", case["expression"], case["op"], case["use_qt"], case["inc_agg"])
    if case.get("null_iterator"):
        exp.add_results(case["null_iterator"], None)
    for var, src in case["vars"].items():
        if isinstance(src, str):
            exp.add_results(var, built[src])
        else:
            it = iterators(case, {var: src}, 0.0)[var]
            if var in fills:
                it.fill = fills[var]
            exp.add_results(var, it)
    return exp


def run_expression(case):
    if "error" in case:
        with pytest.raises(X.JavaError) as ei:
            exp = build_expression(case)
            if not case.get("ctor_only"):
                exp.compile()
        assert ei.value.java == case["error"]
        return
    exp = build_expression(case)
    if case.get("ctor_only"):
        assert sorted(exp.names) == sorted(case["names"]) and exp.values() is None
        return
    exp.compile()
    dps = exp.values()
    if case.get("mode") == "index":
        for i, series in enumerate(case["index_series"]):
            got = []
            while exp.has_next_index(i):
                exp.next_index(i)
                got.append((dps[i].ts, dps[i].to_double()))
            assert len(got) == len(series)
            for (t, v), (wt, wv) in zip(got, series):
                assert t == wt
                close(v, wv, case["tol"], f"series {i}")
        return
    assert len(dps) == case["series_size"]
    its = exp.next_timestamp()
    for k, st in enumerate(case["steps"]):
        assert exp.has_next(), f"step {k}"
        exp.next_ts(its)
        assert len(st["values"]) == len(dps)
        for i, w in enumerate(st["values"]):
            assert dps[i].ts == st["ts"]
            close(dps[i].to_double(), w, case["tol"], f"step {k} series {i}")
        its = exp.next_timestamp()
    assert not exp.has_next()
    for i, d in enumerate(case.get("tags_d", [])):
        assert dps[i].tags.get(uid("D")) == uid(d)
    if case.get("agg_empty"):
        assert all(not d.agg for d in dps)
    if "agg_tags" in case:
        assert dps[0].agg == {uid(a) for a in case["agg_tags"]}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_join_tests(case):
    if case["kind"] in ("union", "intersection"):
        run_join(case)
    elif case["kind"] == "flatten":
        run_flatten(case)
    else:
        run_expression(case)


def test_fixture_counts():
    """Every @Test of the three reference classes is transcribed."""
    by = {}
    for c in CASES:
        by[c["name"].split(".")[0]] = by.get(c["name"].split(".")[0], 0) + 1
    assert by == {"union": 37, "intersection": 36, "expression": 34}


def test_hashmap_order_simulation():
    """java.util.HashMap iteration order: single-letter keys in bucket order, "e1" first."""
    assert X.hashmap_order(["b", "a"]) == ["a", "b"]
    assert X.hashmap_order(["1", "0"], 2) == ["0", "1"]
    assert X.hashmap_order(["e1", "a"]) == ["a", "e1"]   # "e1".hashCode() = 3180 -> bucket 12, "a" -> 1


# ---- the product's host half: flattenTags and the joins (no GPU) -------------------------------
from opentsdb_amd import expression as PX  # noqa: E402
from tests import expr_util as EU  # noqa: E402

FLATTEN = [c for c in CASES if c["kind"] == "flatten" and "error" not in c and c["tags"] is not None]


@pytest.mark.parametrize("case", FLATTEN, ids=[c["name"] for c in FLATTEN])
def test_product_flatten_tags(case):
    tags = {bytes(k): bytes(v) for k, v in case["tags"]}
    agg = [bytes(a) for a in (case["agg"] or [])]
    qt = [bytes(q) for q in case["query_tags"]]
    assert PX.flatten_tags(case["use_qt"], case["inc_agg"], tags, agg, qt) == bytes(case["expect"])


JOINS = [c for c in CASES if c["kind"] in ("union", "intersection") and c.get("results") is not None
         and "next_calls" not in c]


@pytest.mark.parametrize("case", JOINS, ids=[c["name"] for c in JOINS])
def test_product_join_plan(case):
    """The product's join of the fixture's results (variables v0, v1 over sub-queries 0, 1):
    the joined set count, or the exception, as the reference test expects."""
    rs = EU.result_sets(case, EU.num(case["fill"]))
    exp = PX.ExpressionIterator("it", " + ".join(f"v{i}" for i in range(len(rs))) or "v0",
                                "UNION" if case["kind"] == "union" else "INTERSECTION", case["use_qt"], case["inc_agg"])
    for i, r in enumerate(rs):
        exp.add_results(f"v{i}", r)
    if "error" in case:
        with pytest.raises(PX.ExpressionError) as ei:
            exp.plan()
        assert ei.value.java == case["error"]
        return
    flat, members, keys, joined, active, jorder = exp.plan()
    assert len(keys) == case["series_size"]


EXPRS = [c for c in CASES if c["kind"] == "expr" and "error" in c]


@pytest.mark.parametrize("case", EXPRS, ids=[c["name"] for c in EXPRS])
def test_product_expression_errors(case):
    """Constructor / compile exceptions of TestExpressionIterator on the product host."""
    with pytest.raises(PX.ExpressionError) as ei:
        if case.get("ctor_only"):
            PX.ExpressionIterator("ei", case["expression"], case["op"], False, False)
        else:
            exp, built = EU.product_expression(case)
            for e in built.values():
                e.series = []
            exp.plan()
    assert ei.value.java == case["error"]


def test_product_compiler_types():
    """JEXL literal and path rules the compiler folds: integer division truncates, Float literals
    are float32, a division by zero is 0.0, an Integer result is refused."""
    prog, consts, names = PX.compile_expression("(7 / 2) * a + 0.1")
    assert consts == [3.0, float(np.float32(0.1))]
    assert PX.compile_expression("a / 0")[1] == [0.0]
    assert PX.compile_expression("(1 / 0) * a")[1] == [0.0]
    with pytest.raises(PX.ExpressionError) as ei:
        PX.compile_expression("(a > b) + 1")
    assert ei.value.java == "IllegalStateException"
