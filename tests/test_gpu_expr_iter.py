"""GPU parity of /api/query/exp expressions (tsdbhip_expr_sync over the host's UNION /
INTERSECTION joins) against the reference's known answers (TestExpressionIterator,
TestUnionIterator, TestIntersectionIterator -> tests/golden/expression_iter.json) and, bit for
bit, against the oracle's restatement of the iterators (oracle/expr_iter.py) on random stores."""
from __future__ import annotations

import math

import numpy as np
import pytest

from opentsdb_amd import expression as X
from oracle import expr_iter as OI
from tests import expr_util as EU
from tests import golden_util as G

pytestmark = pytest.mark.gpu

GOLD = G.load("expression_iter.json")
CASES = GOLD["cases"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def close(got, want, tol, ctx):
    w = EU.num(want)
    if math.isnan(w):
        assert math.isnan(got), f"{ctx}: {got} != NaN"
    else:
        assert abs(got - w) <= tol, f"{ctx}: {got} != {w}"


SYNC = [c for c in CASES if c["kind"] == "expr" and "error" not in c and not c.get("ctor_only")
        and c.get("mode") != "index"]


@pytest.mark.parametrize("case", SYNC, ids=[c["name"] for c in SYNC])
def test_expression_known_answers(eng, case):
    exp, _ = EU.product_expression(case)
    out = exp.compile(eng)
    assert len(out) == case["series_size"]
    for k, st in enumerate(case["steps"]):
        for i, w in enumerate(st["values"]):
            assert int(out[i].ts[k]) == st["ts"]
            close(out[i].values()[k], w, case["tol"], f"{case['name']} step {k} set {i}")
    assert all(len(s.ts) == len(case["steps"]) for s in out)
    for i, d in enumerate(case.get("tags_d", [])):
        assert out[i].tags.get(EU.uid("D")) == EU.uid(d)
    if case.get("agg_empty"):
        assert all(not s.agg_tags for s in out)
    if "agg_tags" in case:
        assert set(out[0].agg_tags) == {EU.uid(a) for a in case["agg_tags"]}


JOINS = [c for c in CASES if c["kind"] in ("union", "intersection") and c.get("results") is not None
         and "error" not in c]


@pytest.mark.parametrize("case", JOINS, ids=[c["name"] for c in JOINS])
def test_join_known_answers(eng, case):
    """The join iterator's per-set values at every step: expression `v<k>` returns sub-query k's."""
    rs = EU.result_sets(case, EU.num(case["fill"]))
    op = "UNION" if case["kind"] == "union" else "INTERSECTION"
    for k in range(len(rs)):
        exp = X.ExpressionIterator("it", f"v{k}", op, case["use_qt"], case["inc_agg"])
        for i, r in enumerate(rs):
            exp.add_results(f"v{i}", r)
        out = exp.compile(eng)
        assert len(out) == case["series_size"]
        for s, st in enumerate(case.get("steps", [])):
            for j, w in enumerate(st[str(k)]):
                assert int(out[j].ts[s]) == st["ts"]
                close(out[j].values()[s], w, case["tol"], f"{case['name']} v{k} step {s} set {j}")


def test_union_single_series_iteration(eng):
    """TestExpressionIterator.unionSingleSeriesIteration: next(int) through EDPtoDPS, i.e. the
    graphite path (tsdbhip_expr_zip) over the union keyed by flattenTags."""
    case = next(c for c in CASES if c["name"] == "expression.unionSingleSeriesIteration")
    rs = EU.result_sets(case)
    variables = {}
    for var, idx in case["vars"].items():
        variables[var] = [X.Series(s.ts, s.bits, s.is_int, X.flatten_tags(False, False, s.tags, s.agg_tags, None))
                          for s in rs[idx].series]
    out = X.evaluate(eng, case["expression"], variables)
    assert len(out) == len(case["index_series"])
    for s, want in zip(out, case["index_series"]):
        assert [int(t) for t in s.ts] == [w[0] for w in want]
        for g, w in zip(s.values(), want):
            close(g, w[1], 1e-4, "unionSingleSeriesIteration")


# ---- random stores, bit for bit against the oracle ---------------------------------------------
def rand_store(rng, n_vars, n_series, n_points, shared_keys=0.6, gaps=0.2, nan=0.05, kinds=("int", "dbl")):
    """Per variable: series over tag D values (some keys in one variable only), sparse aligned
    timestamps, int or double values with NaNs."""
    subs = []
    for v in range(n_vars):
        series = []
        dvals = [chr(ord("A") + i) for i in range(n_series)]
        for d in dvals:
            if rng.random() > shared_keys and v > 0:
                d = chr(ord(d) + 1)
            if any(s["tags"].get("D") == d for s in series):
                continue
            keep = rng.random(n_points) > gaps
            ts = (1431561600 + np.flatnonzero(keep) * 60) * 1000
            kind = kinds[int(rng.integers(0, len(kinds)))]
            pts = []
            for t in ts:
                if kind == "int":
                    pts.append((int(t), int(rng.integers(-1000, 1000))))
                else:
                    x = float(rng.normal(0, 50))
                    pts.append((int(t), math.nan if rng.random() < nan else x))
            if pts:
                e = {"E": "E"} if rng.random() < 0.5 else {"E": "F"}
                series.append({"points": pts, "tags": {"D": d, **e}, "agg": ["Z"] if rng.random() < 0.3 else []})
        subs.append(series)
    return subs


def build_both(subs, expression, op, use_qt, inc_agg, fills):
    names = [f"v{i}" for i in range(len(subs))]
    pe = X.ExpressionIterator("e", expression, op, use_qt, inc_agg)
    oe = OI.ExpressionIterator("e", expression, op, use_qt, inc_agg)
    for nm, ser, f in zip(names, subs, fills):
        pser = [X.Series.of(s["points"], tags={EU.uid(k): EU.uid(v) for k, v in s["tags"].items()},
                            agg_tags=[EU.uid(a) for a in s["agg"]]) for s in ser]
        pe.add_results(nm, X.ResultSet(pser, frozenset({EU.uid("D")}), f))
        odps = [OI.DataPoints(s["points"], {EU.uid(k): EU.uid(v) for k, v in s["tags"].items()},
                              [EU.uid(a) for a in s["agg"]]) for s in ser]
        oe.add_results(nm, OI.TimeSyncedIterator(nm, {EU.uid("D")}, odps, f))
    return pe, oe


def bit_equal(a, b):
    return (math.isnan(a) and math.isnan(b)) or np.float64(a).view(np.uint64) == np.float64(b).view(np.uint64)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("op", ["UNION", "INTERSECTION"])
def test_random_expressions_vs_oracle(eng, seed, op):
    rng = np.random.default_rng(seed)
    subs = rand_store(rng, 3, 12, 40)
    exprs = ["v0 + v1 * v2", "(v0 - v1) / v2", "v0 % (v1 + 0.5)", "v0 > v1", "v2 / 0 + v0", "-v0 * 2.5 + (v1 <= v2)",
             "(v0 + v1 + v2) / 3", "v1 != v1 * 1"]
    for ex in exprs:
        for use_qt, inc_agg in [(False, False), (True, False), (False, True)]:
            fills = [[0.0, math.nan, 1.5][int(rng.integers(0, 3))] for _ in subs]
            start = 1431561600000 + int(rng.integers(0, 5)) * 60000
            end = start + int(rng.integers(10, 40)) * 60000
            pe, oe = build_both(subs, ex, op, use_qt, inc_agg, fills)
            try:
                oe.compile()
                want = OI.serialize(oe, start, end)
            except OI.JavaError as e:
                with pytest.raises(X.ExpressionError) as ei:
                    pe.compile(eng, start, end)
                assert ei.value.java == e.java
                continue
            out = pe.compile(eng, start, end)
            assert len(out) == len(oe.dps)
            ctx = f"{seed} {op} {ex} qt={use_qt} agg={inc_agg}"
            assert [int(t) for t in pe.steps] == [r[0] for r in want], ctx
            for k, (t, vals) in enumerate(want):
                for j, w in enumerate(vals):
                    assert bit_equal(out[j].values()[k], w), (ctx, k, j, out[j].values()[k], w)
            for j, d in enumerate(oe.dps):
                assert out[j].tags == d.tags and set(out[j].agg_tags) == d.agg, ctx


def test_nested_expression_vs_oracle(eng):
    rng = np.random.default_rng(11)
    subs = rand_store(rng, 2, 8, 30, gaps=0.0, nan=0.0)
    pe, oe = build_both(subs, "v0 * v1 + 1", "UNION", False, False, [0.0, 0.0])
    outer_p = X.ExpressionIterator("o", "x / 2 - x", "UNION", False, False)
    outer_p.add_results("x", pe)
    outer_o = OI.ExpressionIterator("o", "x / 2 - x", "UNION", False, False)
    outer_o.add_results("x", oe)
    outer_o.compile()
    want = OI.serialize(outer_o, 0, 1 << 62)
    out = outer_p.compile(eng)
    assert [int(t) for t in outer_p.steps] == [r[0] for r in want]
    for k, (t, vals) in enumerate(want):
        for j, w in enumerate(vals):
            assert bit_equal(out[j].values()[k], w)


def test_large_join_on_the_device(eng):
    """3 variables x 600 tagged series x 360 steps: the join on the host, 216k evaluations on the
    GPU, against the oracle on a slice of the steps and sets."""
    rng = np.random.default_rng(5)
    n, npts = 600, 360
    subs = []
    for v in range(3):
        ser = []
        for i in range(n):
            keep = rng.random(npts) > 0.1
            ts = (1431561600 + np.flatnonzero(keep) * 10) * 1000
            vals = rng.normal(100, 20, len(ts))
            d = f"{chr(ord('A') + i % 26)}{chr(ord('A') + (i // 26) % 26)}"
            ser.append({"points": list(zip(ts.tolist(), vals.tolist())), "tags": {"D": d[0], "E": d[1]}, "agg": []})
        subs.append(ser)
    # two UID letters per series id: tags D, E (600 distinct sets)
    pe, oe = build_both(subs, "(v0 + v1) * v2 - v0 / v1", "INTERSECTION", False, False, [0.0, 0.0, math.nan])
    out = pe.compile(eng)
    oe.compile()
    want = OI.serialize(oe, 0, 1 << 62)
    assert len(out) == len(oe.dps) and len(pe.steps) == len(want)
    for k in range(0, len(want), 37):
        t, vals = want[k]
        for j in range(0, len(vals), 53):
            assert bit_equal(out[j].values()[k], vals[j])


def with_repeats(rng, subs, p_dup=0.25, max_extra=3):
    """Copies of random points (the same timestamp, a new value) in every series: the step walk
    over repeated timestamps (TimeSyncedIterator.next(long) :125-144 takes one point per step)."""
    out = []
    for ser in subs:
        ns = []
        for s in ser:
            pts = []
            for t, v in s["points"]:
                pts.append((t, v))
                if rng.random() < p_dup:
                    for _ in range(int(rng.integers(1, max_extra + 1))):
                        pts.append((t, int(rng.integers(-50, 50)) if isinstance(v, int) else float(rng.normal(0, 9))))
            ns.append({**s, "points": pts})
        out.append(ns)
    return out


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("op", ["UNION", "INTERSECTION"])
def test_repeated_timestamps_vs_oracle(eng, seed, op):
    """Series repeating timestamps: each timestamp is stepped as often as the series with the most
    copies holds it, the j-th step reading every series' j-th copy or its fill -- against the
    oracle's literal step walk, bit for bit, with and without a query range."""
    rng = np.random.default_rng(100 + seed)
    subs = with_repeats(rng, rand_store(rng, 3, 10, 30))
    for ex in ["v0 + v1 * v2", "(v0 - v1) / v2", "v0 > v1"]:
        fills = [[0.0, math.nan, 1.5][int(rng.integers(0, 3))] for _ in subs]
        for start, end in [(0, 1 << 62), (1431561600000 + 5 * 60000, 1431561600000 + 21 * 60000)]:
            pe, oe = build_both(subs, ex, op, False, True, fills)
            try:
                oe.compile()
                want = OI.serialize(oe, start, end)
            except OI.JavaError as e:
                with pytest.raises(X.ExpressionError) as ei:
                    pe.compile(eng, start, end)
                assert ei.value.java == e.java
                continue
            out = pe.compile(eng, start, end)
            ctx = f"{seed} {op} {ex} [{start}, {end}]"
            assert [int(t) for t in pe.steps] == [r[0] for r in want], ctx
            assert len(set(r[0] for r in want)) < len(want) or not want, ctx   # repeats were stepped
            for k, (t, vals) in enumerate(want):
                for j, w in enumerate(vals):
                    assert bit_equal(out[j].values()[k], w), (ctx, k, j, out[j].values()[k], w)


def test_repeated_timestamps_nested(eng):
    """A nested expression's output repeats the steps its inputs repeat; the outer one walks them."""
    rng = np.random.default_rng(21)
    subs = with_repeats(rng, rand_store(rng, 2, 6, 20, gaps=0.0, nan=0.0))
    pe, oe = build_both(subs, "v0 * v1 + 1", "UNION", False, False, [0.0, 0.0])
    outer_p = X.ExpressionIterator("o", "x / 2 - x", "UNION", False, False)
    outer_p.add_results("x", pe)
    outer_o = OI.ExpressionIterator("o", "x / 2 - x", "UNION", False, False)
    outer_o.add_results("x", oe)
    outer_o.compile()
    want = OI.serialize(outer_o, 0, 1 << 62)
    out = outer_p.compile(eng)
    assert [int(t) for t in outer_p.steps] == [r[0] for r in want]
    for k, (t, vals) in enumerate(want):
        for j, w in enumerate(vals):
            assert bit_equal(out[j].values()[k], w)


def test_decreasing_timestamps_refused(eng):
    from opentsdb_amd.engine import EngineError
    subs = [[{"points": [(2000, 1.0), (1000, 2.0)], "tags": {"D": "A"}, "agg": []}]]
    pe, _ = build_both(subs, "v0 + 1", "UNION", False, False, [0.0])
    with pytest.raises(EngineError, match="out of time order"):
        pe.compile(eng)
