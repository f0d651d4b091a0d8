"""Helpers of the expression-function tests."""
from __future__ import annotations

import json
import math
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "expression.json")


def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def oracle_run(case):
    """A fixture case on the oracle (oracle/expr.py): list of output series [(ts, value)]."""
    from oracle import expr as OX
    fn, params = case["fn"], case["params"]
    subs = [[([tuple(p) for p in s], b"") for s in sub] for sub in case["inputs"]]
    flat = [s for sub in subs for s in sub]
    if fn == "scale":
        out = OX.scale(flat, float(params[0]))
    elif fn in ("absolute", "alias"):
        out = OX.absolute(flat)   # Alias.java's loop is Absolute's
    elif fn == "movingAverage":
        p = params[0]
        if p.startswith("'"):
            from opentsdb_amd.expression import _mavg_window_ms
            out = OX.moving_average(flat, _mavg_window_ms(p), True, case["start"], case["end"])
        else:
            out = OX.moving_average(flat, int(p), False, case["start"], case["end"])
    else:
        op = {"sumSeries": "+", "diffSeries": "-", "multiplySeries": "*", "divideSeries": "/"}[fn]
        letters = [chr(ord("a") + i) for i in range(len(subs))]
        out = OX.combine(op, dict(zip(letters, subs)))
    return [o for o, _ in out]


def check(got, case):
    """got: list of [(ts, value)]; values compared with the test's tolerance, ints as ints."""
    exp = case["expect"]
    assert len(got) == len(exp), (case["name"], len(got), len(exp))
    for g, e in zip(got, exp):
        assert [t for t, _ in g] == [t for t, _ in e], case["name"]
        for (_, gv), (_, ev) in zip(g, e):
            if isinstance(ev, int) and not isinstance(ev, bool):
                assert isinstance(gv, int) and gv == ev, (case["name"], gv, ev)
            else:
                assert abs(float(gv) - float(ev)) <= case["tol"] or (math.isnan(gv) and math.isnan(ev)), \
                    (case["name"], gv, ev)


# ---- /api/query/exp join fixtures (tests/golden/expression_iter.json) --------------------------
def uid(letter: str) -> bytes:
    """test/core/BaseTsdbTest.java:102-110: 'A'..'Z' -> 00 00 0A.."""
    return bytes([0, 0, 10 + ord(letter) - ord("A")])


def num(v):
    return math.nan if v == "NaN" else float(v)


def result_sets(case, fill=0.0):
    """The fixture's sub-query results as product ResultSets (opentsdb_amd.expression)."""
    from opentsdb_amd import expression as X
    out = []
    for sub in case.get("results") or []:
        series = [X.Series.of([tuple(p) for p in s["points"]], tags={uid(k): uid(v) for k, v in s["tags"].items()},
                              agg_tags=[uid(a) for a in s["agg"]]) for s in sub["series"]]
        out.append(X.ResultSet(series, frozenset(uid(k) for k in sub["filter_tagks"]), fill))
    return out


def product_expression(case):
    """The fixture's ExpressionIterator on the product host (nested expressions included, not
    compiled); sub-queries remapped to the case's variables with fill ZERO unless set."""
    from opentsdb_amd import expression as X
    fills = {k: num(v) for k, v in (case.get("fills") or {}).items()}
    rs = result_sets(case)
    built = {}
    for spec in case.get("nested", []):
        e = X.ExpressionIterator(spec["id"], spec["expression"], spec["op"], case["use_qt"], case["inc_agg"])
        for var, src in spec["vars"].items():
            e.add_results(var, built[src] if isinstance(src, str) else rs[src])
        built[spec["id"]] = e
    exp = X.ExpressionIterator("ei", case["expression"], case["op"], case["use_qt"], case["inc_agg"])
    if case.get("null_iterator"):
        exp.add_results(case["null_iterator"], None)
    for var, src in case["vars"].items():
        if isinstance(src, str):
            exp.add_results(var, built[src])
        else:
            r = rs[src]
            exp.add_results(var, X.ResultSet(r.series, r.filter_tagks, fills.get(var, 0.0)))
    return exp, built
