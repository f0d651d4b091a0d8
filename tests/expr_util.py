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
