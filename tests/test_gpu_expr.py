"""Expression functions on the MI355X: k_expr through the C ABI
(tsdbhip_expr_map / tsdbhip_expr_zip, driven by opentsdb_amd.expression) against the reference's
known answers (tests/golden/expression.json) and the oracle (oracle/expr.py), bit for bit."""
from __future__ import annotations

import math

import numpy as np
import pytest

from opentsdb_amd import expression as X
from opentsdb_amd.engine import Engine, EngineError
from oracle import expr as OX
from tests import expr_util as U

pytestmark = pytest.mark.gpu

G = U.golden()


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


def as_series(sub):
    return [X.Series.of([tuple(p) for p in s]) for s in sub]


def run_engine(eng, case):
    subs = [as_series(sub) for sub in case["inputs"]]
    fn = case["fn"]
    if fn == "scale":
        out = X.scale(eng, subs, case["params"])
    elif fn == "absolute":
        out = X.absolute(eng, subs)
    elif fn == "alias":
        out = X.alias(eng, subs, case["params"])
        assert all(s.name == case["alias_name"] for s in out)
    elif fn == "movingAverage":
        out = X.moving_average(eng, subs, case["params"], case["start"], case["end"])
    else:
        out = X.FUNCTIONS[fn](eng, subs)
    return [list(zip([int(t) for t in s.ts], s.values())) for s in out]


def same(got, want):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert len(g) == len(w)
        for (gt, gv), (wt, wv) in zip(g, w):
            assert gt == wt
            assert type(gv) is type(wv) or (isinstance(gv, float) and isinstance(wv, float)), (gv, wv)
            if isinstance(wv, float):
                assert np.float64(gv).view(np.uint64) == np.float64(wv).view(np.uint64) or (math.isnan(gv) and math.isnan(wv)), (gv, wv)
            else:
                assert gv == wv


@pytest.mark.parametrize("case", G["cases"], ids=[c["name"] for c in G["cases"]])
def test_gpu_known_answers(eng, case):
    got = run_engine(eng, case)
    U.check(got, case)
    same(got, U.oracle_run(case))


def rand_series(rng, n, kind, t0=1356998400000, period=10000):
    ts = t0 + np.cumsum(rng.integers(1, 3, n)) * period
    pts = []
    for t in ts:
        if kind == "int":
            v = int(rng.choice([rng.integers(-1000, 1000), rng.integers(-(1 << 62), 1 << 62)]))
            pts.append((int(t), v))
        else:
            v = float(rng.choice([rng.normal(0, 100), float("nan"), 0.0, -0.0, 1e300]))
            pts.append((int(t), v))
    return pts


@pytest.mark.parametrize("factor", ["2", "-3", "1.5", "0", "9223372036854775807", "-0.25"])
def test_gpu_scale_absolute_random(eng, factor):
    rng = np.random.default_rng(len(factor))
    raw = [rand_series(rng, 50, "int"), rand_series(rng, 60, "dbl"), rand_series(rng, 7, "int")]
    subs = [[X.Series.of(p) for p in raw]]
    got = [list(zip([int(t) for t in s.ts], s.values())) for s in X.scale(eng, subs, [factor])]
    same(got, [o for o, _ in OX.scale([(p, b"") for p in raw], float(factor))])
    got = [list(zip([int(t) for t in s.ts], s.values())) for s in X.absolute(eng, subs)]
    same(got, [o for o, _ in OX.absolute([(p, b"") for p in raw])])


@pytest.mark.parametrize("param", ["1", "3", "10", "'1min'", "'5min'", "'1h'"])
def test_gpu_moving_average_random(eng, param):
    rng = np.random.default_rng(7 + len(param))
    raw = [rand_series(rng, 120, "dbl"), rand_series(rng, 90, "int")]
    t0 = raw[0][5][0]
    t1 = raw[0][100][0]
    subs = [[X.Series.of(p) for p in raw]]
    got = [list(zip([int(t) for t in s.ts], s.values())) for s in X.moving_average(eng, subs, [param], t0, t1)]
    timed = param.startswith("'")
    cond = X._mavg_window_ms(param) if timed else int(param)
    same(got, [o for o, _ in OX.moving_average([(p, b"") for p in raw], cond, timed, t0, t1)])


@pytest.mark.parametrize("fn,op", [("sumSeries", "+"), ("diffSeries", "-"), ("multiplySeries", "*")])
def test_gpu_combine_joined_sets(eng, fn, op):
    """Three sub-queries with tag-joined series (some keys in one sub-query only: the absent
    variable reads 0), equal lengths per set, NaN values filled with 0."""
    rng = np.random.default_rng(len(fn))
    keys = [b"\x00\x01", b"\x00\x02", b"\x01\x00", b"\xff"]
    subs, osubs = [], []
    for v in range(3):
        lst, olst = [], []
        for k in keys:
            if rng.random() < 0.3:
                continue
            pts = rand_series(rng, 40 + keys.index(k), "dbl", t0=1356998400000 + v * 7)
            lst.append(X.Series.of(pts, key=k))
            olst.append((pts, k))
        subs.append(lst)
        osubs.append(olst)
    got = [list(zip([int(t) for t in s.ts], s.values())) for s in X.FUNCTIONS[fn](eng, subs)]
    want = [o for o, _ in OX.combine(op, dict(zip("abc", osubs)))]
    same(got, want)


def test_gpu_combine_errors_like_the_reference(eng):
    a = [X.Series.of([(1, 1.0), (2, 2.0)])]
    b = [X.Series.of([(1, 1.0)])]
    with pytest.raises(EngineError) as e:
        X.sum_series(eng, [a, b])
    assert e.value.code == -6
    z = [X.Series.of([(1, 0.0), (2, 1.0)])]   # a division by zero is 0.0 (lenient JEXL)
    out = X.divide_series(eng, [a, z])
    assert out[0].values() == [0.0, 2.0]


def test_gpu_evaluate_general_expression(eng):
    rng = np.random.default_rng(3)
    pa, pb, pc = (rand_series(rng, 30, "dbl") for _ in range(3))
    pb = [(t, v if v != 0 else 1.0) for t, v in pb]
    got = X.evaluate(eng, "a * 2 + -b % 3 - (c + a) / 4", {"a": [X.Series.of(pa)], "b": [X.Series.of(pb)],
                                                          "c": [X.Series.of(pc)]})
    vals = got[0].values()
    for i in range(30):
        a, b, c = (float(x[i][1]) for x in (pa, pb, pc))
        a, b, c = (0.0 if math.isnan(x) else x for x in (a, b, c))
        want = a * 2.0 + math.fmod(-b, 3.0) - (c + a) / 4.0
        assert np.float64(vals[i]).view(np.uint64) == np.float64(want).view(np.uint64) or (math.isnan(vals[i]) and math.isnan(want))
    assert list(got[0].ts) == [min(pa[i][0], pb[i][0], pc[i][0]) for i in range(30)]


def test_gpu_shift_series(eng):
    sh = G["timeshift_shift"]
    for idx, ms, want in sh["cases"]:
        out = X.shift_series(eng, [X.Series.of([tuple(sh["points"][idx])])], ms)
        assert int(out[0].ts[0]) == want and out[0].values()[0] == sh["points"][idx][1]
    with pytest.raises(EngineError) as e:
        X.shift_series(eng, [X.Series.of([(1, 1.5)])], 1000)
    assert e.value.code == -9


# ---- highestMax / highestCurrent (tsdbhip_expr_topn) -------------------------------------
def _topn_engine(eng, case):
    subs = [as_series(sub) for sub in case["inputs"]]
    flat = [s for sub in subs for s in sub]
    out = X.FUNCTIONS[case["fn"]](eng, subs, case["params"], case["start"], case["end"])
    return [next(i for i, s in enumerate(flat) if s is o) for o in out]


def _topn_oracle(flat_pts, n, start, end, fn):
    return OX.highest(flat_pts, n, start, end, current=fn == "highestCurrent")


@pytest.mark.parametrize("case", [c for c in G["topn"] if not c["raises"]], ids=lambda c: c["name"])
def test_gpu_topn_known_answers(eng, case):
    assert _topn_engine(eng, case) == case["expect_index"]


def _rand_topn_series(rng, k, kinds, t0=1356998400000, period=10000, npts=40):
    out = []
    for i in range(k):
        n = int(rng.integers(0, npts))
        ts = np.sort(rng.choice(np.arange(0, 3 * npts), size=n, replace=False)) * period + t0
        kind = kinds[i % len(kinds)]
        pts = []
        for t in ts:
            if kind == "int":
                pts.append((int(t), int(rng.integers(-5000, 5000))))
            elif kind == "float":
                pts.append((int(t), float(rng.choice([rng.normal(0, 100), 0.0, -0.0, 1e6]))))
            else:
                pts.append((int(t), int(rng.integers(-50, 50)) if rng.random() < 0.5 else float(rng.normal(0, 50))))
        out.append(pts)
    return out


@pytest.mark.parametrize("fn", ["highestMax", "highestCurrent"])
@pytest.mark.parametrize("seed,k,kinds", [(1, 5, ("int",)), (2, 12, ("float",)), (3, 30, ("int", "float")),
                                          (4, 70, ("mixed",)), (5, 130, ("int", "mixed", "float"))])
def test_gpu_topn_random_vs_oracle(eng, fn, seed, k, kinds):
    """Late starts, early ends, empty series, LERP between points, long / double points; more
    series than a wave's lanes (positions carried across 64-span chunks)."""
    rng = np.random.default_rng(seed)
    pts = _rand_topn_series(rng, k, kinds)
    t0 = 1356998400000
    for start, end in [(t0, t0 + 10 ** 7), (t0 + 200000, t0 + 900000)]:
        for n in (1, 3, k, 1000):
            subs = [[X.Series.of(p) for p in pts[: k // 2]], [X.Series.of(p) for p in pts[k // 2:]]]
            flat = [s for sub in subs for s in sub]
            try:
                want = _topn_oracle(pts, n, start, end, fn)
                werr = None
            except OX.OracleExprError as e:
                want, werr = None, e.java
            try:
                out = X.FUNCTIONS[fn](eng, subs, [str(n)], start, end)
                got = [next(i for i, s in enumerate(flat) if s is o) for o in out]
                gerr = None
            except EngineError as e:
                got, gerr = None, e.java
            assert gerr == werr, (fn, seed, start, n, gerr, werr)
            assert got == want, (fn, seed, start, n)


def test_gpu_topn_no_point_in_range_raises(eng):
    subs = [[X.Series.of([(1000, 5)]), X.Series.of([(2000, 7)])]]
    with pytest.raises(EngineError) as e:
        X.highest_max(eng, subs, ["1"], 5000, 9000)
    assert e.value.java == "NullPointerException"
    with pytest.raises(OX.OracleExprError):
        OX.highest([[(1000, 5)], [(2000, 7)]], 1, 5000, 9000)


def test_gpu_nested_expression_tree(eng):
    """Expressions.parse + ExpressionTree.evaluate (opentsdb_amd/expression_tree.py) over the GPU
    functions: scale(absolute(sum:a),, 2) and movingAverage(scale(sum:a,,3),, 4) against the
    oracle's functions composed the same way; sumSeries over two metric queries."""
    from opentsdb_amd import expression_tree as T
    rng = np.random.default_rng(99)
    raw = [rand_series(rng, 80, "int"), rand_series(rng, 70, "dbl")]
    raw_b = [rand_series(rng, 70, "dbl")]   # as long as a's last series (positional join)
    results = [[X.Series.of(p) for p in raw], [X.Series.of(p) for p in raw_b]]
    t0, t1 = raw[0][3][0], raw[0][70][0]
    mq = []
    tree = T.parse("scale(absolute(sum:a),, 2)", mq, (t0, t1))
    assert mq == ["sum:a"] and str(tree) == "scale(absolute(a))"
    got = [list(zip([int(t) for t in s.ts], s.values())) for s in tree.evaluate(eng, results)]
    inner = [o for o, _ in OX.absolute([(p, b"") for p in raw])]
    same(got, [o for o, _ in OX.scale([(p, b"") for p in inner], 2.0)])
    tree = T.parse("movingAverage(scale(sum:a,,3),, 4)", [], (t0, t1))   # (a space inside a nested
    # call ends the parameter: ExpressionReader.readNextParameter stops at whitespace)
    got = [list(zip([int(t) for t in s.ts], s.values())) for s in tree.evaluate(eng, results)]
    inner = [o for o, _ in OX.scale([(p, b"") for p in raw], 3.0)]
    same(got, [o for o, _ in OX.moving_average([(p, b"") for p in inner], 4, False, t0, t1)])
    [tree] = T.parse_expressions(["sumSeries(sum:a, sum:b)"], (t0, t1), [])
    got = [list(zip([int(t) for t in s.ts], s.values())) for s in tree.evaluate(eng, results)]
    want = [o for o, _ in OX.combine("+", {"a": [(p, b"") for p in raw], "b": [(p, b"") for p in raw_b]})]
    same(got, want)
