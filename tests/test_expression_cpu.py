"""Expression functions on the CPU: the oracle (oracle/expr.py) against the
reference's own known answers (tests/golden/expression.json, tests/golden/make_expression_golden.py),
the host mirror's parsing (TimeShift / MovingAverage parameters, the JEXL subset) and the library's
expression symbols."""
from __future__ import annotations

import pytest

from oracle import expr as OX
from opentsdb_amd import expression as X
from tests import expr_util as U

G = U.golden()


@pytest.mark.parametrize("case", G["cases"], ids=[c["name"] for c in G["cases"]])
def test_oracle_known_answers(case):
    U.check(U.oracle_run(case), case)


@pytest.mark.parametrize("param,ms", G["timeshift_parse"]["cases"])
def test_timeshift_parse_known_answers(param, ms):
    assert X.time_shift_parse(param) == ms


def test_timeshift_shift_known_answers():
    sh = G["timeshift_shift"]
    for idx, ms, want in sh["cases"]:
        out = OX.shift([([tuple(sh["points"][idx])], b"")], ms)
        assert out[0][0][0][0] == want


def test_timeshift_evaluate_rejects_quoted_units_like_the_reference():
    """TimeShift.evaluate requires "'1min'"; parseParam then reads the unit "min'" -> unknown."""
    with pytest.raises(X.ExpressionError) as e:
        X.shift(None, [[X.Series.of([(1, 1)])]], ["'1min'"])
    assert e.value.java == "RuntimeException"


@pytest.mark.parametrize("text,n_ops,names", [("a + b", 3, ["a", "b"]), ("a * (b - 2) / c", 7, ["a", "b", "c"]),
                                              ("-a % 3", 4, ["a"]), ("x.y + x.y", 3, ["x.y"])])
def test_compile_expression(text, n_ops, names):
    prog, consts, nm = X.compile_expression(text)
    assert len(prog) == n_ops and nm == names


@pytest.mark.parametrize("bad", ["", "a +", "(a", "a & b", "1 + 2", "(a > b) + 1"])
def test_compile_expression_rejects(bad):
    with pytest.raises(X.ExpressionError):
        X.compile_expression(bad)


def test_parameter_validation_like_the_reference():
    with pytest.raises(X.ExpressionError):
        X.scale(None, [[X.Series.of([(1, 1)])]], ["abc"])
    with pytest.raises(X.ExpressionError):
        X.moving_average(None, [[X.Series.of([(1, 1)])]], ["0"], 0, 10)
    with pytest.raises(X.ExpressionError):
        X.moving_average(None, [[X.Series.of([(1, 1)])]], ["'5parsecs'"], 0, 10)
    with pytest.raises(X.ExpressionError):
        X.sum_series(None, [[X.Series.of([(1, 1)])]])
    assert X.scale(None, [], ["2"]) == []


def test_oracle_zip_errors():
    """A series that ends before another: RuntimeException (TimeSyncedIterator.next(int)); a
    division by zero is 0.0 (the lenient JEXL interpreter, TestExpressionIterator.java:283-319)."""
    a = [([(1, 1), (2, 2)], b"")]
    b = [([(1, 1)], b"")]
    with pytest.raises(OX.OracleExprError):
        OX.combine("+", {"a": a, "b": b})
    out = OX.combine("/", {"a": a, "b": [([(1, 0), (2, 1)], b"")]})
    assert out[0][0] == [(1, 0.0), (2, 2.0)]


def test_library_exports_expression_symbols():
    from opentsdb_amd import engine as E
    for s in ("tsdbhip_expr_map", "tsdbhip_expr_zip"):
        assert hasattr(E.lib(), s)


# ---- highestMax / highestCurrent --------------------------------------------------------
def _topn_oracle(case):
    subs = [[[tuple(p) for p in s] for s in sub] for sub in case["inputs"]]
    if not subs:
        return []
    n = OX.topn_parse(case["params"])
    flat = [s for sub in subs for s in sub]
    return OX.highest(flat, n, case["start"], case["end"], current=case["fn"] == "highestCurrent")


@pytest.mark.parametrize("case", G["topn"], ids=[c["name"] for c in G["topn"]])
def test_oracle_topn_known_answers(case):
    if case["raises"]:
        with pytest.raises(OX.OracleExprError) as e:
            _topn_oracle(case)
        assert e.value.java == case["raises"]
    else:
        assert _topn_oracle(case) == case["expect_index"]


@pytest.mark.parametrize("case", [c for c in G["topn"] if c["raises"]], ids=lambda c: c["name"])
def test_host_topn_parameter_checks(case):
    """The host mirror rejects the parameters before any device call (engine None)."""
    with pytest.raises(X.ExpressionError) as e:
        X.FUNCTIONS[case["fn"]](None, [[X.Series.of([(1, 1)])]], case["params"], case["start"], case["end"])
    assert e.value.java == case["raises"]


def test_oracle_topn_positional_quirk():
    """MaxCacheAggregator keeps operands by position among the spans with a value, not by
    series: a series absent from the early points has its values credited to another slot."""
    S, I = 1356998400000, 60000
    a = [(S + 2 * I, 100)]                        # starts late
    b = [(S, 1), (S + I, 2), (S + 2 * I, 3)]
    # points S, S+I: only b has a value -> position 0 gets 1, 2 (and a 0 for position 1);
    # S+2I: a=100 at position 0, b=3 at position 1 -> maxima [100, 3]: a first
    assert OX.highest([a, b], 2, S, S + 3 * I) == [0, 1]
    # MaxLatest takes the last point only: [100, 3] as well
    assert OX.highest([a, b], 2, S, S + 3 * I, current=True) == [0, 1]
    # d starts when c has ended: every point has one operand, so c's 50 and 60 land in slot 0
    # -- d's -- and d (max 3) outranks c (max 60)
    c = [(S, 50), (S + I, 60)]
    d = [(S + 2 * I, 3)]
    assert OX.highest([d, c], 1, S, S + 3 * I) == [0]
