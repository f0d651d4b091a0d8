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


@pytest.mark.parametrize("bad", ["", "a +", "(a", "a & b", "1 + 2"])
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
    """A series that ends before another: RuntimeException (TimeSyncedIterator.next(int));
    JEXL divides by zero: ArithmeticException."""
    a = [([(1, 1), (2, 2)], b"")]
    b = [([(1, 1)], b"")]
    with pytest.raises(OX.OracleExprError):
        OX.combine("+", {"a": a, "b": b})
    with pytest.raises(OX.OracleExprError):
        OX.combine("/", {"a": a, "b": [([(1, 0), (2, 1)], b"")]})


def test_library_exports_expression_symbols():
    from opentsdb_amd import engine as E
    for s in ("tsdbhip_expr_map", "tsdbhip_expr_zip"):
        assert hasattr(E.lib(), s)
