"""The nested-expression host path (opentsdb_amd/expression_tree.py) against the reference's own
tests, transcribed test by test: TestExpressions (test/query/expression/TestExpressions.java:48-129),
TestExpressionReader (TestExpressionReader.java:27-204) and TestExpressionTree
(TestExpressionTree.java:83-265, with its TreeTestExpr as a registered test function), plus the
SyntaxChecker grammar (src/parser.jj) that Expressions.parseExpressions runs (no reference test)."""
from __future__ import annotations

import pytest

from opentsdb_amd import expression_tree as T
from opentsdb_amd.expression import ExpressionError


class Foo(T.Function):
    """TestExpressions.FooExpression (:134-146)."""

    def __init__(self):
        super().__init__("foo", impl=lambda *a: [], writer=lambda params, inner: "foo(" + inner + ")")

    def evaluate(self, engine, data_query, results, params):
        return []


class TreeTestExpr(T.Function):
    """TestExpressionTree.TreeTestExpr (:293-318): records its inputs, returns one slot per
    incoming series."""

    def __init__(self):
        super().__init__("treeTestExpr", writer=lambda params, inner: "treeTestExpr(" + inner + ")")
        self.data_query = self.results = self.params = None
        self.query_results = None

    def evaluate(self, engine, data_query, results, params):
        self.data_query, self.results, self.params = data_query, results, params
        return [None] * sum(len(r) for r in self.query_results)


@pytest.fixture(autouse=True)
def registry():
    T.add_function("foo", Foo())
    yield


def raises(java, fn, *a):
    with pytest.raises(ExpressionError) as ei:
        fn(*a)
    assert ei.value.java == java
    return ei.value


# ---- TestExpressions -----------------------------------------------------------------------
DQ = (1356998400000, 1356998700000)


def test_parse():
    assert str(T.parse("scale(sys.cpu)", [], DQ)) == "scale()"
    assert str(T.parse("   scale(sys.cpu)", [], DQ)) == "scale()"        # parseWithWhitespace


def test_parse_multi_parameter():
    mq = []
    tree = T.parse("foo(sum:proc.sys.cpu,, sum:proc.meminfo.memfree)", mq, None)
    assert str(tree) == "foo(proc.sys.cpu,proc.meminfo.memfree)"
    assert mq == ["sum:proc.sys.cpu", "sum:proc.meminfo.memfree"]
    assert tree.func_params is None


def test_parse_nested_expr():
    mq = []
    tree = T.parse("foo(sum:proc.sys.cpu,, foo(sum:proc.a.b))", mq, None)
    assert str(tree) == "foo(foo(proc.a.b),proc.sys.cpu)"
    assert mq == ["sum:proc.sys.cpu", "sum:proc.a.b"]
    assert tree.func_params is None


def test_parse_expr_with_param():
    mq = []
    tree = T.parse("foo(sum:proc.sys.cpu,, 100,, 3.1415)", mq, None)
    assert str(tree) == "foo(proc.sys.cpu)"
    assert mq == ["sum:proc.sys.cpu"]
    assert tree.func_params == ["100", "3.1415"]


@pytest.mark.parametrize("expr", [None, "", "scalesys.cpu)", "scale(sys.cpu"])
def test_parse_invalid(expr):
    raises("IllegalArgumentException", T.parse, expr, [], DQ)


def test_parse_null_metric_queries_and_query():
    assert str(T.parse("scale(sys.cpu)", None, DQ)) == "scale()"
    assert str(T.parse("scale(sys.cpu)", [], None)) == "scale()"


# ---- TestExpressionReader -------------------------------------------------------------------
EXP = "test(sys.cpu.user)"


def test_reader_ctor_and_peek():
    r = T.ExpressionReader(EXP)
    assert str(r) == EXP and r.getMark() == 0 and r.peek() == "t"
    raises("IllegalArgumentException", T.ExpressionReader, None)
    r.next()
    assert r.getMark() == 1 and r.peek() == "e" and r.getMark() == 1


def test_reader_empty():
    r = T.ExpressionReader("")
    assert r.getMark() == 0 and r.isEOF()
    for f in (r.peek, r.next, lambda: r.isNextChar("o"), r.readFuncName):
        raises("NoSuchElementException", f)
    r.readNextParameter()
    assert not r.isNextSeq("laska")
    r.skipWhitespaces()
    r.skip(52)


def test_reader_next_skip():
    r = T.ExpressionReader(EXP)
    assert [r.next() for _ in EXP] == list(EXP) and r.isEOF()
    r = T.ExpressionReader(EXP)
    r.skip(4)
    assert r.getMark() == 4 and r.peek() == "("
    r = T.ExpressionReader(EXP)
    r.skip(len(EXP))
    assert r.getMark() == len(EXP) and r.isEOF()
    raises("UnsupportedOperationException", T.ExpressionReader(EXP).skip, -1)


def test_reader_is_next():
    r = T.ExpressionReader(EXP)
    assert r.isNextChar("t")
    r.skip(4)
    assert r.isNextChar("(") and not r.isNextChar("t")
    r = T.ExpressionReader(EXP)
    assert r.isNextSeq("test(") and not r.isNextSeq("est(") and r.isNextSeq(EXP) and not r.isNextSeq(EXP + "morestuff")


def test_reader_read_func_name():
    r = T.ExpressionReader(EXP)
    assert [r.readFuncName(), r.readFuncName(), r.readFuncName()] == ["test", "", ""] and not r.isEOF()
    for text in ("test (foo)", "  test(foo)", "  test(foo)  "):
        r = T.ExpressionReader(text)
        assert [r.readFuncName(), r.readFuncName()] == ["test", ""]
    r = T.ExpressionReader("test(foo(bar()))")
    assert [r.readFuncName(), r.readFuncName(), r.readFuncName()] == ["test", "", ""]
    for text, third in (("test(foo(bar()))", "bar"), ("test ( foo ( bar()))", "bar"), ("test ( foo  bar()))", "ar")):
        r = T.ExpressionReader(text)
        assert r.readFuncName() == "test"
        r.next()
        assert r.readFuncName() == "foo"
        r.next()
        assert r.readFuncName() == third
    assert T.ExpressionReader("test ").readFuncName() == "test"


def test_reader_read_next_parameter():
    assert T.ExpressionReader(EXP).readNextParameter() == EXP
    r = T.ExpressionReader(EXP)
    r.readFuncName()
    assert r.readNextParameter() == "(sys.cpu.user)"
    r = T.ExpressionReader("test(foo,1,2)")
    r.readFuncName()
    r.next()
    assert r.readNextParameter() == "foo,1,2"


# ---- TestExpressionTree ---------------------------------------------------------------------
METRIC = "sys.cpu"
NAME = "treeTestExpr"


@pytest.fixture
def tree_expr():
    e = TreeTestExpr()
    e.query_results = [["dps"]]
    T.add_function(NAME, e)
    return e


def test_tree_ctor(tree_expr):
    for t in (T.ExpressionTree(NAME, DQ), T.ExpressionTree(tree_expr, DQ)):
        assert str(t) == NAME + "()"
        assert t.sub_expressions is None and t.func_params is None and t.sub_metric_queries is None
        assert t.parameter_index == {}
    for name in (None, "", "No such method"):
        raises("UnsupportedOperationException", T.ExpressionTree, name, DQ)


def test_tree_add_sub_expression(tree_expr):
    t = T.ExpressionTree(NAME, DQ)
    child = T.ExpressionTree("scale", DQ)
    t.addSubExpression(child, 1)
    assert t.sub_expressions == [child] and t.func_params is None and t.sub_metric_queries is None
    assert t.parameter_index == {1: T.SUB_EXPRESSION}
    raises("IllegalArgumentException", T.ExpressionTree(NAME, DQ).addSubExpression, None, 1)
    t2 = T.ExpressionTree(NAME, DQ)
    raises("IllegalDataException", t2.addSubExpression, t2, 1)


def test_tree_add_sub_metric_query(tree_expr):
    t = T.ExpressionTree(NAME, DQ)
    t.addSubMetricQuery(METRIC, 1, 1)
    assert str(t) == NAME + "(" + METRIC + ")"
    assert t.sub_metric_queries == {1: METRIC} and t.parameter_index == {1: T.METRIC_QUERY}
    for args in ((None, 1, 1), ("", 1, 1), (METRIC, -1, 1), (METRIC, 1, -1)):
        raises("IllegalArgumentException", T.ExpressionTree(NAME, DQ).addSubMetricQuery, *args)


def test_tree_add_function_parameter(tree_expr):
    t = T.ExpressionTree(NAME, DQ)
    t.addFunctionParameter("vimes")
    assert str(t) == NAME + "()" and t.func_params == ["vimes"] and t.parameter_index == {}
    for p in (None, ""):
        raises("IllegalArgumentException", T.ExpressionTree(NAME, DQ).addFunctionParameter, p)


def test_tree_evaluate(tree_expr):
    qr = tree_expr.query_results
    t = T.ExpressionTree(NAME, DQ)                                   # evaluateNothingSet
    assert len(t.evaluate(None, qr)) == 1
    assert tree_expr.data_query is DQ and tree_expr.results == [] and tree_expr.params is None
    t = T.ExpressionTree(NAME, DQ)                                   # evaluateSubMetricQuerySet
    t.addSubMetricQuery(METRIC, 0, 0)
    assert len(t.evaluate(None, qr)) == 1 and len(tree_expr.results) == 1 and tree_expr.params is None
    t.addFunctionParameter("foo")                                    # ...WithParam
    assert str(t) == NAME + "(" + METRIC + ")"
    assert len(t.evaluate(None, qr)) == 1 and tree_expr.params == ["foo"]


def test_tree_evaluate_sub_expression(tree_expr):
    calls = []

    class Scale(T.Function):
        def __init__(self):
            super().__init__("scale")

        def evaluate(self, engine, data_query, results, params):
            calls.append((results, params))
            return results[0]

    child = T.ExpressionTree(Scale(), DQ)
    child.addSubMetricQuery(METRIC, 0, 0)
    child.addFunctionParameter("1")
    t = T.ExpressionTree(NAME, DQ)
    t.addSubExpression(child, 0)
    assert str(t) == NAME + "(scale(" + METRIC + "))"
    assert len(t.evaluate(None, tree_expr.query_results)) == 1
    assert len(tree_expr.results) == 1 and tree_expr.params is None and len(calls) == 1


def test_tree_evaluate_parameter_index_gap(tree_expr):
    """A string parameter between two series leaves index 1 without a series: ExpressionTree
    .evaluate reads parameter_index.get(1) == null and throws (ExpressionTree.java:162-180)."""
    mq = []
    t = T.parse(NAME + "(sum:a,, 100,, sum:b)", mq, DQ)
    raises("IllegalDataException", t.evaluate, None, [["x"], ["y"]])


# ---- the SyntaxChecker grammar (src/parser.jj) -----------------------------------------------
def test_parse_expressions_grammar():
    mq = []
    trees = T.parse_expressions(["foo(sum:1m-avg:rate:sys.cpu{host=web01,dc=lga}, 10, foo(max:a.b))",
                                 "scale(sum:x, 2)"], DQ, mq)
    assert mq == ["sum:1m-avg:rate:sys.cpu{host=web01,dc=lga}", "max:a.b", "sum:x"]
    assert str(trees[0]) == "foo(foo(a.b),sys.cpu)" and trees[0].func_params == ["10"]
    assert str(trees[1]) == "scale(x)" and trees[1].func_params == ["2"]
    assert trees[1].sub_metric_queries == {2: "sum:x"}
    e = raises("IllegalArgumentException", T.parse_expressions, ["foo(sum:a"], DQ, [])
    assert "Failed to parse foo(sum:a" in str(e)
    raises("UnsupportedOperationException", T.parse_expressions, ["nosuch(sum:a)"], DQ, [])
    raises("TokenMgrError", T.parse_expressions, ["foo(sum:a%b)"], DQ, [])
