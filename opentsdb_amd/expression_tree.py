"""Nested graphite-style expressions: the host restatement of Expressions.parse, ExpressionReader,
ExpressionTree and the JavaCC grammar's SyntaxChecker (src/query/expression/Expressions.java:43-163,
ExpressionReader.java:23-156, ExpressionTree.java:41-257, src/parser.jj), evaluating every node
through the GPU functions of :mod:`opentsdb_amd.expression` (ExpressionFactory's registry).

A tree's leaves are sub metric queries (indices into the query results the caller runs, e.g.
"sum:sys.cpu{host=*}") and string parameters; its inner nodes are functions.  Evaluation walks the
parameter indices in order, materialises each leaf or sub-tree, and calls the node's function
with the materialised results and its parameters, as ExpressionTree.evaluate does -- including
its failure on a gap in the parameter indices (a string parameter between two series)."""
from __future__ import annotations

import re

from . import expression as X
from .expression import ExpressionError

# ---- ExpressionFactory (ExpressionFactory.java:30-95) ------------------------------------------
# name -> (the function's evaluate, its writeStringField prefix); "alias" appends its parameters
_WRITERS = {
    "alias": "alias", "scale": "scale", "absolute": "absolute", "movingAverage": "movingAverage",
    "highestCurrent": "highestCurrent", "highestMax": "highestMax", "shift": "timeshift", "timeShift": "timeshift",
    "divideSeries": "divideSeries", "divide": "divideSeries", "sumSeries": "sumSeries", "sum": "sumSeries",
    "diffSeries": "diffSeries", "difference": "diffSeries", "multiplySeries": "multiplySeries",
    "multiply": "multiplySeries",
}
_WINDOWED = {"movingAverage", "highestMax", "highestCurrent"}   # evaluate reads the TSQuery's start / end


class Function:
    """An Expression: evaluate(data_query, results, params) and writeStringField."""

    def __init__(self, name: str, impl=None, writer=None):
        self.name = name
        self.impl = impl
        self.writer = writer

    def evaluate(self, engine, data_query, results, params):
        if self.name in _WINDOWED:
            start, end = query_window(data_query)
            return self.impl(engine, results, params, start, end)
        return self.impl(engine, results, params)

    def write_string_field(self, params, inner: str) -> str:
        if self.writer is not None:
            return self.writer(params, inner)
        prefix = _WRITERS[self.name]
        if self.name == "alias":   # Alias.writeStringField :89-99
            return "alias(" + inner + ("" if not params else "," + ",".join(params)) + ")"
        return prefix + "(" + inner + ")"


_EXTRA: dict[str, Function] = {}


def add_function(name: str, fn: Function):
    """ExpressionFactory.addFunction (:70-78)."""
    if not name:
        raise ExpressionError("IllegalArgumentException", "Missing function name")
    if fn is None:
        raise ExpressionError("IllegalArgumentException", "Function cannot be null")
    _EXTRA[name] = fn


def get_by_name(name) -> Function:
    """ExpressionFactory.getByName (:87-94)."""
    if name in _EXTRA:
        return _EXTRA[name]
    if name in X.FUNCTIONS:
        return Function(name, X.FUNCTIONS[name])
    raise ExpressionError("UnsupportedOperationException", f"Function {name} has not been implemented")


def query_window(data_query):
    """TSQuery.startTime() / endTime() in ms: an object with start_ms / end_ms, startTime() /
    endTime(), or a (start_ms, end_ms) pair."""
    if data_query is None:
        raise ExpressionError("NullPointerException", "no TSQuery for a windowed function")
    if isinstance(data_query, tuple):
        return data_query
    if hasattr(data_query, "start_ms"):
        return data_query.start_ms, data_query.end_ms
    return data_query.startTime(), data_query.endTime()


# ---- ExpressionReader (ExpressionReader.java:23-156) ---------------------------------------------
def _ws(c: str) -> bool:   # Character.isWhitespace over the characters an expression holds
    return c in " \t\n\r\x0b\x0c\x1c\x1d\x1e\x1f"


class ExpressionReader:
    def __init__(self, chars):
        if chars is None:
            raise ExpressionError("IllegalArgumentException", "Character set cannot be null")
        self.chars = list(chars)
        self.mark = 0

    def getMark(self) -> int:
        return self.mark

    def isEOF(self) -> bool:
        return self.mark >= len(self.chars)

    def peek(self) -> str:
        if self.isEOF():
            raise ExpressionError("NoSuchElementException", f"Index {self.mark} is out of bounds {len(self.chars)}")
        return self.chars[self.mark]

    def next(self) -> str:
        c = self.peek()
        self.mark += 1
        return c

    def skip(self, num: int):
        if num < 0:
            raise ExpressionError("UnsupportedOperationException", "Skipping backwards is not allowed")
        self.mark += num

    def isNextChar(self, c: str) -> bool:
        return self.peek() == c

    def isNextSeq(self, seq) -> bool:
        if seq is None:
            raise ExpressionError("IllegalArgumentException", "Comparative sequence cannot be null")
        for i, ch in enumerate(seq):
            if self.mark + i >= len(self.chars) or self.chars[self.mark + i] != ch:
                return False
        return True

    def readFuncName(self) -> str:
        self.skipWhitespaces()
        out = []
        while self.peek() != "(" and not _ws(self.peek()):
            out.append(self.next())
        self.skipWhitespaces()
        return "".join(out)

    def skipWhitespaces(self):
        while self.mark < len(self.chars) and _ws(self.chars[self.mark]):
            self.mark += 1

    def readNextParameter(self) -> str:
        out = []
        nested = 0
        while not self.isEOF() and not _ws(self.peek()):
            ch = self.peek()
            if ch == "(":
                nested += 1
            elif ch == ")":
                nested -= 1
            if nested < 0:
                break
            if nested <= 0 and self.isNextSeq(",,"):
                break
            out.append(self.next())
        return "".join(out)

    def __str__(self):
        return "".join(self.chars)


# ---- ExpressionTree (ExpressionTree.java:41-257) -------------------------------------------------
SUB_EXPRESSION, METRIC_QUERY = "SUB_EXPRESSION", "METRIC_QUERY"


class ExpressionTree:
    def __init__(self, expression, data_query=None):
        self.expression = expression if isinstance(expression, Function) else get_by_name(expression)
        self.data_query = data_query
        self.sub_expressions = None
        self.func_params = None
        self.sub_metric_queries = None   # {sub query index: metric query}
        self.parameter_index = {}        # {parameter index: SUB_EXPRESSION / METRIC_QUERY}

    def addSubExpression(self, child, param_index: int):
        if child is None:
            raise ExpressionError("IllegalArgumentException", "Cannot add a null child tree")
        if child is self:
            raise ExpressionError("IllegalDataException", f"Recursive sub expression detected: {self}")
        if param_index < 0:
            raise ExpressionError("IllegalArgumentException", "Parameter index must be 0 or greater")
        if self.sub_expressions is None:
            self.sub_expressions = []
        self.sub_expressions.append(child)
        self.parameter_index[param_index] = SUB_EXPRESSION

    def addSubMetricQuery(self, metric_query, sub_query_index: int, param_index: int):
        if not metric_query:
            raise ExpressionError("IllegalArgumentException", "Metric query cannot be null or empty")
        if sub_query_index < 0:
            raise ExpressionError("IllegalArgumentException", "Sub query index must be 0 or greater")
        if param_index < 0:
            raise ExpressionError("IllegalArgumentException", "Parameter index must be 0 or greater")
        if self.sub_metric_queries is None:
            self.sub_metric_queries = {}
        self.sub_metric_queries[sub_query_index] = metric_query
        self.parameter_index[param_index] = METRIC_QUERY

    def addFunctionParameter(self, param):
        if not param:
            raise ExpressionError("IllegalArgumentException", "Parameter cannot be null or empty")
        if self.func_params is None:
            self.func_params = []
        self.func_params.append(param)

    def evaluate(self, engine, query_results):
        """The materialised parameters in index order, then the node's function.  A parameter index
        without a series (a string parameter between two series) fails as the reference does."""
        materialized = []
        keys = sorted(self.sub_metric_queries) if self.sub_metric_queries else None
        metric_pointer = sub_pointer = 0
        for i in range(len(self.parameter_index)):
            param = self.parameter_index.get(i)
            if param == METRIC_QUERY:
                if keys is None:
                    raise ExpressionError("RuntimeException", "Attempt to read metric results when none exist")
                materialized.append(query_results[keys[metric_pointer]])
                metric_pointer += 1
            elif param == SUB_EXPRESSION:
                materialized.append(self.sub_expressions[sub_pointer].evaluate(engine, query_results))
                sub_pointer += 1
            else:
                raise ExpressionError("IllegalDataException", f"Unknown parameter type: null in tree: {self}")
        return self.expression.evaluate(engine, self.data_query, materialized, self.func_params)

    def __str__(self):
        return self.writeStringField()

    def writeStringField(self) -> str:
        strs = [str(s) for s in self.sub_expressions or []]
        if self.sub_metric_queries:
            sub = _clean(self.sub_metric_queries[k] for k in sorted(self.sub_metric_queries))
            if sub:
                strs.append(sub)
        return self.expression.write_string_field(self.func_params, ",".join(strs))


def _clean(values) -> str:
    """ExpressionTree.clean (:219-236): tags dropped (replaceAll("\\{.*\\}", "")), then the text
    after the last ':' (the metric name)."""
    out = []
    for v in values:
        t = re.sub(r"\{.*\}", "", v)
        ix = t.rfind(":")
        out.append(t if ix < 0 else t[ix + 1:])
    return ",".join(out)


# ---- Expressions.parse (Expressions.java:43-163) --------------------------------------------------
def parse(expression, metric_queries, data_query=None) -> ExpressionTree:
    if not expression:
        raise ExpressionError("IllegalArgumentException", "Expression may not be null or empty")
    if "(" not in expression or ")" not in expression:
        raise ExpressionError("IllegalArgumentException", f"Invalid Expression: {expression}")
    reader = ExpressionReader(expression)
    reader.skipWhitespaces()
    root = ExpressionTree(reader.readFuncName(), data_query)
    reader.skipWhitespaces()
    if reader.peek() == "(":
        reader.next()
        _parse_params(reader, metric_queries, root, data_query)
    return root


def _parse_params(reader, metric_queries, root, data_query):
    index = 0
    reader.skipWhitespaces()
    if reader.peek() != ")":
        _parse_param(reader.readNextParameter(), metric_queries, root, data_query, index)
        index += 1
    while not reader.isEOF():
        reader.skipWhitespaces()
        if reader.peek() == ")":
            return
        if reader.isNextSeq(",,"):
            reader.skip(2)
            reader.skipWhitespaces()
            _parse_param(reader.readNextParameter(), metric_queries, root, data_query, index)
            index += 1
        else:
            raise ExpressionError("IllegalArgumentException",
                                  f"Invalid delimiter in parameter list at pos={reader.getMark()}, expr={reader}")


def _parse_param(param, metric_queries, root, data_query, index):
    if not param:
        raise ExpressionError("IllegalArgumentException", "Parameter cannot be null or empty")
    if param.find("(") > 0 and param.find(")") > 0:
        root.addSubExpression(parse(param, metric_queries, data_query), index)
    elif ":" in param:
        if metric_queries is None:
            raise ExpressionError("NullPointerException", "metric_queries")
        metric_queries.append(param)
        root.addSubMetricQuery(param, len(metric_queries) - 1, index)
    else:
        root.addFunctionParameter(param)


# ---- Expressions.parseExpressions: the JavaCC SyntaxChecker (src/parser.jj) ------------------------
_NAME = re.compile(r"[*A-Za-z0-9\-_#/$@|.'\]\[]+")


def _tokens(text: str):
    """The grammar's tokens: NAME, "&&" (PARAM) and the literal punctuation; whitespace skipped.
    Any other character is a lexical error (TokenMgrError)."""
    out, i = [], 0
    while i < len(text):
        c = text[i]
        if c in " \t\n\r":
            i += 1
            continue
        if text.startswith("&&", i):
            out.append(("PARAM", "&&"))
            i += 2
            continue
        m = _NAME.match(text, i)
        if m:
            out.append(("NAME", m.group(0)))
            i = m.end()
            continue
        if c in "(),:{}=":
            out.append((c, c))
            i += 1
            continue
        raise ExpressionError("TokenMgrError", f"Lexical error at column {i + 1}. Encountered: {c!r}")
    out.append(("EOF", ""))
    return out


class _Checker:
    def __init__(self, text, data_query, metric_queries):
        self.t = _tokens(text)
        self.p = 0
        self.data_query = data_query
        self.metric_queries = metric_queries

    def kind(self, k=0):
        return self.t[min(self.p + k, len(self.t) - 1)][0]

    def take(self, kind):
        if self.kind() != kind:
            raise ExpressionError("ParseException", f"Encountered {self.t[self.p][1]!r}, expected {kind}")
        tok = self.t[self.p][1]
        self.p += 1
        return tok

    def expression(self):
        tree = ExpressionTree(self.take("NAME"), self.data_query)
        self.take("(")
        index = 0
        self.parameter(tree, index)
        index += 1
        while self.kind() == ",":
            self.take(",")
            self.parameter(tree, index)
            index += 1
        self.take(")")
        return tree

    def parameter(self, tree, index):
        if self.kind() == "NAME" and self.kind(1) == "(":
            tree.addSubExpression(self.expression(), index)
        elif self.kind() == "NAME" and self.kind(1) == ":":
            m = self.metric()
            self.metric_queries.append(m)
            tree.addSubMetricQuery(m, len(self.metric_queries) - 1, index)
        else:
            tree.addFunctionParameter(self.take("NAME"))

    def metric(self):
        parts = [self.take("NAME") + ":"]
        self.take(":")
        for _ in range(2):   # (itvl ":")? (rate ":")?
            if self.kind() == "NAME" and self.kind(1) == ":":
                parts.append(self.take("NAME") + ":")
                self.take(":")
        parts.append(self.take("NAME"))
        if self.kind() == "{":
            self.take("{")
            pairs = []
            while True:
                k = self.take("NAME")
                self.take("=")
                pairs.append(k + "=" + self.take("NAME"))
                if self.kind() != ",":
                    break
                self.take(",")
            self.take("}")
            parts.append("{" + ",".join(pairs) + "}")
        return "".join(parts)


def parse_expressions(expressions, ts_query, metric_queries):
    """Expressions.parseExpressions (:79-96): one tree per expression (single-comma parameter
    lists, metric queries agg[:interval][:rate]:metric[{k=v,...}]); a ParseException becomes
    IllegalArgumentException("Failed to parse ...")."""
    trees = []
    for expr in expressions:
        try:
            trees.append(_Checker(expr, ts_query, metric_queries).expression())
        except ExpressionError as e:
            if e.java == "ParseException":
                raise ExpressionError("IllegalArgumentException", f"Failed to parse {expr}") from e
            raise
    return trees
