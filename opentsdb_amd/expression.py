"""Expression functions over query results: host mirror of
src/query/expression/ (ExpressionFactory.java:41-63) on top of libtsdbhip's k_expr kernels.

A result series is a :class:`Series`: its points (ts, value bits, is_int -- the tsdbhip_result
layout), a join key (the flattened tag UIDs UnionIterator.flattenTags builds; series of one
variable with equal keys keep the last) and a name.  Functions take, like Expression.evaluate,
the list of sub-query results (each a list of Series) and the string parameters, validate them as
the reference does (IllegalArgumentException -> :class:`ExpressionError`) and run the arithmetic on
the GPU:

  alias / scale / absolute / shift, timeShift / movingAverage   tsdbhip_expr_map
  sumSeries, sum / diffSeries, difference / multiplySeries,  tsdbhip_expr_zip (ExpressionIterator
  multiply / divideSeries, divide / evaluate(expression)     with a UNION of the variables)
  highestMax / highestCurrent                                 tsdbhip_expr_topn (AggregationIterator
                                                             over every series, positional maxima)
"""
from __future__ import annotations

import ctypes as C
import math
import re
from dataclasses import dataclass, field

import numpy as np

from . import abi

EXPR_SCALE, EXPR_ABSOLUTE, EXPR_SHIFT, EXPR_MOVING_AVG, EXPR_HIGHEST_MAX, EXPR_HIGHEST_CURRENT = 0, 1, 2, 3, 4, 5
XOP_VAR, XOP_CONST, XOP_ADD, XOP_SUB, XOP_MUL, XOP_DIV, XOP_MOD, XOP_NEG = range(8)


class SeriesSet(C.Structure):
    _fields_ = [("n_series", C.c_int64), ("ptr", C.POINTER(C.c_int64)), ("ts_ms", C.POINTER(C.c_int64)),
                ("value_bits", C.POINTER(C.c_uint64)), ("is_int", C.POINTER(C.c_uint8))]


class ExpressionError(Exception):
    def __init__(self, java: str, msg: str):
        self.java = java
        super().__init__(f"{java}: {msg}")


@dataclass
class Series:
    ts: np.ndarray
    bits: np.ndarray
    is_int: np.ndarray
    key: bytes = b""
    name: str = ""
    tags: dict = field(default_factory=dict)          # {tagk UID: tagv UID} (DataPoints.getTagUids)
    agg_tags: list = field(default_factory=list)      # aggregated tagk UIDs (getAggregatedTagUids)

    @classmethod
    def of(cls, points, key=b"", name="", tags=None, agg_tags=()):
        """points: [(ts, value)] -- ints are longs, floats doubles."""
        ts = np.array([p[0] for p in points], np.int64)
        bits = np.array([(p[1] & 0xFFFFFFFFFFFFFFFF) if isinstance(p[1], (int, np.integer)) and not isinstance(p[1], bool)
                         else int(np.float64(p[1]).view(np.uint64)) for p in points], np.uint64)
        is_int = np.array([1 if isinstance(p[1], (int, np.integer)) else 0 for p in points], np.uint8)
        return cls(ts, bits, is_int, key, name, dict(tags or {}), sorted(agg_tags))

    def values(self):
        return [int(np.int64(b.view(np.int64))) if i else float(b.view(np.float64))
                for b, i in zip(self.bits.view(np.uint64), self.is_int)]


def _pack(series):
    ptr = np.zeros(len(series) + 1, np.int64)
    for i, s in enumerate(series):
        ptr[i + 1] = ptr[i] + len(s.ts)
    cat = lambda xs, dt: np.ascontiguousarray(np.concatenate(xs).astype(dt)) if xs else np.zeros(1, dt)  # noqa: E731
    ts = cat([s.ts for s in series], np.int64)
    bits = cat([s.bits for s in series], np.uint64)
    ii = cat([s.is_int for s in series], np.uint8)
    keep = (ptr, ts, bits, ii)
    ss = SeriesSet(len(series), ptr.ctypes.data_as(C.POINTER(C.c_int64)), ts.ctypes.data_as(C.POINTER(C.c_int64)),
                   bits.ctypes.data_as(C.POINTER(C.c_uint64)), ii.ctypes.data_as(C.POINTER(C.c_uint8)))
    return ss, keep


def _unpack(res, names, keys):
    out = []
    r = res.contents
    for g in range(r.n_groups):
        a, b = r.group_ptr[g], r.group_ptr[g + 1]
        n = b - a
        ts = np.ctypeslib.as_array(r.ts_ms, (b,))[a:b].copy() if n else np.zeros(0, np.int64)
        bits = np.ctypeslib.as_array(r.value_bits, (b,))[a:b].copy() if n else np.zeros(0, np.uint64)
        ii = np.ctypeslib.as_array(r.is_int, (b,))[a:b].copy() if n else np.zeros(0, np.uint8)
        out.append(Series(ts, bits, ii, keys[g], names[g]))
    return out


def _lib():
    from . import engine as E
    L = E.lib()
    if not getattr(L, "_expr_types", False):
        L.tsdbhip_expr_map.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_int64, C.c_int64, C.c_int64,
                                       C.POINTER(SeriesSet), C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_expr_zip.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int, C.POINTER(C.c_double), C.c_int,
                                       C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_double), C.POINTER(SeriesSet),
                                       C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_expr_topn.argtypes = [C.c_void_p, C.c_int, C.c_int32, C.c_int64, C.c_int64, C.POINTER(SeriesSet),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L._expr_types = True
    return L, E


def _map(engine, fn, series, fparam=0.0, iparam=0, start=-(1 << 62), end=1 << 62):
    L, E = _lib()
    ss, keep = _pack(series)
    res = C.POINTER(abi.Result)()
    E._check(L.tsdbhip_expr_map(engine.ctx, fn, float(fparam), int(iparam), int(start), int(end), C.byref(ss),
                                C.byref(res)))
    try:
        return _unpack(res, [s.name for s in series], [s.key for s in series])
    finally:
        L.tsdbhip_result_free(res)
        del keep


# ---- JEXL 2.1.1 subset -----------------------------------------------------------------------
# commons-jexl 2.1.1 (the reference's pinned build dependency, third_party/jexl/include.mk; not in the
# tree) evaluates an expression over the variables ExpressionIterator binds -- always Doubles -- and the
# literals of the text: integers are Integer / Long, decimals without a suffix Float, with `d` Double.
# JexlArithmetic takes the double path when either operand is a Float or Double (so every
# sub-expression that touches a variable), the integer path (BigInteger, narrowed) otherwise; Booleans
# from comparisons read 1 / 0 there; the lenient interpreter answers a division or modulo error with
# Double 0.0 (TestExpressionIterator.aDivideByZeroWithTwoSeries); negating a Boolean is a logical not.
# The compiler folds the constant sub-expressions with those rules on the host and emits a postfix
# program over doubles for the kernels; its static types say which path each runtime operation takes.
XOP_LT, XOP_GT, XOP_LE, XOP_GE, XOP_EQ, XOP_NE, XOP_NOT, XOP_IDIV, XOP_IMOD = range(8, 17)
_TOK = re.compile(r"\s*(?:(\d+\.\d*(?:[eE][-+]?\d+)?[fFdD]?|\.\d+(?:[eE][-+]?\d+)?[fFdD]?|\d+[lL]?)"
                  r"|([A-Za-z_$][A-Za-z0-9_$.]*)|(<=|>=|==|!=|[-+*/%()<>]))")
_CMP = {"<": XOP_LT, ">": XOP_GT, "<=": XOP_LE, ">=": XOP_GE, "==": XOP_EQ, "!=": XOP_NE}
_ARITH = {"+": XOP_ADD, "-": XOP_SUB, "*": XOP_MUL, "/": XOP_DIV, "%": XOP_MOD}


def _f32(x: float) -> float:
    return float(np.float32(x))


def _const_arith(op, lt, lv, rt, rv):
    """JexlArithmetic on two constants: (type, value); types I (Integer/Long), F (Float), D
    (Double), B (Boolean)."""
    if lt in "FD" or rt in "FD":
        a, b = float(lv), float(rv)
        if op in "/%" and b == 0.0:
            return "D", 0.0
        return "D", {"+": a + b, "-": a - b, "*": a * b, "/": a / b if op == "/" else 0.0,
                     "%": math.fmod(a, b) if op == "%" else 0.0}[op]
    a, b = int(lv), int(rv)
    if op == "+":
        return "I", a + b
    if op == "-":
        return "I", a - b
    if op == "*":
        return "I", a * b
    if op == "/":
        if b == 0:
            return "D", 0.0
        q = abs(a) // abs(b)
        return "I", q if (a >= 0) == (b >= 0) else -q
    if b <= 0:               # BigInteger.mod: modulus not positive -> lenient 0.0
        return "D", 0.0
    return "I", a % b


def compile_expression(text: str):
    """Postfix program [(op, arg)], constants, variable names (first-use order)."""
    if text is None or text == "":
        raise ExpressionError("IllegalArgumentException", "The expression cannot be  null")
    toks = []
    pos = 0
    src = text.rstrip()
    while pos < len(src):
        m = _TOK.match(src, pos)
        if not m or m.end() == pos:
            raise ExpressionError("JexlException", f"cannot parse {text!r}")
        pos = m.end()
        num, name, op = m.groups()
        toks.append(("num", num) if num is not None else ("var", name) if name is not None else ("op", op))
    names = []
    i = 0

    def peek():
        return toks[i] if i < len(toks) else (None, None)

    def take():
        nonlocal i
        i += 1
        return toks[i - 1]

    # AST nodes: ("c", type, value) constants, ("v", index), ("u", op, node), ("b", op, l, r)
    def primary():
        kind, v = peek()
        if kind == "num":
            take()
            if re.fullmatch(r"\d+[lL]?", v):
                return ("c", "I", int(v.rstrip("lL")))
            if v[-1] in "dD":
                return ("c", "D", float(v[:-1]))
            return ("c", "F", _f32(float(v[:-1] if v[-1] in "fF" else v)))
        if kind == "var":
            take()
            if v not in names:
                names.append(v)
            return ("v", names.index(v))
        if (kind, v) == ("op", "("):
            take()
            e = comparison()
            if peek() != ("op", ")"):
                raise ExpressionError("JexlException", f"unbalanced parentheses in {text!r}")
            take()
            return e
        if (kind, v) == ("op", "-"):
            take()
            return ("u", "-", primary())
        raise ExpressionError("JexlException", f"cannot parse {text!r}")

    def binary(sub, ops):
        def f():
            e = sub()
            while peek()[0] == "op" and peek()[1] in ops:
                o = take()[1]
                e = ("b", o, e, sub())
            return e
        return f

    multiplicative = binary(primary, ("*", "/", "%"))
    additive = binary(multiplicative, ("+", "-"))
    comparison = binary(additive, tuple(_CMP))
    ast = comparison()
    if i != len(toks):
        raise ExpressionError("JexlException", f"cannot parse {text!r}")
    if not names:
        raise ExpressionError("IllegalArgumentException", "The expression didn't appear to have any variables")

    prog, consts = [], []

    def typed(node):
        """(static type, constant value or None) with constants folded."""
        k = node[0]
        if k == "c":
            return node[1], node[2]
        if k == "v":
            return "D", None
        if k == "u":
            t, v = typed(node[2])
            if v is not None:
                if t == "B":
                    return "B", not v
                return t, -v
            return ("B" if t == "B" else t), None
        lt, lv = typed(node[2])
        rt, rv = typed(node[3])
        if node[1] in _CMP:
            if lv is not None and rv is not None:
                a, b = (float(lv), float(rv)) if (lt in "FD" or rt in "FD") else (int(lv), int(rv))
                return "B", {"<": a < b, ">": a > b, "<=": a <= b, ">=": a >= b, "==": a == b, "!=": a != b}[node[1]]
            return "B", None
        if lv is not None and rv is not None:
            return _const_arith(node[1], lt, lv, rt, rv)
        return ("D" if (lt in "FD" or rt in "FD") else "I"), None

    def emit(node):
        t, v = typed(node)
        if v is not None:
            consts.append(float(v))
            prog.append((XOP_CONST, len(consts) - 1))
            return t
        k = node[0]
        if k == "v":
            prog.append((XOP_VAR, node[1]))
            return "D"
        if k == "u":
            st = emit(node[2])
            prog.append((XOP_NOT if st == "B" else XOP_NEG, 0))
            return t
        lt = emit(node[2])
        rt = emit(node[3])
        o = node[1]
        if o in _CMP:
            prog.append((_CMP[o], 0))
        elif lt in "FD" or rt in "FD":
            prog.append((_ARITH[o], 0))
        else:   # integer path (Booleans / integer constants): truncating division, BigInteger.mod
            prog.append(({"/": XOP_IDIV, "%": XOP_IMOD}.get(o, _ARITH[o]), 0))
        return t

    root = emit(ast)
    if root == "I":
        # ExpressionIterator accepts a Double or a Boolean result only (ExpressionIterator.java:347-354)
        raise ExpressionError("IllegalStateException",
                              f"Expression returned a result of type: java.lang.Integer for {text}")
    return prog, consts, names


def union_sets(variables: dict[str, list[Series]]):
    """UnionIterator.computeUnion (UnionIterator.java:140-200): the joined sets in ByteMap order of
    the flattened tag keys, each [series index per variable or -1]; a variable's later series with
    an equal key replaces the earlier."""
    names = list(variables)
    by_key: dict[bytes, list[int]] = {}
    flat = []
    for vi, nm in enumerate(names):
        for s in variables[nm]:
            flat.append(s)
            by_key.setdefault(s.key, [-1] * len(names))[vi] = len(flat) - 1
    keys = sorted(by_key)   # ByteMap: Bytes.memcmp, unsigned lexicographic
    return names, keys, [by_key[k] for k in keys], flat


def evaluate(engine, expression: str, variables: dict[str, list[Series]], fill=None, name="expression"):
    """ExpressionIterator(expression, UNION) over TimeSyncedIterators of each variable's series,
    read as EDPtoDPS does (ExpressionIterator.java:282-318, EDPtoDPS.java:148-160)."""
    prog, consts, expr_names = compile_expression(expression)
    missing = [v for v in expr_names if v.lower() not in {k.lower() for k in variables}]
    if missing:
        raise ExpressionError("IllegalArgumentException", f"Missing results for variable {missing[0]}")
    names, keys, sets, flat = union_sets(variables)
    lower = {k.lower(): i for i, k in enumerate(names)}
    var_index = [lower[v.lower()] for v in expr_names]
    # program variables -> set columns in expression-variable order
    set_series = np.array([[row[var_index[v]] for v in range(len(expr_names))] for row in sets], np.int32).reshape(
        len(sets), len(expr_names))
    fills = np.array([(fill or {}).get(v, 0.0) for v in expr_names], np.float64)   # NumericFillPolicy ZERO
    L, E = _lib()
    ss, keep = _pack(flat)
    p = np.array([x for op in prog for x in op], np.int32)
    cs = np.array(consts or [0.0], np.float64)
    res = C.POINTER(abi.Result)()
    E._check(L.tsdbhip_expr_zip(engine.ctx, p.ctypes.data_as(C.POINTER(C.c_int32)), len(prog),
                                cs.ctypes.data_as(C.POINTER(C.c_double)), len(expr_names), len(sets),
                                np.ascontiguousarray(set_series).ctypes.data_as(C.POINTER(C.c_int32)),
                                fills.ctypes.data_as(C.POINTER(C.c_double)), C.byref(ss), C.byref(res)))
    try:
        return _unpack(res, [name] * len(sets), keys)
    finally:
        L.tsdbhip_result_free(res)
        del keep


# ---- /api/query/exp: ExpressionIterator over UNION / INTERSECTION joins ----------------------
# QueryExecutor (src/tsd/QueryExecutor.java:197-213, 254-443) builds one ExpressionIterator per
# expression: its variables are the sub-queries' results as TimeSyncedIterators (or other
# expressions), joined by tags into sets with a UnionIterator or an IntersectionIterator
# (Join.operator), and serialized by stepping the join in time (:668-708).  The join is host logic
# over the series' tag UIDs (restated below); every step's arithmetic runs on the GPU
# (tsdbhip_expr_sync, k_expr_sync).
def java_hashmap_order(keys, initial_capacity=None):
    """Iteration order of a java.util.HashMap<String, ?> filled with `keys` (new HashMap() or
    new HashMap(initial_capacity)): bucket order of the spread String.hashCode at the final table
    size, ties in insertion order.  The reference iterates such maps to pick the join's first
    sub-query and the variable whose tags an expression's series carry."""
    uniq = list(dict.fromkeys(keys))

    def spread(k):
        h = 0
        for ch in k:
            h = (31 * h + ord(ch)) & 0xFFFFFFFF
        return h ^ (h >> 16)
    if initial_capacity is None:
        n = 16
    else:
        n = 1
        while n < max(1, initial_capacity):
            n <<= 1
    while len(uniq) > n * 0.75:
        n <<= 1
    return sorted(uniq, key=lambda k: (spread(k) & (n - 1), uniq.index(k)))


def flatten_tags(use_query_tags: bool, include_agg_tags: bool, tags: dict, agg_tags, query_tagks) -> bytes:
    """UnionIterator.flattenTags (UnionIterator.java:259-309) / IntersectionIterator.flattenTags
    (:397-444): the tag pairs in UID order -- with use_query_tags only the sub-query's filter tagks,
    none when it has none -- then the aggregated tagks; an empty tag map gives an empty key."""
    if not tags:
        return b""
    qt = set(query_tagks or ())
    out = bytearray()
    for k in sorted(tags):
        if use_query_tags and k not in qt:
            continue
        out += k + tags[k]
    if include_agg_tags:
        for k in sorted(agg_tags):
            out += k
    return bytes(out)


@dataclass
class ResultSet:
    """One sub-query's results as its TimeSyncedIterator sees them: the group-by series (each with
    tags {tagk UID: tagv UID} and aggregated tagk UIDs), the sub-query's filter tagks
    (TSSubQuery.getFilterTagKs) and its NumericFillPolicy value (ZERO unless set)."""
    series: list
    filter_tagks: frozenset = frozenset()
    fill: float = 0.0


@dataclass
class _Member:
    name: str
    entries: list            # [(tags, agg, series index in `flat` or None)] one per series / output set
    query_tagks: object      # None for a nested expression (getQueryTagKs() is null)
    fill: float
    nested: "ExpressionIterator | None" = None


class ExpressionIterator:
    """ExpressionIterator (src/query/expression/ExpressionIterator.java:135-485) as /api/query/exp
    uses it: add_results(), compile(), then the time-synchronised steps (next(timestamp)) that
    QueryExecutor serializes -- computed at once on the GPU by compile(engine, start, end).
    Afterwards `series` holds one Series per joined set (every step's double value, the set's
    tags / aggregated tags as the reference's ExpressionDataPoint carries them) and `steps` the
    step timestamps.  QueryExecutor's defaults: UNION, use_query_tags False, include_agg_tags True
    (:201-204); the expression's own fill is NaN (:156)."""

    def __init__(self, id_: str, expression: str, set_operator: str = "UNION", use_query_tags: bool = False,
                 include_agg_tags: bool = True):
        if expression is None or expression == "":
            raise ExpressionError("IllegalArgumentException", "The expression cannot be  null")
        if set_operator is None:
            raise ExpressionError("IllegalArgumentException", "The set operator cannot be null")
        if set_operator not in ("UNION", "INTERSECTION"):
            raise ExpressionError("IllegalArgumentException", f"unknown set operator {set_operator}")
        self.id = id_
        self.expression = expression
        self.prog, self.consts, self.names = compile_expression(expression)
        self.set_operator = set_operator
        self.use_qt = use_query_tags
        self.inc_agg = include_agg_tags
        self.fill = math.nan
        self.results: dict = {}
        self.series = None
        self.steps = None

    def add_results(self, id_: str, results):
        if id_ is None:
            raise ExpressionError("IllegalArgumentException", "Missing ID")
        if results is None:
            raise ExpressionError("IllegalArgumentException", "Iterator cannot be null")
        self.results[id_] = results

    # -- the join (host) ------------------------------------------------------------------------
    def _members(self, flat):
        order = java_hashmap_order(list(self.results))
        members = []
        for name in order:
            r = self.results[name]
            if isinstance(r, ExpressionIterator):
                entries = []
                for s in r.series:
                    flat.append(s)
                    entries.append((s.tags, s.agg_tags, len(flat) - 1))
                members.append(_Member(name, entries, None, r.fill, r))
            else:
                entries = []
                for s in r.series:
                    if len(s.ts) == 0:   # TimeSyncedIterator keeps no emitter for it: flattenTags NPEs
                        raise ExpressionError("NullPointerException", "a result series without data points")
                    flat.append(s)
                    entries.append((s.tags, s.agg_tags, len(flat) - 1))
                members.append(_Member(name, entries, r.filter_tagks, r.fill))
        return order, members

    def _key(self, m: _Member, e):
        return flatten_tags(self.use_qt, self.inc_agg, e[0], e[1], m.query_tagks)

    def _join(self, order, members, flat):
        """-> (keys in ByteMap order, per key {member name: entry}, active flag per flat series)."""
        # queries = new HashMap(results.size()) filled in results' order: the join's iteration order
        jorder = java_hashmap_order(order, len(order))
        by = {m.name: m for m in members}
        active = [True] * len(flat)
        if self.set_operator == "UNION":          # UnionIterator.computeUnion (:171-244)
            joined: dict = {}
            for name in jorder:
                m = by[name]
                for e in m.entries:
                    joined.setdefault(self._key(m, e), {})[name] = e
            return sorted(joined), joined, active, jorder
        # IntersectionIterator.computeIntersection (:270-359)
        if max((len(m.entries) for m in members), default=0) < 1:
            return [], {}, active, jorder
        first = by[jorder[0]]
        flattened = {first.name: {}}
        inter: dict = {}
        for idx, e in enumerate(first.entries):
            k = self._key(first, e)
            flattened[first.name][k] = idx
            inter[k] = {first.name: e}
        for name in jorder[1:]:
            m = by[name]
            tags = {}
            flattened[name] = tags
            for idx, e in enumerate(m.entries):
                k = self._key(m, e)
                tags[k] = idx
                if k not in inter:
                    if m.nested is None:   # nullIterator; an ExpressionIterator ignores it (:402-408)
                        active[e[2]] = False
                    continue
                inter[k][name] = e
            for k in sorted(inter):
                if k not in tags:
                    for other, ftags in flattened.items():
                        if other == name or k not in ftags:
                            continue
                        om = by[other]
                        if om.nested is None:
                            active[om.entries[ftags[k]][2]] = False
                    del inter[k]
        if len(jorder) > 1 and not inter:
            raise ExpressionError("IllegalDataException", "No intersections found")
        return sorted(inter), inter, active, jorder

    def plan(self):
        """The host half of compile() (:237-302): checks, then the join -> (flattened series,
        members, keys, {key: {member: entry}}, active flags, join order)."""
        if len(self.results) < 1:
            raise ExpressionError("IllegalArgumentException", "No results for any variables in the expression")
        if len(self.results) < len(self.names):
            raise ExpressionError("IllegalArgumentException", "Not enough query results for the expression variables")
        for v in self.names:
            r = self.results.get(v.lower())
            if r is None:
                raise ExpressionError("IllegalArgumentException", "Missing results for variable " + v)
            if isinstance(r, ExpressionIterator) and r.series is None:
                raise ExpressionError("IllegalStateException", f"nested expression {r.id} is not compiled")
        flat: list = []
        order, members = self._members(flat)
        keys, joined, active, jorder = self._join(order, members, flat)
        return flat, members, keys, joined, active, jorder

    def compile(self, engine, start_ms: int = -(1 << 62), end_ms: int = 1 << 62):
        """compile() and the serializer's walk (QueryExecutor.java:668-708): every step whose
        timestamp lies in [start_ms, end_ms].  Nested expressions are compiled first (they are
        consumed as iterators: every step, no window)."""
        for r in self.results.values():
            if isinstance(r, ExpressionIterator) and r.series is None:
                r.compile(engine)
        flat, members, keys, joined, active, jorder = self.plan()
        # a nested expression advances one step per step of this one (ExpressionIterator.next(long)
        # on its own join): the same as reading it in time when every timestamp of the other
        # variables is one of its steps
        nested = [m for m in members if m.nested is not None]
        if nested:
            others = set()
            for m in members:
                if m.nested is None:
                    for e in m.entries:
                        if active[e[2]]:
                            others.update(int(t) for t in flat[e[2]].ts)
            steps0 = set(int(t) for t in nested[0].nested.steps)
            if any(set(int(t) for t in m.nested.steps) != steps0 for m in nested) or not others <= steps0:
                raise ExpressionError("NotImplemented", "a nested expression whose steps the other variables do not share")
        var_member = [v.lower() if v.lower() in self.results else v for v in self.names]
        set_series = np.full((len(keys), len(self.names)), -1, np.int32)
        for j, k in enumerate(keys):
            row = joined[k]
            for vi, mname in enumerate(var_member):
                e = row.get(mname)
                if e is not None:
                    set_series[j, vi] = e[2]
        by = {m.name: m for m in members}
        fills = np.array([by[mname].fill for mname in var_member], np.float64)
        act = np.array([1 if a else 0 for a in active] or [0], np.uint8)
        L, E = _lib()
        if not getattr(L, "_expr_sync_types", False):
            L.tsdbhip_expr_sync.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int, C.POINTER(C.c_double), C.c_int,
                                            C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_double), C.c_double,
                                            C.POINTER(C.c_uint8), C.c_int64, C.c_int64, C.POINTER(SeriesSet),
                                            C.POINTER(C.POINTER(abi.Result))]
            L._expr_sync_types = True
        ss, keep = _pack(flat)
        p = np.array([x for op in self.prog for x in op], np.int32)
        cs = np.array(self.consts or [0.0], np.float64)
        res = C.POINTER(abi.Result)()
        E._check(L.tsdbhip_expr_sync(engine.ctx, p.ctypes.data_as(C.POINTER(C.c_int32)), len(self.prog),
                                     cs.ctypes.data_as(C.POINTER(C.c_double)), len(self.names), len(keys),
                                     np.ascontiguousarray(set_series).ctypes.data_as(C.POINTER(C.c_int32)),
                                     fills.ctypes.data_as(C.POINTER(C.c_double)), 0.0,
                                     act.ctypes.data_as(C.POINTER(C.c_uint8)), int(start_ms), int(end_ms),
                                     C.byref(ss), C.byref(res)))
        try:
            out = _unpack(res, [self.id] * len(keys), keys)
        finally:
            L.tsdbhip_result_free(res)
            del keep
        # ExpressionIterator.compile (:280-297): each set's series carries the tags of the join's
        # first result map entry (current_values, a HashMap in the join's order) -- none for a
        # union's fill -- and the aggregated tags of all
        cur_order = java_hashmap_order(jorder, len(jorder))
        for j, k in enumerate(keys):
            row = joined[k]
            e0 = row.get(cur_order[0])
            out[j].tags = dict(e0[0]) if e0 is not None else {}
            agg = set(e0[1]) if e0 is not None else set()
            for mname in cur_order[1:]:
                e = row.get(mname)
                if e is not None:
                    agg |= set(e[1])
            out[j].agg_tags = sorted(agg)
        self.series = out
        self.steps = out[0].ts.copy() if out else np.zeros(0, np.int64)
        return out


# ---- the graphite-style functions -----------------------------------------------------------
def _flatten(query_results):
    return [s for sub in (query_results or []) for s in sub]


def scale(engine, query_results, params):
    """Scale.evaluate (src/query/expression/Scale.java:34-84)."""
    if not query_results:
        return []
    if not params:
        raise ExpressionError("IllegalArgumentException", "Missing scaling factor")
    f = params[0]
    if f is None or not re.fullmatch(r"[-0-9\.]+", f):
        raise ExpressionError("IllegalArgumentException", "Unparseable scale factor value: 0.0")
    try:
        factor = float(f)
    except ValueError as e:
        raise ExpressionError("IllegalArgumentException", "Invalid parameter, must be an integer or floating point") from e
    return _map(engine, EXPR_SCALE, _flatten(query_results), fparam=factor)


def absolute(engine, query_results, params=None):
    """Absolute.evaluate (Absolute.java:34-62)."""
    if not query_results:
        return []
    return _map(engine, EXPR_ABSOLUTE, _flatten(query_results))


def alias(engine, query_results, params):
    """Alias.evaluate (src/query/expression/Alias.java:38-85): every series renamed to the
    comma-joined parameters -- and, as the reference does (its loop is Absolute's), with the
    absolute value of every point."""
    if not query_results:
        return []
    if not params:
        raise ExpressionError("IllegalArgumentException", "Missing the alias")
    out = _map(engine, EXPR_ABSOLUTE, _flatten(query_results))
    name = ",".join(params)
    for s in out:
        s.name = name
    return out


def _mavg_window_ms(param):
    """MovingAverage.parseParam (MovingAverage.java:125-160): "'<n><unit>'"."""
    idx = 0
    for ch in param[1:]:
        if ch.isdigit():
            idx += 1
        else:
            break
    if idx < 1:
        raise ExpressionError("IllegalArgumentException", f"Invalid moving window parameter: {param}")
    t = int(param[1:idx + 1])
    unit = param[idx + 1:len(param) - 1]
    table = {"day": 86400000, "d": 86400000, "hr": 3600000, "hour": 3600000, "h": 3600000, "min": 60000,
             "m": 60000, "sec": 1000, "s": 1000}
    if unit not in table:
        raise ExpressionError("IllegalArgumentException", f"Unknown time unit={unit} in window={param}")
    return t * table[unit]


def time_shift_parse(param):
    """TimeShift.parseParam (TimeShift.java:83-119): the digits after the first character, then the
    unit (trimmed) -- sec, min, hr, day(s), week(s)."""
    idx = 0
    for ch in param[1:]:
        if ch.isdigit():
            idx += 1
        else:
            break
    if idx == 0:
        raise ExpressionError("RuntimeException", f"Invalid Parameter: {param}")
    t = int(param[1:idx + 1])
    unit = param[idx + 1:].strip()
    table = {"sec": 1000, "min": 60000, "hr": 3600000, "day": 86400000, "days": 86400000, "week": 7 * 86400000,
             "weeks": 7 * 86400000}
    if unit not in table:
        raise ExpressionError("RuntimeException", f"unknown time unit={unit}")
    return t * table[unit]


def shift_series(engine, series, ms):
    """TimeShift.shift(DataPoints, ms) over every series (TimeShift.java:121-141) on the GPU."""
    return _map(engine, EXPR_SHIFT, list(series), iparam=ms)


def shift(engine, query_results, params):
    """TimeShift.evaluate (TimeShift.java:33-60): the first sub-query's series only.  The quoted
    parameter it requires ("'1min'") keeps its closing quote in the unit parseParam reads, so the
    reference raises "unknown time unit" for every such parameter; so does this mirror."""
    if not query_results:
        return []
    if not params:
        raise ExpressionError("IllegalArgumentException", "Need amount of timeshift to perform timeshift")
    p = (params[0] or "").strip()
    if not p:
        raise ExpressionError("IllegalArgumentException", f"Invalid timeshift='{params[0]}'")
    if not (p.startswith("'") and p.endswith("'")):
        raise ExpressionError("RuntimeException", "Invalid timeshift parameter: eg '10min'")
    ms = time_shift_parse(p)
    if ms <= 0:
        raise ExpressionError("RuntimeException", "timeshift <= 0")
    return shift_series(engine, query_results[0], ms)


def moving_average(engine, query_results, params, start_ms, end_ms):
    """MovingAverage.evaluate (MovingAverage.java:60-123) with the TSQuery's start / end."""
    if not query_results:
        return []
    if not params or not params[0]:
        raise ExpressionError("IllegalArgumentException", "Missing moving average window size")
    p = params[0].strip()
    if re.fullmatch(r"[0-9]+", p):
        cond, timed = int(p), False
    elif p.startswith("'") and p.endswith("'"):
        cond, timed = _mavg_window_ms(p), True
    else:
        raise ExpressionError("IllegalArgumentException", f"Unparseable window size: {p}")
    if cond <= 0:
        raise ExpressionError("IllegalArgumentException", "Moving average window must be an integer greater than zero")
    return _map(engine, EXPR_MOVING_AVG, _flatten(query_results), fparam=1.0 if timed else 0.0, iparam=cond,
                start=start_ms, end=end_ms)


def _combine(op, fname):
    def f(engine, query_results, params=None):
        """SumSeries / DiffSeries / MultiplySeries / DivideSeries.evaluate: 'a op b op ...' through an
        ExpressionIterator with a UNION of the sub-queries (e.g. DivideSeries.java:35-75)."""
        if not query_results:
            return []
        if len(query_results) < 2 or len(query_results) > 26:
            raise ExpressionError("IllegalArgumentException",
                                  f"Must have 2 to 26 series, got {len(query_results)} instead")
        letters = [chr(ord("a") + i) for i in range(len(query_results))]
        return evaluate(engine, f" {op} ".join(letters), dict(zip(letters, query_results)), name=fname)
    f.__name__ = fname
    return f


def topn_parse(params):
    """The top-n parameter of HighestMax / HighestCurrent.evaluate (HighestMax.java:47-72)."""
    if not params:
        raise ExpressionError("IllegalArgumentException", "Need aggregation window for moving average")
    p = params[0]
    if p is None or p == "":
        raise ExpressionError("IllegalArgumentException", "Missing top n value (number of series to return)")
    if not re.fullmatch(r"[0-9]+", p):
        raise ExpressionError("IllegalArgumentException", "Unparseable top n value: " + p)
    n = int(p)
    if n > (1 << 31) - 1:
        raise ExpressionError("IllegalArgumentException", "Invalid parameter, must be an integer")
    if n < 1:
        raise ExpressionError("IllegalArgumentException", f"Top n value must be greater than zero: {n}")
    return n


def _highest(fn, fname):
    def f(engine, query_results, params, start_ms, end_ms):
        """HighestMax / HighestCurrent.evaluate with the TSQuery's start / end: the top-n series of
        every sub-query's group-bys, as tsdbhip_expr_topn ranks them on the GPU; the series are
        returned unchanged."""
        if not query_results:
            return []
        n = topn_parse(params)
        flat = _flatten(query_results)
        if not flat:
            return []
        L, E = _lib()
        ss, keep = _pack(flat)
        idx = (C.c_int32 * len(flat))()
        cnt = C.c_int32(0)
        E._check(L.tsdbhip_expr_topn(engine.ctx, fn, n, int(start_ms), int(end_ms), C.byref(ss), idx, C.byref(cnt)))
        del keep
        return [flat[idx[i]] for i in range(cnt.value)]
    f.__name__ = fname
    return f


highest_max = _highest(EXPR_HIGHEST_MAX, "highestMax")
highest_current = _highest(EXPR_HIGHEST_CURRENT, "highestCurrent")

sum_series = _combine("+", "sumSeries")
diff_series = _combine("-", "diffSeries")
multiply_series = _combine("*", "multiplySeries")
divide_series = _combine("/", "divideSeries")

FUNCTIONS = {
    "alias": alias, "scale": scale, "absolute": absolute, "movingAverage": moving_average, "shift": shift, "timeShift": shift,
    "divideSeries": divide_series, "divide": divide_series, "sumSeries": sum_series, "sum": sum_series,
    "diffSeries": diff_series, "difference": diff_series, "multiplySeries": multiply_series,
    "multiply": multiply_series, "highestMax": highest_max, "highestCurrent": highest_current,
}
