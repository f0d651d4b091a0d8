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
import re
from dataclasses import dataclass

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

    @classmethod
    def of(cls, points, key=b"", name=""):
        """points: [(ts, value)] -- ints are longs, floats doubles."""
        ts = np.array([p[0] for p in points], np.int64)
        bits = np.array([(p[1] & 0xFFFFFFFFFFFFFFFF) if isinstance(p[1], (int, np.integer)) and not isinstance(p[1], bool)
                         else int(np.float64(p[1]).view(np.uint64)) for p in points], np.uint64)
        is_int = np.array([1 if isinstance(p[1], (int, np.integer)) else 0 for p in points], np.uint8)
        return cls(ts, bits, is_int, key, name)

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


# ---- JEXL subset: + - * / % unary minus, parentheses, numbers, variables -------------------
_TOK = re.compile(r"\s*(?:(\d+\.\d*|\.\d+|\d+)|([A-Za-z_][A-Za-z0-9_.]*)|(.))")


def compile_expression(text: str):
    """Postfix program [(op, arg)], constants, variable names (first-use order)."""
    toks = []
    for m in _TOK.finditer(text):
        num, name, op = m.groups()
        if num is not None:
            toks.append(("num", float(num)))
        elif name is not None:
            toks.append(("var", name))
        elif op and op.strip():
            if op not in "+-*/%()":
                raise ExpressionError("IllegalArgumentException", f"unsupported token {op!r} in {text!r}")
            toks.append(("op", op))
    prog, consts, names = [], [], []
    pos = 0

    def peek():
        return toks[pos] if pos < len(toks) else (None, None)

    def primary():
        nonlocal pos
        kind, v = peek()
        if kind == "num":
            pos += 1
            consts.append(v)
            prog.append((XOP_CONST, len(consts) - 1))
        elif kind == "var":
            pos += 1
            if v not in names:
                names.append(v)
            prog.append((XOP_VAR, names.index(v)))
        elif (kind, v) == ("op", "("):
            pos += 1
            additive()
            if peek() != ("op", ")"):
                raise ExpressionError("IllegalArgumentException", f"unbalanced parentheses in {text!r}")
            pos += 1
        elif (kind, v) == ("op", "-"):
            pos += 1
            primary()
            prog.append((XOP_NEG, 0))
        else:
            raise ExpressionError("IllegalArgumentException", f"cannot parse {text!r}")

    def multiplicative():
        nonlocal pos
        primary()
        while peek()[0] == "op" and peek()[1] in "*/%":
            o = peek()[1]
            pos += 1
            primary()
            prog.append(({"*": XOP_MUL, "/": XOP_DIV, "%": XOP_MOD}[o], 0))

    def additive():
        nonlocal pos
        multiplicative()
        while peek()[0] == "op" and peek()[1] in "+-":
            o = peek()[1]
            pos += 1
            multiplicative()
            prog.append((XOP_ADD if o == "+" else XOP_SUB, 0))

    additive()
    if pos != len(toks):
        raise ExpressionError("IllegalArgumentException", f"cannot parse {text!r}")
    if not names:
        raise ExpressionError("IllegalArgumentException", "The expression didn't appear to have any variables")
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
