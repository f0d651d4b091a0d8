"""TEST INFRASTRUCTURE ONLY -- oracle of the expression functions.

A literal Python restatement of src/query/expression/ over small result series, point by
point in the reference's order (pure-Python loops: small cases only):
  Scale.scale .............. src/query/expression/Scale.java:86-112
  Absolute.abs ............. src/query/expression/Absolute.java:64-83
  TimeShift.shift .......... src/query/expression/TimeShift.java:121-141
  MovingAverage ............ src/query/expression/MovingAverage.java:60-123 (a one-span
                             AggregationIterator over [start, end]) and MovingAverageAggregator
                             .runDouble :262-330 (its LinkedList window, newest first)
  ExpressionIterator ....... src/query/expression/ExpressionIterator.java:282-318 read through
                             EDPtoDPS (EDPtoDPS.java:148-160), UnionIterator.computeUnion
                             (UnionIterator.java:140-200), TimeSyncedIterator.next(int)
                             (TimeSyncedIterator.java:152-160) and JEXL 2.1.1's JexlArithmetic on
                             Doubles (third_party/jexl/include.mk:1, not vendored: +, -, *, /, %; a
                             zero divisor gives 0.0 -- the lenient interpreter, pinned by
                             TestExpressionIterator.aDivideByZeroWithTwoSeries)
  HighestMax / HighestCurrent src/query/expression/HighestMax.java:37-150, :182-292 and
                             HighestCurrent.java:37-151, :172-283: an AggregationIterator
                             (src/core/AggregationIterator.java:395-797, LERP, no rate) over every
                             result series with MaxCacheAggregator / MaxLatestAggregator, then
                             TopNSortingEntry (descending Double.compare, stable Arrays.sort)
Series are (points, key): points [(ts, value)] with int = long, float = double.
"""
from __future__ import annotations

import math
import struct


class OracleExprError(Exception):
    def __init__(self, java, msg=""):
        self.java = java
        super().__init__(f"{java}: {msg}")


def _j_long(x):   # Java long wrap
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >> 63 else x


def _d2l(d):      # (long) d
    if d != d:
        return 0
    if d >= 9.223372036854775807e18:
        return (1 << 63) - 1
    if d <= -9.223372036854775808e18:
        return -(1 << 63)
    return int(d)


def to_double(v):
    return float(v)


def scale(series, factor):
    scale_is_int = factor == math.floor(factor) and not math.isinf(factor)
    out = []
    for pts, key in series:
        o = []
        for ts, v in pts:
            if isinstance(v, int) and scale_is_int:
                o.append((ts, _j_long(_d2l(factor) * v)))
            else:
                o.append((ts, factor * float(v)))
        out.append((o, key))
    return out


def absolute(series):
    out = []
    for pts, key in series:
        o = []
        for ts, v in pts:
            if isinstance(v, int):
                o.append((ts, _j_long(-v) if v < 0 else v))
            else:
                o.append((ts, math.fabs(v) if v == v else float("nan")))
        out.append((o, key))
    return out


def shift(series, ms):
    out = []
    for pts, key in series:
        o = []
        for ts, v in pts:
            if not isinstance(v, int):
                raise OracleExprError("ClassCastException", "Not a long")
            o.append((ts + ms, v))
        out.append((o, key))
    return out


class _MovingAverageAggregator:
    def __init__(self, condition, is_time_unit):
        self.acc = []            # LinkedList, index 0 = first (newest)
        self.condition = condition
        self.timed = is_time_unit
        self.started = False

    def run_double(self, ts, value):
        self.acc.insert(0, (ts, value))
        if self.timed and not self.started:
            self.started = True
            return 0.0
        s, count, met = 0.0, 0, False
        cum, last = 0, -1
        i = 0
        while i < len(self.acc):
            t, v = self.acc[i]
            i += 1
            if self.timed:
                if last < 0:
                    last = t
                else:
                    cum += last - t
                    last = t
                    if cum >= self.condition:
                        met = True
                        break
            v = float(v)
            if v == v:
                s += v
                count += 1
            if not self.timed and count >= self.condition:
                met = True
                break
        del self.acc[i:]
        if not met or count == 0:
            return 0.0
        return s / count


def moving_average(series, condition, timed, start, end):
    out = []
    for pts, key in series:
        agg = _MovingAverageAggregator(condition, timed)
        o = []
        # the one-span AggregationIterator: seek(start), then points while ts <= end
        i = 0
        while i < len(pts) and pts[i][0] < start:
            i += 1
        while i < len(pts) and pts[i][0] <= end:
            ts, v = pts[i]
            o.append((ts, agg.run_double(ts, float(v))))   # PostAggregatedDataPoints: doubles
            i += 1
        out.append((o, key))
    return out


def _jexl(op, l, r):
    if op == "+":
        return l + r
    if op == "-":
        return l - r
    if op == "*":
        return l * r
    if r == 0.0:
        return 0.0   # the lenient JEXL interpreter: a divide / modulo error is Double 0.0
    if op == "/":
        return l / r
    return math.fmod(l, r)


def combine(op, variables, fills=None):
    """sumSeries & co.: 'a op b op ...' over {var: [series]} with a UNION join; returns the
    EDPtoDPS series of every joined set in ByteMap order."""
    names = list(variables)
    by_key = {}
    for vi, nm in enumerate(names):
        for pts, key in variables[nm]:
            by_key.setdefault(key, [None] * len(names))[vi] = pts
    out = []
    for key in sorted(by_key):
        row = by_key[key]
        cursors = [0] * len(names)
        o = []
        while any(r is not None and cursors[i] < len(r) for i, r in enumerate(row)):   # UnionIterator.hasNext(index)
            ts = (1 << 63) - 1
            vals = []
            for i, r in enumerate(row):
                if r is None:
                    vals.append(0.0)   # fill_dp: a default MutableDataPoint
                    continue
                if cursors[i] >= len(r):
                    raise OracleExprError("RuntimeException", "No more elements")
                t, v = r[cursors[i]]
                cursors[i] += 1
                ts = min(ts, t)
                v = float(v)
                vals.append(v if v == v else (fills or {}).get(names[i], 0.0))
            acc = vals[0]
            for v in vals[1:]:
                acc = _jexl(op, acc, v)
            o.append((ts, acc))
        out.append((o, key))
    return out


def bits(v):
    return v & 0xFFFFFFFFFFFFFFFF if isinstance(v, int) else struct.unpack("<Q", struct.pack("<d", v))[0]


# ---- highestMax / highestCurrent ---------------------------------------------------------
_TIME_MASK = (1 << 63) - 1
_LONG_MIN = -(1 << 63)
_DOUBLE_MIN = 4.9e-324   # Double.MIN_VALUE


def _jdiv(a, b):          # Java long division (truncating; / 0 throws)
    if b == 0:
        raise OracleExprError("ArithmeticException", "/ by zero")
    q = abs(a) // abs(b)
    return _j_long(q if (a >= 0) == (b >= 0) else -q)


def _agg_walk(series, start, end):
    """AggregationIterator(views, start, end, agg, LERP, rate=false) over sorted point lists,
    yielding per emitted point (ts, isInteger, [the operands nextLongValue / nextDoubleValue
    hand the aggregator, in hasNextValue order]).  Slots follow the Java: ts[i] / ts[k + i] with
    0 = no value, TIME_MASK = ended; the float flag lives with the timestamp word, so ending a
    slot or zeroing it clears it."""
    k = len(series)
    ts = [0] * (2 * k)
    val = [0] * (2 * k)
    flt = [False] * (2 * k)
    pos_in = [0] * k          # each view's next index (PostAggregatedDataPoints' iterator)
    live = [True] * k

    def put(i, p):
        ts[i], val[i] = p[0], p[1]
        flt[i] = not isinstance(p[1], int)

    def end_reached(i):
        ts[k + i], flt[k + i] = _TIME_MASK, False
        live[i] = False

    for i, pts in enumerate(series):           # constructor :395-465 (seek to start first)
        j = 0
        while j < len(pts) and pts[j][0] < start:
            j += 1
        if j >= len(pts):
            end_reached(i)
            continue
        put(k + i, pts[j])
        pos_in[i] = j + 1

    def move_to_next(i):                       # :573-588
        ts[i], val[i], flt[i] = ts[k + i], val[k + i], flt[k + i]
        if not live[i]:
            raise OracleExprError("NullPointerException", "iterator already ended")
        if pos_in[i] < len(series[i]):
            put(k + i, series[i][pos_in[i]])
            pos_in[i] += 1
        else:
            end_reached(i)

    current = 0
    while any(ts[k + i] <= end for i in range(k)):   # hasNext :500-512
        for i in range(current, k):                    # next :514-567
            if ts[i + k] == _TIME_MASK:
                ts[i], flt[i] = 0, False
        current, min_ts, multiple = -1, None, False
        for i in range(k):
            t = ts[k + i]
            if t <= end:
                if min_ts is None or t < min_ts:
                    min_ts, current, multiple = t, i, False
                elif t == min_ts:
                    multiple = True
        move_to_next(current)
        if multiple:
            for i in range(current + 1, k):
                if ts[k + i] == min_ts:
                    move_to_next(i)
        is_int = not any(flt)                  # isInteger :612-625
        x = ts[current]
        ops = []
        for p in range(k):                     # hasNextValue order :667-680
            if ts[p] == 0:
                continue
            y0 = val[p]
            if p == current or x == ts[p]:
                ops.append(y0 if is_int else float(y0))
                continue
            x0, x1, y1 = ts[p], ts[p + k], val[p + k]
            if x == x1:
                ops.append(y1 if is_int else float(y1))
                continue
            if is_int:                         # nextLongValue LERP :682-729
                ops.append(_j_long(y0 + _jdiv(_j_long((x - x0) * _j_long(y1 - y0)), x1 - x0)))
            else:                              # nextDoubleValue LERP :735-797
                ops.append(float(y0) + float(x - x0) * (float(y1) - float(y0)) / float(x1 - x0))
        yield x, is_int, ops


def _java_max(a, b):                           # Math.max(double, double)
    if a != a or b != b:
        return math.nan
    if a == 0.0 and b == 0.0:
        return b if math.copysign(1.0, a) < 0 else a
    return a if a > b else b


def _double_compare_key(v):                    # Double.compare order
    if v != v:
        return (2, 0.0)
    if v == 0.0:
        return (1, 0.0) if math.copysign(1.0, v) > 0 else (0, 0.0)
    return (0 if v < 0 else 1, v)


def topn_parse(params):
    """The top-n parameter checks of HighestMax / HighestCurrent.evaluate (:44-72)."""
    if not params:
        raise OracleExprError("IllegalArgumentException", "Need aggregation window for moving average")
    p = params[0]
    if p is None or p == "":
        raise OracleExprError("IllegalArgumentException", "Missing top n value")
    if not p.isdigit() or not p.isascii():
        raise OracleExprError("IllegalArgumentException", "Unparseable top n value: " + p)
    n = int(p)
    if n > (1 << 31) - 1:
        raise OracleExprError("IllegalArgumentException", "Invalid parameter, must be an integer")
    if n < 1:
        raise OracleExprError("IllegalArgumentException", "Top n value must be greater than zero")
    return n


def highest(series, topn, start, end, current=False):
    """Indices (into `series`, a flat list of point lists over every sub-query's group-bys) of
    the series highestMax (current=False) or highestCurrent (current=True) returns, in order."""
    idx = list(range(len(series)))
    if current:                               # HighestCurrent drops empty series (:94-97)
        idx = [i for i in idx if len(series[i]) > 0]
    views = [series[i] for i in idx]
    n = len(views)
    max_l = [_LONG_MIN] * n
    max_d = [_DOUBLE_MIN] * n
    has_l = has_d = False
    for ts, is_int, ops in _agg_walk(views, start, end):
        if ts < start or ts > end:
            continue
        arr = list(ops) + [0 if is_int else 0.0] * (n - len(ops))
        if is_int:
            max_l = arr if current else [max(a, b) for a, b in zip(max_l, arr)]
            has_l = True
        else:
            max_d = arr if current else [_java_max(a, b) for a, b in zip(max_d, arr)]
            has_d = True
    if has_l and has_d:
        vals = [_java_max(float(a), b) for a, b in zip(max_l, max_d)]
    elif has_l:
        vals = [float(a) for a in max_l]
    elif has_d:
        vals = list(max_d)
    else:
        vals = None
    count = min(topn, n)
    if vals is None:
        if n > 0:
            raise OracleExprError("NullPointerException", "no datapoint in the query range")
        return []
    order = sorted(range(n), key=lambda i: _double_compare_key(vals[i]), reverse=True)
    # sorted(..., reverse=True) keeps equal keys in their original order (stable), as the
    # reference's Arrays.sort with a negated Double.compare does
    return [idx[i] for i in order[:count]]
