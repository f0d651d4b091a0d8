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
                             Doubles (third_party/jexl/include.mk:1, not vendored: +, -, *, and /, %
                             throwing ArithmeticException for a zero divisor)
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
        raise OracleExprError("RuntimeException", "ArithmeticException /")
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
