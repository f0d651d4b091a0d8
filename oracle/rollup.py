"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the rollup codec and of rollup
generation.  Only tests/ may import this module.

Pinned by tests/golden/rollup.json (extracted from test/rollup/TestRollupInterval.java
and test/rollup/TestRollupUtils.java).  The calendar arithmetic uses Python's datetime
(proleptic Gregorian UTC), independent of the engine's civil-date code.
"""
from __future__ import annotations

import datetime as _dt
import struct

import numpy as np

from . import oracle

INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1
SECOND_MASK = 0xFFFFFFFF00000000


class RollupError(ValueError):
    """IllegalArgumentException."""


def jint(x: int) -> int:
    """Java (int) of a long: two's-complement wrap to 32 bits."""
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


def jdiv(a: int, b: int) -> int:
    """Java int / (truncating)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


class Interval:
    """RollupInterval ctor + validateAndCompile (src/rollup/RollupInterval.java:62-103,169-235)."""

    def __init__(self, interval: str, row_span: str):
        if not row_span:
            raise RollupError("Duration cannot be null or empty")
        u = 0
        while u < len(row_span) and row_span[u].isdigit():   # DateTime.getDurationUnits (:237-254)
            u += 1
        units = row_span[u:].lower()
        if units not in ("ms", "s", "m", "h", "d", "w", "n", "y"):
            raise RollupError("Invalid units in the duration: " + units)
        if len(units) > 1:
            raise RollupError("Milliseconds are not supported")
        if "." in row_span:                                   # DateTime.getDurationInterval (:265-284)
            raise RollupError("Floating point intervals are not supported")
        try:
            mult = int(row_span[:u])
        except ValueError:
            raise RollupError("Invalid duration (number): " + row_span)
        if mult > INT_MAX:
            raise RollupError("Invalid duration (number): " + row_span)
        if mult <= 0:
            raise RollupError("Zero or negative duration: " + row_span)
        self.units = units
        self.unit_multiplier = mult
        if units != "h" and mult > 1:
            raise RollupError("Multipliers are only usable with the 'h' unit")
        if units == "h" and mult > 1 and mult % 2 != 0:
            raise RollupError("The multiplier must be 1 or an even value")
        try:
            ms = oracle.parse_duration(interval)
        except Exception as e:
            raise RollupError(str(e))
        iv = jint(ms // 1000)
        if iv < 1:
            raise RollupError("Millisecond intervals are not supported")
        if iv >= INT_MAX:
            raise RollupError("Interval is too big")
        self.interval_units = interval[-1]
        spans = {"h": 3600, "d": 86400, "n": 86400 * 32, "y": 86400 * 366}
        if units not in spans:
            raise RollupError("Unrecogznied span")
        num_span = jint(spans[units] * mult)
        if iv >= num_span:
            raise RollupError("Interval is too large for the span")
        self.intervals = jdiv(num_span, iv)
        if self.intervals > 7774:
            raise RollupError("Too many intervals")
        if self.intervals < 12:
            raise RollupError("Not enough intervals")
        self.interval_s = iv


def basetime(ts: int, iv: Interval) -> int:
    """RollupUtils.getRollupBasetime (src/rollup/RollupUtils.java:52-112)."""
    if ts < 0:
        raise RollupError("Not supporting negative timestamps")
    if iv.units == "h":
        modulo = iv.unit_multiplier * 3600 if iv.unit_multiplier > 1 else 3600
        if ts & SECOND_MASK:
            s = ts // 1000
            return jint(s - s % modulo)
        return jint(ts - ts % modulo)
    ms = ts if ts & SECOND_MASK else ts * 1000
    t = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc) + _dt.timedelta(milliseconds=ms)
    t = t.replace(hour=0, minute=0, second=0)
    if iv.units == "d":
        pass
    elif iv.units == "n":
        t = t.replace(day=1)
    elif iv.units == "y":
        t = t.replace(day=1, month=1)
    else:
        raise RollupError("Unrecogznied span")
    epoch_ms = (t - _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)) // _dt.timedelta(milliseconds=1)
    return jint(epoch_ms // 1000)


def qualifier(ts: int, base: int, flags: int, agg_id: int, iv: Interval) -> bytes:
    """RollupUtils.buildRollupQualifier (src/rollup/RollupUtils.java:143-171)."""
    tsec = jint(ts // 1000 if ts & SECOND_MASK else ts)
    off = jdiv(jint(tsec - base), iv.interval_s)
    if off >= iv.intervals:
        raise RollupError("Offset greater than the configured intervals")
    off = jint(off << 4) | flags
    return bytes([agg_id & 0xFF]) + struct.pack(">H", off & 0xFFFF)


def vle_encode(v: int) -> bytes:
    """Internal.vleEncodeLong (src/core/Internal.java:963-973)."""
    if -128 <= v <= 127:
        return struct.pack(">b", v)
    if -32768 <= v <= 32767:
        return struct.pack(">h", v)
    if INT_MIN <= v <= INT_MAX:
        return struct.pack(">i", v)
    return struct.pack(">q", v)


def java_long(v: float) -> int:
    if v != v:
        return 0
    if v >= 9.223372036854775807e18:
        return (1 << 63) - 1
    if v <= -9.223372036854775808e18:
        return -(1 << 63)
    return int(v)


def encode_value(v: float, as_long: bool):
    """(flags, bytes) as TSDB.addAggregatePoint(long / float / double) stores them
    (src/core/TSDB.java:1322-1438); NaN / Inf are rejected."""
    if as_long:
        b = vle_encode(java_long(v))
        return len(b) - 1, b
    if v != v or v in (float("inf"), float("-inf")):
        raise RollupError("value is NaN or Infinite")
    with np.errstate(over="ignore"):
        f = float(np.float32(v))
    if f == v:   # Tags.fitsInFloat (src/core/Tags.java:853-858)
        return 0x8 | 0x3, struct.pack(">f", v)
    return 0x8 | 0x7, struct.pack(">d", v)


def _series_rows(batch, s):
    r0, r1 = int(batch.series_row_ptr[s]), int(batch.series_row_ptr[s + 1])
    bts, qs, vs = [], [], []
    for r in range(r0, r1):
        bts.append(int(batch.row_base_time[r]))
        qs.append(bytes(batch.qual[int(batch.row_qual_off[r]):int(batch.row_qual_off[r + 1])]))
        vs.append(bytes(batch.val[int(batch.row_val_off[r]):int(batch.row_val_off[r + 1])]))
    return bts, qs, vs


def generate(batch, iv: Interval, start_s: int, end_s: int, funcs=(("sum", 0), ("count", 1), ("max", 2), ("min", 3))):
    """Reference-side rollup generation: per series (batch order) and function, the
    Downsampler (fixed interval = the rollup interval) of the Span, each bucket starting in
    [start_s, end_s) written as addAggregatePoint would store it.  Returns a list of
    (series, base_time, qualifier bytes, value bytes) in (function, series, time) order.
    Series with group_id < 0 are not part of the batch (tsdbhip_load drops them)."""
    out = []
    ns = len(batch.series_row_ptr) - 1
    for fn, aid in funcs:
        for s in range(ns):
            if int(batch.group_id[s]) < 0:
                continue
            bts, qs, vs = _series_rows(batch, s)
            raw = oracle.span_view(bts, qs, vs).drain() if bts else []
            all_int = all(p[1] for p in raw)
            if not bts:
                continue
            view = oracle.downsampler_raw(oracle.span_view(bts, qs, vs), fn, iv.interval_s * 1000)
            for ts, _isi, v in view.drain():
                if not (start_s * 1000 <= ts < end_s * 1000):
                    continue
                flags, vb = encode_value(float(v), fn == "count" or all_int)
                b = basetime(ts // 1000, iv)
                out.append((s, b, qualifier(ts // 1000, b, flags, aid, iv), vb))
    return out
