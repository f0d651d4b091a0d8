"""The arithmetic of k_raw_eval's strip-wide long LERP (lerpw_init / lerpw_eval in
opentsdb_amd/csrc/k_raw_eval.hip) restated with Python floats (IEEE doubles) and checked against
Java's long LERP y0 + (x - x0) * (y1 - y0) / (x1 - x0) with truncating division
(src/core/AggregationIterator.java:682-729) -- the bound it relies on (the reciprocal quotient
is off by at most one while |dy| (x1 - x0) < 2^51) and the mantissa conversion of the quotient.
The kernel itself is checked against the oracle by the raw-path GPU tests."""
from __future__ import annotations

import math
import struct

import numpy as np


def java_lerp(x, x0, y0, x1, y1):
    num = (x - x0) * (y1 - y0)
    q = abs(num) // (x1 - x0)
    return y0 + (q if num >= 0 else -q)


def lerpw(x, x0, y0, x1, y1):
    den, dy = x1 - x0, y1 - y0
    ok = 0 < den < 2 ** 32 and abs(dy) < 2 ** 51 and float(abs(dy)) * float(den) < 2.0 ** 50
    if not ok:
        return None
    dyd, dend = float(dy), float(den)
    rd = 1.0 / dend
    nd = float(x - x0) * dyd
    assert nd == (x - x0) * dy                 # the product is exact
    q = math.trunc(nd * rd) * 1.0
    r = int(nd) - int(q) * den                 # the FMA's exact remainder
    if dy >= 0:
        q += (1.0 if r >= den else 0.0) - (1.0 if r < 0 else 0.0)
    else:
        q += (1.0 if r > 0 else 0.0) - (1.0 if r <= -den else 0.0)
    bits = struct.unpack("<q", struct.pack("<d", q + 6755399441055744.0))[0]
    return y0 + (bits - 0x4338000000000000)


def test_lerp_window_matches_java_long_lerp():
    rng = np.random.default_rng(5)
    checked = 0
    for scale_x, scale_y in [(10, 10), (3600000, 1000), (2 ** 31, 2 ** 18), (2 ** 20, 2 ** 30), (7, 2 ** 47)]:
        for _ in range(4000):
            den = int(rng.integers(1, scale_x + 2))
            x0 = int(rng.integers(0, 2 ** 40))
            y0 = int(rng.integers(-2 ** 50, 2 ** 50))
            dy = int(rng.integers(-scale_y, scale_y + 1))
            x = x0 + int(rng.integers(1, den)) if den > 1 else x0
            got = lerpw(x, x0, y0, x0 + den, y0 + dy)
            if got is None:
                continue
            assert got == java_lerp(x, x0, y0, x0 + den, y0 + dy), (x, x0, y0, den, dy)
            checked += 1
    # near the bound: quotients close to 2^50 and exact multiples
    for den, dy in [(2 ** 32 - 1, 262143), (3, 2 ** 48 + 1), (1000, -(2 ** 40) - 7), (999983, 1125899)]:
        for dx in [1, den // 2, den - 1]:
            got = lerpw(dx, 0, -5, den, dy - 5)
            if got is not None:
                assert got == java_lerp(dx, 0, -5, den, dy - 5)
                checked += 1
    assert checked > 15000
