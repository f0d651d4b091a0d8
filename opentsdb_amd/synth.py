"""Host-side synthetic store generator (numpy), byte-identical to tsdbhip_synth.

The BASELINE configs use seeded synthetic series loaded the way MockBase loads them:
every point goes through TSDB.addPoint (src/core/TSDB.java:1012-1110) and every hour
row through CompactionQueue (src/core/CompactionQueue.java:594-612).  Values are pure
functions of (seed, global series id i, point index k) via splitmix64:
  value_kind 0: float32 50 + 10 (u - 0.5)            (addPoint(float), 4 bytes)
  value_kind 1: int  u mod int_mod                    (addPoint(long), 1/2/4/8 bytes)
  value_kind 2: even series int, odd series float32
  value_kind 3: float64 holding the kind-0 float32 value (8-byte float cells; host only)
  value_kind 4: float64 50 + 10 (u - 0.5) with a full 53-bit mantissa (host only)
Series i belongs to group i % n_groups; the batch lists series grouped (group-major).
"""
from __future__ import annotations

import numpy as np

from . import abi

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def series_order(n_series: int, n_groups: int):
    """Batch position -> (global series id, group)."""
    gids, grp = [], []
    for g in range(n_groups):
        ids = np.arange(g, n_series, n_groups, dtype=np.int64)
        gids.append(ids)
        grp.append(np.full(len(ids), g, np.int32))
    return np.concatenate(gids), np.concatenate(grp)


def values(seed: int, i: int, k: np.ndarray, value_kind: int, int_mod: int):
    u = splitmix64(np.uint64(seed) ^ (np.uint64(i) << np.uint64(32)) ^ k.astype(np.uint64))
    is_int = value_kind == 1 or (value_kind == 2 and i % 2 == 0)
    if is_int:
        return True, (u % np.uint64(int_mod)).astype(np.int64)
    d = (u >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    if value_kind == 4:
        return False, 50.0 + 10.0 * (d - 0.5)
    if value_kind == 3:
        return False, (50.0 + 10.0 * (d - 0.5)).astype(np.float32).astype(np.float64)
    return False, (50.0 + 10.0 * (d - 0.5)).astype(np.float32)


def vle_lengths(v: np.ndarray) -> np.ndarray:
    L = np.full(v.shape, 8, np.int64)
    L[(v >= -(1 << 31)) & (v <= (1 << 31) - 1)] = 4
    L[(v >= -32768) & (v <= 32767)] = 2
    L[(v >= -128) & (v <= 127)] = 1
    return L


def generate(n_series: int, start_s: int, n_points: int, period_ms: int, value_kind: int = 0,
             n_groups: int = 1, int_mod: int = 2000, seed: int = 0x5EED) -> abi.HostBatch:
    start_ms = start_s * 1000
    ms_qual = (period_ms % 1000) != 0
    ks = np.arange(n_points, dtype=np.int64)
    ts = start_ms + ks * period_ms
    bases = (ts // 1000) - (ts // 1000) % 3600
    # hour rows (identical for every series)
    cut = np.flatnonzero(np.diff(bases)) + 1
    row_k0 = np.concatenate([[0], cut])
    row_k1 = np.concatenate([cut, [n_points]])
    order, grp = series_order(n_series, n_groups)
    quals, vals, row_base = [], [], []
    row_ptr = [0]
    # qualifiers do not depend on values: build once per row
    for i in order:
        is_int, v = values(seed, int(i), ks, value_kind, int_mod)
        for a, b in zip(row_k0, row_k1):
            base = int(bases[a])
            off = ts[a:b] - base * 1000
            n = b - a
            if is_int:
                L = vle_lengths(v[a:b])
                flags = (L - 1).astype(np.uint32)
            elif v.dtype == np.float64:
                L = np.full(n, 8, np.int64)
                flags = np.full(n, 0xF, np.uint32)
            else:
                L = np.full(n, 4, np.int64)
                flags = np.full(n, 0xB, np.uint32)
            if ms_qual:
                q = (np.uint32(0xF0000000) | (off.astype(np.uint32) << np.uint32(6)) | flags).astype(">u4").tobytes()
            else:
                q = (((off // 1000).astype(np.uint32) << np.uint32(4)) | flags).astype(">u2").tobytes()
            if is_int:
                parts = []
                vv = v[a:b]
                for x, l in zip(vv.tolist(), L.tolist()):
                    parts.append(int(x).to_bytes(l, "big", signed=True))
                vb = b"".join(parts)
            elif v.dtype == np.float64:
                vb = v[a:b].astype(">f8").tobytes()
            else:
                vb = v[a:b].astype(">f4").tobytes()
            if n > 1:
                vb += b"\x00"
            quals.append(q)
            vals.append(vb)
            row_base.append(base)
        row_ptr.append(len(row_base))
    qo = np.zeros(len(quals) + 1, np.uint64)
    vo = np.zeros(len(vals) + 1, np.uint64)
    qo[1:] = np.cumsum([len(x) for x in quals])
    vo[1:] = np.cumsum([len(x) for x in vals])
    return abi.HostBatch(np.array(row_ptr, np.int64), np.array(row_base, np.uint32), qo, vo,
                         np.frombuffer(b"".join(quals), np.uint8), np.frombuffer(b"".join(vals), np.uint8), grp)
