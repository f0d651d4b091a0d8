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


def encode_rows(ts_ms, lvals, fvals, kind, ms):
    """Compacted hour rows of one series, as TSDB.addPoint + CompactionQueue write them.

    Per point: ts_ms (sorted, distinct), kind 0 = long (vle 1/2/4/8 B), 1 = float32 (4 B),
    2 = float64 (8 B); ms = millisecond qualifier (4 B, src/core/Internal.java:848-856) or
    second qualifier (2 B).  A row mixing both carries meta byte MS_MIXED_COMPACT (0x01,
    src/core/Const.java:83; CompactionQueue.java:594-612).  Returns [(base_s, qual, val)]."""
    ts_ms = np.asarray(ts_ms, np.int64)
    bases = (ts_ms // 1000) - (ts_ms // 1000) % 3600
    rows = []
    a = 0
    n = len(ts_ms)
    while a < n:
        b = a
        while b < n and bases[b] == bases[a]:
            b += 1
        base = int(bases[a])
        q, v = [], []
        any_ms = any_s = False
        for j in range(a, b):
            off = int(ts_ms[j]) - base * 1000
            if kind[j] == 0:
                x = int(lvals[j])
                L = 1 if -128 <= x <= 127 else 2 if -32768 <= x <= 32767 else 4 if -(1 << 31) <= x < (1 << 31) else 8
                flags = L - 1
                vb = x.to_bytes(L, "big", signed=True)
            elif kind[j] == 1:
                flags = 0xB
                vb = np.array([fvals[j]], ">f4").tobytes()   # (numpy scalars are always native-endian)
            else:
                flags = 0xF
                vb = np.array([fvals[j]], ">f8").tobytes()
            if ms[j]:
                any_ms = True
                q.append((0xF0000000 | (off << 6) | flags).to_bytes(4, "big"))
            else:
                any_s = True
                assert off % 1000 == 0
                q.append((((off // 1000) << 4) | flags).to_bytes(2, "big"))
            v.append(vb)
        val = b"".join(v)
        if b - a > 1:
            val += b"\x01" if (any_ms and any_s) else b"\x00"
        rows.append((base, b"".join(q), val))
        a = b
    return rows


def from_series(series_rows, group_ids) -> abi.HostBatch:
    """HostBatch from per-series row lists (encode_rows output) and group ids."""
    quals, vals, row_base = [], [], []
    row_ptr = [0]
    for rows in series_rows:
        for base, q, v in rows:
            row_base.append(base)
            quals.append(q)
            vals.append(v)
        row_ptr.append(len(row_base))
    qo = np.zeros(len(quals) + 1, np.uint64)
    vo = np.zeros(len(vals) + 1, np.uint64)
    qo[1:] = np.cumsum([len(x) for x in quals])
    vo[1:] = np.cumsum([len(x) for x in vals])
    qb = np.frombuffer(b"".join(quals), np.uint8) if quals else np.zeros(0, np.uint8)
    vb = np.frombuffer(b"".join(vals), np.uint8) if vals else np.zeros(0, np.uint8)
    return abi.HostBatch(np.array(row_ptr, np.int64), np.array(row_base, np.uint32), qo, vo, qb, vb,
                         np.asarray(group_ids, np.int32))


def _h(seed: int, i: np.ndarray, k: np.ndarray, salt: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        return splitmix64(np.uint64(seed ^ salt) ^ (i.astype(np.uint64) << np.uint64(32)) ^ k.astype(np.uint64))


def generate_counters(n_series: int, start_s: int, n_points: int, period_ms: int = 10000,
                      jitter_ms: int = 4000, n_groups: int = 64, reset_p: float = 1.0 / 500,
                      seed: int = 0x5EED) -> abi.HostBatch:
    """BASELINE config 4 shape, vectorised: jittered millisecond timestamps (nominal period,
    uniform integer jitter in [-jitter, +jitter]), monotone counters (start [0, 1e9),
    increments [0, 1000)) that reset to [0, 100) with probability ~reset_p per point.  Every
    draw is a splitmix64 hash of (seed, global series id i, point k).  Series i belongs to
    group i % n_groups; the batch is group-major.  Cells are what TSDB.addPoint(long) with
    millisecond timestamps + compaction write: 4-byte ms qualifiers, vle values, meta 0x00."""
    assert period_ms > 2 * jitter_ms, "jitter must keep timestamps strictly increasing"
    order, grp = series_order(n_series, n_groups)
    S, P = len(order), n_points
    I = np.repeat(order, P).reshape(S, P)
    K = np.tile(np.arange(P, dtype=np.int64), S).reshape(S, P)
    jit = (_h(seed, I, K, 0x11) % np.uint64(2 * jitter_ms + 1)).astype(np.int64) - jitter_ms
    ts = start_s * 1000 + K * period_ms + jit
    inc = (_h(seed, I, K, 0x22) % np.uint64(1000)).astype(np.int64)
    reset = (_h(seed, I, K, 0x33).astype(np.float64) / 18446744073709551616.0) < reset_p
    rval = (_h(seed, I, K, 0x44) % np.uint64(100)).astype(np.int64)
    start = (_h(seed, I[:, :1], K[:, :1], 0x55) % np.uint64(1_000_000_000)).astype(np.int64)
    # value[k] = value at the last reset (or the start) + increments since
    step = np.where(reset, 0, inc)
    step[:, 0] = np.where(reset[:, 0], 0, inc[:, 0])
    anchor = np.where(reset, rval, 0)
    anchor[:, 0] = np.where(reset[:, 0], rval[:, 0], start[:, 0] + inc[:, 0])
    step[:, 0] = 0
    cs = np.cumsum(step, axis=1)
    seg = np.maximum.accumulate(np.where(reset | (K == 0), K, 0), axis=1)
    base_v = np.take_along_axis(anchor, seg, axis=1)
    v = base_v + cs - np.take_along_axis(cs, seg, axis=1)
    # vle lengths and the flat byte layout (rows split at hour boundaries)
    L = vle_lengths(v)
    bases = (ts // 1000) - (ts // 1000) % 3600
    newrow = np.ones((S, P), bool)
    newrow[:, 1:] = bases[:, 1:] != bases[:, :-1]
    flat_new = newrow.ravel()
    row_id = np.cumsum(flat_new) - 1
    n_rows = int(row_id[-1]) + 1
    row_start = np.flatnonzero(flat_new)
    row_n = np.diff(np.concatenate([row_start, [S * P]]))
    row_base = bases.ravel()[row_start].astype(np.uint32)
    series_of_row = row_start // P
    row_ptr = np.searchsorted(series_of_row, np.arange(S + 1), side="left").astype(np.int64)
    # qualifiers: 4 B each
    off = ts.ravel() - bases.ravel() * 1000
    q = (np.uint32(0xF0000000) | (off.astype(np.uint32) << np.uint32(6)) | (L.ravel() - 1).astype(np.uint32))
    qual = q.astype(">u4").view(np.uint8)
    qo = np.zeros(n_rows + 1, np.uint64)
    qo[1:] = np.cumsum(row_n * 4)
    # values: vle bytes + one meta byte per multi-point row
    Lf = L.ravel()
    row_vbytes = np.add.reduceat(Lf, row_start) + (row_n > 1)
    vo = np.zeros(n_rows + 1, np.uint64)
    vo[1:] = np.cumsum(row_vbytes)
    # byte position of each point's value
    excl = np.cumsum(Lf) - Lf
    row_excl0 = excl[row_start]
    pos = vo[row_id].astype(np.int64) + (excl - row_excl0[row_id])
    val = np.zeros(int(vo[-1]), np.uint8)
    vf = v.ravel()
    for nb in (1, 2, 4, 8):
        sel = np.flatnonzero(Lf == nb)
        if not len(sel):
            continue
        be = vf[sel].astype(">i8").view(np.uint8).reshape(-1, 8)[:, 8 - nb:]
        idx = pos[sel][:, None] + np.arange(nb)[None, :]
        val[idx.ravel()] = be.ravel()
    return abi.HostBatch(row_ptr, row_base, qo, vo, qual, val, grp)
