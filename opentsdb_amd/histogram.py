"""Histogram path: host-side mirror of the reference's histogram API.

- ``HistBatch`` / ``HistResult``: ctypes mirrors of ``tsdbhip_hist_batch`` / ``tsdbhip_hist_result``
  (include/tsdbhip.h); ``HostHistBatch`` owns the arrays.
- ``SimpleHistogram``: the reference's bucketed histogram as a value object with its storage
  encoding (src/core/SimpleHistogram.java:61-122; Kryo 2.21 ``Output``: big-endian short / float,
  ``writeLong(v, true)`` varints) and ``initializeHistogram`` (:305-365) -- what a writer
  (``TSDB.addHistogramPoint``, src/core/TSDB.java:1132-1148) stores.
- ``histogram_qualifier``: ``Internal.getQualifier(timestamp, HistogramDataPoint.PREFIX)``.
- ``HistogramDataPoints``: one result series -- a percentile series
  (HistogramDataPointsToDataPointsAdaptor) or a bucket series (HistogramBucketDataPointsAdaptor),
  with the reference's metric-name suffixes.  ``result_to_series`` builds them from an engine result;
  the bucket series follow the adaptor's ``TreeMap`` lookups (see ``bucket_value``).

The arithmetic runs in libtsdbhip (k_hist.hip); nothing here computes histogram values.
"""
from __future__ import annotations

import ctypes as C
import math
import struct

import numpy as np

HCODEC_NONE, HCODEC_SIMPLE, HCODEC_LONG = 0, 1, 2   # tsdbhip.h TSDB_HCODEC_*
PREFIX = 0x06                                         # HistogramDataPoint.PREFIX
BK_UNDER, BK_REG, BK_OVER = 0, 1, 2                   # HistogramBucket.BucketType


class HistBatch(C.Structure):
    _fields_ = [
        ("n_series", C.c_int64),
        ("series_row_ptr", C.POINTER(C.c_int64)),
        ("n_rows", C.c_int64),
        ("row_base_time", C.POINTER(C.c_uint32)),
        ("row_cell_ptr", C.POINTER(C.c_int64)),
        ("n_cells", C.c_int64),
        ("cell_qual_off", C.POINTER(C.c_uint64)),
        ("cell_val_off", C.POINTER(C.c_uint64)),
        ("qual", C.POINTER(C.c_uint8)),
        ("val", C.POINTER(C.c_uint8)),
        ("group_id", C.POINTER(C.c_int32)),
        ("codec", C.c_uint8 * 256),
    ]


class HistResult(C.Structure):
    _fields_ = [
        ("n_groups", C.c_int64),
        ("group_id", C.POINTER(C.c_int32)),
        ("group_ptr", C.POINTER(C.c_int64)),
        ("ts_ms", C.POINTER(C.c_int64)),
        ("n_pct", C.c_int32),
        ("pct", C.POINTER(C.c_double)),
        ("show_buckets", C.c_int32),
        ("n_buckets", C.c_int32),
        ("bucket_lower", C.POINTER(C.c_uint32)),
        ("bucket_upper", C.POINTER(C.c_uint32)),
        ("count", C.POINTER(C.c_int64)),
        ("present", C.POINTER(C.c_uint8)),
        ("codec", C.POINTER(C.c_uint8)),
    ]


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class HostHistBatch:
    """Owns the arrays behind a :class:`HistBatch`."""

    def __init__(self, series_row_ptr, row_base_time, row_cell_ptr, cell_qual_off, cell_val_off, qual, val, group_id,
                 codecs):
        self.series_row_ptr = np.ascontiguousarray(series_row_ptr, dtype=np.int64)
        self.row_base_time = np.ascontiguousarray(row_base_time, dtype=np.uint32)
        self.row_cell_ptr = np.ascontiguousarray(row_cell_ptr, dtype=np.int64)
        self.cell_qual_off = np.ascontiguousarray(cell_qual_off, dtype=np.uint64)
        self.cell_val_off = np.ascontiguousarray(cell_val_off, dtype=np.uint64)
        self.qual = np.ascontiguousarray(qual, dtype=np.uint8)
        self.val = np.ascontiguousarray(val, dtype=np.uint8)
        self.group_id = np.ascontiguousarray(group_id, dtype=np.int32)
        if self.qual.size == 0:
            self.qual = np.zeros(1, np.uint8)
        if self.val.size == 0:
            self.val = np.zeros(1, np.uint8)
        if self.row_base_time.size == 0:
            self.row_base_time = np.zeros(1, np.uint32)
        ns = len(self.series_row_ptr) - 1
        nr = len(self.row_cell_ptr) - 1
        nc = len(self.cell_qual_off) - 1
        assert len(self.group_id) == ns and len(self.cell_val_off) == nc + 1
        cod = (C.c_uint8 * 256)()
        for cid, kind in dict(codecs).items():
            cod[int(cid)] = int(kind)
        self.codecs = dict(codecs)
        self.c = HistBatch(ns, _ptr(self.series_row_ptr, C.c_int64), nr, _ptr(self.row_base_time, C.c_uint32),
                           _ptr(self.row_cell_ptr, C.c_int64), nc, _ptr(self.cell_qual_off, C.c_uint64),
                           _ptr(self.cell_val_off, C.c_uint64), _ptr(self.qual, C.c_uint8), _ptr(self.val, C.c_uint8),
                           _ptr(self.group_id, C.c_int32), cod)

    @classmethod
    def from_rows(cls, series, group_ids, codecs):
        """series: [[(base_time, [(qualifier bytes, value bytes), ...]), ...], ...] in scan order;
        codecs: {codec id: HCODEC_*} (tsd.core.histograms.config)."""
        srp, bases, rcp, qo, vo = [0], [], [0], [0], [0]
        qb, vb = bytearray(), bytearray()
        for rows in series:
            for base, cols in rows:
                bases.append(base)
                for q, v in cols:
                    qb += q
                    vb += v
                    qo.append(len(qb))
                    vo.append(len(vb))
                rcp.append(len(qo) - 1)
            srp.append(len(bases))
        return cls(srp, bases, rcp, qo, vo, np.frombuffer(bytes(qb), np.uint8), np.frombuffer(bytes(vb), np.uint8),
                   group_ids, codecs)


# ---- storage encoding ----------------------------------------------------------------------
def kryo_varlong(v: int) -> bytes:
    """Kryo 2.21 Output.writeLong(v, true): 7-bit groups little end first, the 9th byte 8 bits."""
    u = v & 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    for _ in range(8):
        if u >> 7 == 0:
            out.append(u)
            return bytes(out)
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u & 0xFF)
    return bytes(out)


def f32bits(x: float) -> int:
    return struct.unpack(">I", struct.pack(">f", x))[0]


def bits_f32(b: int) -> float:
    return struct.unpack(">f", struct.pack(">I", b & 0xFFFFFFFF))[0]


def _fcmp_key(bits: int):
    """Float.compare order of float bits (canonical NaN greatest, -0.0 < 0.0)."""
    b = bits & 0xFFFFFFFF
    if (b & 0x7F800000) == 0x7F800000 and (b & 0x7FFFFF):
        b = 0x7FC00000
    return (~b & 0xFFFFFFFF) if b & 0x80000000 else (b | 0x80000000)


class SimpleHistogram:
    """src/core/SimpleHistogram.java: REGULAR buckets (lower, upper float bits) -> count."""

    def __init__(self, codec_id: int = 0):
        self.id = codec_id
        self.buckets: dict[tuple[int, int], int] = {}
        self.underflow = 0
        self.overflow = 0

    def addBucket(self, lo: float, up: float, count: int):
        lb, ub = f32bits(lo), f32bits(up)
        key = next((k for k in self.buckets if _fcmp_key(k[0]) == _fcmp_key(lb) and _fcmp_key(k[1]) == _fcmp_key(ub)),
                   (lb, ub))
        self.buckets[key] = count
        return self

    def histogram(self, include_id: bool = True) -> bytes:
        """SimpleHistogram.histogram(include_id) (:72-95): the bytes TSDB.addHistogramPoint stores."""
        out = bytearray()
        if include_id:
            out.append(self.id & 0xFF)
        out += struct.pack(">h", len(self.buckets))
        for k in sorted(self.buckets, key=lambda k: (_fcmp_key(k[0]), _fcmp_key(k[1]))):
            out += struct.pack(">II", k[0], k[1]) + kryo_varlong(self.buckets[k])
        out += kryo_varlong(self.underflow) + kryo_varlong(self.overflow)
        return bytes(out)

    @staticmethod
    def initializeHistogram(start: float, end: float, focus_start: float, focus_end: float, error_pct: float):
        """SimpleHistogram.initializeHistogram (:305-365): bucket lower bounds (float arithmetic)."""
        f = np.float32
        start, end, fs, fe, err = f(start), f(end), f(focus_start), f(focus_end), f(error_pct)
        if not start < end:
            raise ValueError("Histogram start must be less than Histogram end")
        if not fs < fe:
            raise ValueError("Histogram focus range start must be less than Histogram focus end")
        if start > fs or fs >= end or start >= fe or fe > end:
            raise ValueError("Focus range must lie inside the histogram range")
        if not err > 0:
            raise ValueError("Error rate must be greater than zero")
        step = f((f(1) + err) / (f(1) - err))
        count = int(math.ceil(math.log(float(f(fe / fs))) / math.log(float(step)))) + 1
        count += int(start < fs) + int(fe < end)
        if count > 100:
            raise ValueError(f"A max of 100 buckets are supported. {count} were requested")
        out = [0.0] * count
        j = 0
        if start < fs:
            out[j] = float(start)
            j += 1
        i = fs
        while i < fe:
            out[j] = float(i)
            i = f(i * step)
            j += 1
        if fe < end:
            out[j] = float(fe)
            j += 1
        out[j] = float(end)
        return out


def long_histogram(codec_id: int, value: int) -> bytes:
    """test/core/LongHistogramDataPointForTest.histogram(true): [id][BE64 value]."""
    return bytes([codec_id & 0xFF]) + struct.pack(">q", value)


def histogram_qualifier(timestamp: int) -> tuple[int, bytes]:
    """Internal.getQualifier(timestamp, 0x06) with the row base time (TSDB.storeIntoDB):
    (base_time, qualifier) -- 3 bytes of second offset or 5 bytes of millisecond offset."""
    if timestamp & 0xFFFFFFFF00000000:
        base = (timestamp // 1000) - (timestamp // 1000) % 3600
        return base, bytes([PREFIX]) + struct.pack(">I", timestamp - base * 1000)
    base = timestamp - timestamp % 3600
    return base, bytes([PREFIX]) + struct.pack(">H", timestamp - base)


# ---- results -------------------------------------------------------------------------------
def java_float_str(x: float) -> str:
    """Float.toString for the metric-name suffixes (shortest repr of the float32)."""
    f = np.float32(x)
    if math.isnan(f):
        return "NaN"
    if math.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if math.copysign(1.0, float(f)) < 0 else "0.0"
    a = abs(float(f))
    r = np.format_float_scientific(f, unique=True, trim="0") if (a < 1e-3 or a >= 1e7) else \
        np.format_float_positional(f, unique=True, trim="0")
    if "e" in r:
        m, e = r.split("e")
        if "." not in m:
            m += ".0"
        return f"{m}E{int(e)}"
    return r if "." in r and not r.endswith(".") else r.rstrip(".") + ".0"


class HistogramDataPoints:
    """One DataPoints of a histogram query: a percentile or a bucket series of a group."""

    def __init__(self, group_id, ts, values, is_int, percentile=None, bucket=None):
        self.group_id = group_id
        self.ts = ts
        self.values = values
        self.is_int = is_int
        self.percentile = percentile   # float, isPercentile()
        self.bucket = bucket           # (type, lower bits, upper bits)

    def isPercentile(self) -> bool:
        return self.percentile is not None

    def size(self) -> int:
        return len(self.ts)

    def metricNameSuffix(self) -> str:
        if self.percentile is not None:
            return "_pct_" + java_float_str(self.percentile)
        t, lo, up = self.bucket
        if t == BK_UNDER:
            return "_UNDERFLOW"
        if t == BK_OVER:
            return "_OVERFLOW"
        return "_" + java_float_str(bits_f32(lo)) + "_" + java_float_str(bits_f32(up))


def bucket_value(key, reg_keys_sorted, counts, under, over) -> int:
    """HistogramBucketDataPointsAdaptor's value of bucket `key` in one point: the point's
    getHistogramBucketsIfHas TreeMap (its REGULAR buckets, then UNDERFLOW, then OVERFLOW) and
    containsKey / get under HistogramBucket.compareTo.  Regular keys present are found; UNDER /
    OVER always are.  An absent REGULAR key whose compareTo against UNDERFLOW / OVERFLOW is 0 --
    (+0.0, +0.0), whose Float.compare with those buckets' 0.0 bounds is equal -- is found at the
    leaf it descends to: the UNDERFLOW leaf if it sorts before every regular bucket of the point,
    the OVERFLOW leaf if after every one (both are leaves of the red-black tree: inserted last at
    its extremes), else nothing."""
    t, lo, up = key
    if t == BK_UNDER:
        return under
    if t == BK_OVER:
        return over
    k = (_fcmp_key(lo), _fcmp_key(up))
    if k in counts:
        return counts[k]
    if lo == 0 and up == 0:
        if not reg_keys_sorted or k < reg_keys_sorted[0]:
            return under
        if k > reg_keys_sorted[-1]:
            return over
    return 0


def result_to_series(res: HistResult, percentiles) -> list[list[HistogramDataPoints]]:
    """Per emitted group: its percentile series (in request order) then its bucket series (the
    first point's buckets, HistogramBucketDataPointsAdaptor) -- TsdbQuery.java:1257-1287."""
    out = []
    P = res.n_pct
    D = res.n_buckets
    n_all = res.group_ptr[res.n_groups] if res.n_groups else 0

    def arr(ptr, n, dtype):
        return np.ctypeslib.as_array(ptr, (n,)).copy() if n else np.zeros(0, dtype)
    ts_all = arr(res.ts_ms, n_all, np.int64)
    pct_all = arr(res.pct, n_all * P, np.float64).reshape(n_all, P) if P else None
    kind_all = arr(res.codec, n_all, np.uint8)
    if res.show_buckets and n_all:
        cnt_all = arr(res.count, n_all * (D + 2), np.int64).reshape(n_all, D + 2)
        pres_all = arr(res.present, n_all * D, np.uint8).reshape(n_all, D).astype(bool)
        lo = [res.bucket_lower[d] for d in range(D)]
        up = [res.bucket_upper[d] for d in range(D)]
        # bucket_value for every (point, dictionary bucket) at once: each dictionary bucket's
        # rank in compareTo order, and per point the lowest / highest rank it holds
        order = sorted(range(D), key=lambda d: (_fcmp_key(lo[d]), _fcmp_key(up[d])))
        rank = np.empty(D, np.int64)
        rank[order] = np.arange(D)
        zero_key = np.array([lo[d] == 0 and up[d] == 0 for d in range(D)], bool)
        rmin = np.where(pres_all, rank[None, :], D).min(axis=1) if D else np.zeros(n_all, np.int64)
        rmax = np.where(pres_all, rank[None, :], -1).max(axis=1) if D else np.full(n_all, -1, np.int64)
        simple = kind_all == HCODEC_SIMPLE
        under_all = np.where(simple, cnt_all[:, D], 0)
        over_all = np.where(simple, cnt_all[:, D + 1], 0)
        reg_all = np.where(pres_all, cnt_all[:, :D], 0)
        if zero_key.any():
            absent = ~pres_all[:, zero_key]
            zr = rank[zero_key][None, :]
            none_held = (rmax < 0)[:, None]
            below = none_held | (zr < rmin[:, None])
            above = ~none_held & (zr > rmax[:, None])
            reg_all[:, zero_key] = np.where(absent & below, cnt_all[:, D][:, None],
                                            np.where(absent & above, cnt_all[:, D + 1][:, None],
                                                     reg_all[:, zero_key]))
        # getHistogramBucketsIfHas throws UnsupportedOperationException for other codecs: 0
        reg_all[~simple] = 0
    for g in range(res.n_groups):
        a, b = res.group_ptr[g], res.group_ptr[g + 1]
        gid = res.group_id[g]
        ts = ts_all[a:b]
        series = []
        for j, p in enumerate(percentiles):
            series.append(HistogramDataPoints(gid, ts, pct_all[a:b, j].copy(), np.zeros(b - a, np.uint8), percentile=p))
        if res.show_buckets and b > a and kind_all[a] == HCODEC_SIMPLE:   # (n_all > 0 here)
            first = np.flatnonzero(pres_all[a])
            keys = [(BK_UNDER, 0, 0)] + [(BK_REG, lo[d], up[d]) for d in first] + [(BK_OVER, 0, 0)]
            vals = np.concatenate([under_all[None, a:b], reg_all[a:b, first].T, over_all[None, a:b]])
            for kidx, key in enumerate(keys):
                series.append(HistogramDataPoints(gid, ts, vals[kidx], np.ones(b - a, np.uint8), bucket=key))
        out.append(series)
    return out
