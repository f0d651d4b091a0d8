"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU oracle (oracle/refcpu.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module.  The product (opentsdb_amd, libtsdbhip) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess

import numpy as np

from opentsdb_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSDB_ORACLE_LIB") or os.path.join(HERE, "build", "librefcpu.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        target = ["san"] if LIB_PATH.endswith("_ubsan.so") else []
        subprocess.run(["make", "-C", HERE] + target, check=True, stdout=subprocess.DEVNULL)
    return LIB_PATH


_lib = None


class RefHistResult(C.Structure):
    _fields_ = [
        ("n_groups", C.c_int64),
        ("group_id", C.POINTER(C.c_int32)),
        ("group_ptr", C.POINTER(C.c_int64)),
        ("ts", C.POINTER(C.c_int64)),
        ("n_pct", C.c_int32),
        ("pct", C.POINTER(C.c_double)),
        ("bk_ptr", C.POINTER(C.c_int64)),
        ("bk_type", C.POINTER(C.c_int32)),
        ("bk_lo", C.POINTER(C.c_uint32)),
        ("bk_up", C.POINTER(C.c_uint32)),
        ("bk_val_off", C.POINTER(C.c_int64)),
        ("bk_val", C.POINTER(C.c_int64)),
    ]


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.ref_last_error.restype = C.c_char_p
        L.ref_view_array.restype = vp
        L.ref_view_array.argtypes = [C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_int64, C.c_int]
        L.ref_view_span.restype = vp
        L.ref_view_span.argtypes = [C.c_int64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint8), C.POINTER(C.c_uint8)]
        L.ref_view_downsampler.restype = vp
        L.ref_view_downsampler.argtypes = [vp, C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int64, C.c_int64,
                                           C.c_int64, C.c_int64, C.c_int32]
        L.ref_view_downsampler_tz.restype = vp
        L.ref_view_downsampler_tz.argtypes = [vp, C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int64, C.c_int64,
                                              C.c_int64, C.c_int64, C.c_int32, C.POINTER(abi.TZ)]
        L.ref_view_rate.restype = vp
        L.ref_view_rate.argtypes = [vp, C.c_int32, C.c_int64, C.c_int64, C.c_int32]
        L.ref_view_aggregate.restype = vp
        L.ref_view_aggregate.argtypes = [C.POINTER(vp), C.c_int64, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int32]
        L.ref_view_free.argtypes = [vp]
        L.ref_has_next.argtypes = [vp]
        L.ref_seek.argtypes = [vp, C.c_int64]
        L.ref_drain.restype = C.c_int64
        L.ref_drain.argtypes = [vp, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
        L.ref_agg_run_long.argtypes = [C.c_int32, C.POINTER(C.c_int64), C.c_int64, C.POINTER(C.c_int64)]
        L.ref_agg_run_double.argtypes = [C.c_int32, C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double)]
        L.ref_parse_duration.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
        L.ref_parse_downsample.argtypes = [C.c_char_p, C.POINTER(abi.Query)]
        L.ref_aggregator_get.argtypes = [C.c_char_p]
        L.ref_scan_bounds.argtypes = [C.POINTER(abi.Query), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.ref_run_query.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Query), C.POINTER(C.POINTER(abi.Result))]
        L.ref_run_query_mt.argtypes = [C.POINTER(abi.Batch), C.POINTER(abi.Query), C.c_int,
                                       C.POINTER(C.POINTER(abi.Result))]
        L.ref_result_free.argtypes = [C.POINTER(abi.Result)]
        L.ref_compact_row.argtypes = [C.c_int64, C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.POINTER(C.c_void_p),
                                      C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_int, C.c_int,
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.POINTER(C.c_void_p),
                                      C.POINTER(C.c_int64)]
        L.ref_free.argtypes = [C.c_void_p]
        L.ref_run_rollup_query.argtypes = [C.POINTER(abi.RollupBatch), C.POINTER(abi.Query),
                                           C.POINTER(C.POINTER(abi.Result))]
        L.ref_run_hist.argtypes = [C.c_void_p, C.POINTER(abi.Query), C.c_int, C.POINTER(C.c_float), C.c_int,
                                   C.POINTER(C.POINTER(RefHistResult))]
        L.ref_run_hist_range.argtypes = [C.c_void_p, C.POINTER(abi.Query), C.c_int64, C.c_int64, C.c_int,
                                         C.POINTER(C.c_float), C.c_int, C.POINTER(C.POINTER(RefHistResult))]
        L.ref_hist_result_free.argtypes = [C.POINTER(RefHistResult)]
        L.ref_hist_value_percentile.argtypes = [C.c_char_p, C.c_int64, C.c_int, C.c_double, C.POINTER(C.c_double)]
        L.ref_rollup_scan_bounds.argtypes = [C.POINTER(abi.Query), C.POINTER(abi.RollupInterval),
                                             C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        _lib = L
    return _lib


class OracleError(Exception):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{abi.ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code
        self.java = abi.ERROR_NAMES.get(code, str(code))


def _err(code):
    raise OracleError(code, lib().ref_last_error().decode(errors="replace"))


def d2bits(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", x))[0]


def bits2d(b: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", b & 0xFFFFFFFFFFFFFFFF))[0]


class View:
    """Owning handle of a ref_view; ownership moves into wrapping views."""

    def __init__(self, ptr, keep=()):
        if not ptr:
            _err(-3)
        self.ptr = ptr
        self.keep = list(keep)
        self.owned = True

    def _take(self):
        assert self.owned, "view already consumed"
        self.owned = False
        return self.ptr

    def seek(self, ts: int):
        rc = lib().ref_seek(self.ptr, ts)
        if rc < 0:
            _err(rc)

    def has_next(self) -> bool:
        rc = lib().ref_has_next(self.ptr)
        if rc < 0:
            _err(rc)
        return bool(rc)

    def drain(self, cap: int = 1 << 20):
        ts = np.zeros(cap, np.int64)
        isi = np.zeros(cap, np.int32)
        bits = np.zeros(cap, np.uint64)
        n = lib().ref_drain(self.ptr, cap, ts.ctypes.data_as(C.POINTER(C.c_int64)),
                            isi.ctypes.data_as(C.POINTER(C.c_int32)), bits.ctypes.data_as(C.POINTER(C.c_uint64)))
        if n < 0:
            _err(n)
        n = min(n, cap)
        out = []
        for i in range(n):
            if isi[i]:
                out.append((int(ts[i]), True, int(np.int64(bits[i].astype(np.int64)))))
            else:
                out.append((int(ts[i]), False, bits2d(int(bits[i]))))
        return out

    def __del__(self):
        if getattr(self, "owned", False) and self.ptr:
            try:
                lib().ref_view_free(self.ptr)
            except Exception:
                pass


def array_view(points, generator: bool = False) -> View:
    """points: iterable of (ts_ms, is_int, value)."""
    pts = list(points)
    n = len(pts)
    ts = np.array([p[0] for p in pts] or [0], np.int64)
    isi = np.array([1 if p[1] else 0 for p in pts] or [0], np.int32)
    bits = np.array([(int(p[2]) if p[1] else d2bits(float(p[2]))) for p in pts] or [0], np.int64)
    ptr = lib().ref_view_array(ts.ctypes.data_as(C.POINTER(C.c_int64)), isi.ctypes.data_as(C.POINTER(C.c_int32)),
                               bits.ctypes.data_as(C.POINTER(C.c_int64)), n, int(generator))
    return View(ptr)


def span_view(base_times, quals, vals) -> View:
    """One Span from a list of compacted rows (base_time_s, qualifier bytes, value bytes)."""
    qo = np.zeros(len(quals) + 1, np.uint64)
    vo = np.zeros(len(vals) + 1, np.uint64)
    qo[1:] = np.cumsum([len(q) for q in quals])
    vo[1:] = np.cumsum([len(v) for v in vals])
    qb = np.frombuffer(b"".join(quals) or b"\0", np.uint8).copy()
    vb = np.frombuffer(b"".join(vals) or b"\0", np.uint8).copy()
    bt = np.array(base_times, np.uint32)
    ptr = lib().ref_view_span(len(quals), bt.ctypes.data_as(C.POINTER(C.c_uint32)),
                              qo.ctypes.data_as(C.POINTER(C.c_uint64)), vo.ctypes.data_as(C.POINTER(C.c_uint64)),
                              qb.ctypes.data_as(C.POINTER(C.c_uint8)), vb.ctypes.data_as(C.POINTER(C.c_uint8)))
    return View(ptr, keep=(qo, vo, qb, vb, bt))


def parse_downsample(spec: str) -> abi.Query:
    q = abi.new_query(0, 0)
    rc = lib().ref_parse_downsample(spec.encode(), C.byref(q))
    if rc < 0:
        _err(rc)
    return q


def downsampler(src: View, spec: str, start_time: int = 0, end_time: int = 0,
                query_start: int = 0, query_end: int = abi.LONG_MAX, tz=None) -> View:
    """Downsampler (fill none) or FillingDownsampler, as Span.downsampler builds them; tz: the
    specification's time zone (a zone id or opentsdb_amd.tz.TzTable; None = UTC)."""
    q = parse_downsample(spec)
    tzs = None
    if tz is not None:
        from opentsdb_amd import tz as _tz
        tzs = (tz if isinstance(tz, _tz.TzTable) else _tz.table(tz)).struct
    ptr = lib().ref_view_downsampler_tz(src._take(), q.ds_function, q.ds_interval_ms, q.ds_fill, q.ds_all,
                                        start_time, end_time, query_start, query_end, q.ds_calendar,
                                        C.byref(tzs) if tzs is not None else None)
    if not ptr:
        _err(-3)
    keep = list(src.keep) + ([tzs] if tzs is not None else [])
    return View(ptr, keep=keep)


def downsampler_raw(src: View, function: str, interval_ms: int, fill: int = abi.FILL_NONE,
                    start_time: int = 0, end_time: int = 0) -> View:
    """The deprecated Downsampler(source, interval_ms, function) constructor."""
    ptr = lib().ref_view_downsampler(src._take(), abi.AGG[function], interval_ms, fill, 0,
                                     start_time, end_time, 0, 0, 0)
    if not ptr:
        _err(-3)
    return View(ptr, keep=src.keep)


def rate(src: View, counter=False, counter_max=abi.LONG_MAX, reset_value=0, drop_resets=False) -> View:
    ptr = lib().ref_view_rate(src._take(), int(counter), counter_max, reset_value, int(drop_resets))
    return View(ptr, keep=src.keep)


def aggregate(srcs, start_time: int, end_time: int, aggregator: str, interpolation: int | None = None,
              rate: bool = False) -> View:
    agg = abi.AGG[aggregator]
    if interpolation is None:
        interpolation = abi.interpolation_of(agg)
    arr = (C.c_void_p * max(1, len(srcs)))()
    keep = []
    for i, s in enumerate(srcs):
        arr[i] = s._take()
        keep += s.keep
    ptr = lib().ref_view_aggregate(arr, len(srcs), start_time, end_time, agg, interpolation, int(rate))
    if not ptr:
        _err(-3)
    return View(ptr, keep=keep)


def agg_run_long(name: str, values) -> int:
    v = np.ascontiguousarray(values, np.int64)
    out = C.c_int64()
    rc = lib().ref_agg_run_long(abi.AGG[name], v.ctypes.data_as(C.POINTER(C.c_int64)), len(v), C.byref(out))
    if rc < 0:
        _err(rc)
    return out.value


def agg_run_double(name: str, values) -> float:
    v = np.ascontiguousarray(values, np.float64)
    out = C.c_double()
    rc = lib().ref_agg_run_double(abi.AGG[name], v.ctypes.data_as(C.POINTER(C.c_double)), len(v), C.byref(out))
    if rc < 0:
        _err(rc)
    return out.value


def parse_duration(s: str) -> int:
    out = C.c_int64()
    rc = lib().ref_parse_duration(s.encode(), C.byref(out))
    if rc < 0:
        _err(rc)
    return out.value


def scan_bounds(q: abi.Query):
    s, e = C.c_int64(), C.c_int64()
    lib().ref_scan_bounds(C.byref(q), C.byref(s), C.byref(e))
    return s.value, e.value


def compact_row(columns, fix_duplicates: bool = True, timestamps=None, use_otsdb_timestamp: bool = False,
                use_max_value: bool = True):
    """CompactionQueue.Compaction.compact() of one row (query time): columns = [(qualifier
    bytes, value bytes)] in scan order, timestamps = their KeyValue timestamps (default: the
    position).  use_otsdb_timestamp selects dtcsMergeDataPoints (CompactionQueue.java:508-547),
    keeping the max (use_max_value) or min value at a repeated offset.  Returns (qualifier,
    value), None (no datapoint) or raises OracleError."""
    n = len(columns)
    bufs = [(C.create_string_buffer(bytes(q), max(1, len(q))), C.create_string_buffer(bytes(v), max(1, len(v))))
            for q, v in columns]
    qp = (C.c_void_p * max(1, n))(*[C.cast(b[0], C.c_void_p) for b in bufs])
    vp = (C.c_void_p * max(1, n))(*[C.cast(b[1], C.c_void_p) for b in bufs])
    ql = (C.c_int64 * max(1, n))(*[len(q) for q, _ in columns])
    vl = (C.c_int64 * max(1, n))(*[len(v) for _, v in columns])
    ts = (C.c_int64 * max(1, n))(*(timestamps if timestamps is not None else range(n)))
    oq, ov = C.c_void_p(), C.c_void_p()
    oql, ovl = C.c_int64(), C.c_int64()
    rc = lib().ref_compact_row(n, qp, ql, vp, vl, ts, int(fix_duplicates),
                               (1 if use_max_value else 2) if use_otsdb_timestamp else 0, C.byref(oq), C.byref(oql), C.byref(ov),
                               C.byref(ovl))
    if rc < 0:
        _err(rc)
    if rc == 0:
        return None
    try:
        return C.string_at(oq, oql.value), C.string_at(ov, ovl.value)
    finally:
        lib().ref_free(oq)
        lib().ref_free(ov)


def run_rollup_query(rb: abi.HostRollupBatch, q: abi.Query):
    """TsdbQuery.run() with a RollupQuery (RollupSpans over rb) on the oracle."""
    res = C.POINTER(abi.Result)()
    rc = lib().ref_run_rollup_query(C.byref(rb.c), C.byref(q), C.byref(res))
    if rc < 0:
        _err(rc)
    try:
        return abi.result_to_groups(res.contents)
    finally:
        lib().ref_result_free(res)


def rollup_scan_bounds(q: abi.Query, iv: abi.RollupInterval):
    s, e = C.c_int64(), C.c_int64()
    rc = lib().ref_rollup_scan_bounds(C.byref(q), C.byref(iv), C.byref(s), C.byref(e))
    if rc < 0:
        _err(rc)
    return s.value, e.value


def run_query(batch: abi.HostBatch, q: abi.Query, threads: int = 1):
    """TsdbQuery.run() on the oracle: list of (group_id, ts, bits, is_int)."""
    res = C.POINTER(abi.Result)()
    if threads > 1:
        rc = lib().ref_run_query_mt(C.byref(batch.c), C.byref(q), threads, C.byref(res))
    else:
        rc = lib().ref_run_query(C.byref(batch.c), C.byref(q), C.byref(res))
    if rc < 0:
        _err(rc)
    try:
        return abi.result_to_groups(res.contents)
    finally:
        lib().ref_result_free(res)


def run_hist(hb, q: abi.Query, percentiles=(), show_buckets: bool = False, span_range=None):
    """TsdbQuery.runHistogram on the oracle (oracle/refhist.c): per emitted group the list of its
    DataPoints (opentsdb_amd.histogram.HistogramDataPoints), percentile series then bucket series."""
    from opentsdb_amd import histogram as H
    pct = (C.c_float * max(1, len(percentiles)))(*[float(x) for x in percentiles])
    res = C.POINTER(RefHistResult)()
    if span_range is None:
        rc = lib().ref_run_hist(C.cast(C.byref(hb.c), C.c_void_p), C.byref(q), len(percentiles), pct,
                                int(bool(show_buckets)), C.byref(res))
    else:
        rc = lib().ref_run_hist_range(C.cast(C.byref(hb.c), C.c_void_p), C.byref(q), int(span_range[0]),
                                      int(span_range[1]), len(percentiles), pct, int(bool(show_buckets)),
                                      C.byref(res))
    if rc < 0:
        _err(rc)
    try:
        r = res.contents
        P = len(percentiles)
        out = []
        for g in range(r.n_groups):
            a, b = r.group_ptr[g], r.group_ptr[g + 1]
            gid = r.group_id[g]
            ts = np.array([r.ts[i] for i in range(a, b)], np.int64)
            series = []
            for j in range(P):
                vals = np.array([r.pct[i * P + j] for i in range(a, b)], np.float64)
                series.append(H.HistogramDataPoints(gid, ts, vals, np.zeros(b - a, np.uint8),
                                                    percentile=float(pct[j])))
            off = r.bk_val_off[g]
            for k, bi in enumerate(range(r.bk_ptr[g], r.bk_ptr[g + 1])):
                vals = np.array([r.bk_val[off + k * (b - a) + i] for i in range(b - a)], np.int64)
                series.append(H.HistogramDataPoints(gid, ts, vals, np.ones(b - a, np.uint8),
                                                    bucket=(r.bk_type[bi], r.bk_lo[bi], r.bk_up[bi])))
            out.append(series)
        return out
    finally:
        lib().ref_hist_result_free(res)


def hist_value_percentile(value: bytes, kind: int, p: float):
    """SimpleHistogram.percentile / the long test codec's percentile of one stored value (with
    its codec id byte); None if the value does not decode."""
    out = C.c_double()
    rc = lib().ref_hist_value_percentile(value, len(value), kind, p, C.byref(out))
    return None if rc < 0 else out.value
