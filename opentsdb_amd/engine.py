"""ctypes binding of libtsdbhip (the MI355X engine behind include/tsdbhip.h).

The shared library is built in-tree (opentsdb_amd/lib/libtsdbhip.so, see
opentsdb_amd/csrc/Makefile).  There is no CPU fallback: if the library or a HIP device
is missing, constructing an Engine raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time

import numpy as np

from . import abi
from . import histogram as H

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSDBHIP_LIB") or os.path.join(HERE, "lib", "libtsdbhip.so")
CSRC = os.path.join(HERE, "csrc")

# every symbol include/tsdbhip.h declares
EXPORTS = [
    "tsdbhip_abi_version", "tsdbhip_last_error", "tsdbhip_aggregator_get", "tsdbhip_aggregator_interpolation",
    "tsdbhip_parse_duration", "tsdbhip_parse_downsample", "tsdbhip_scan_bounds", "tsdbhip_init",
    "tsdbhip_destroy", "tsdbhip_load", "tsdbhip_synth", "tsdbhip_batch_sizes", "tsdbhip_batch_download",
    "tsdbhip_run", "tsdbhip_result_free", "tsdbhip_last_timing", "tsdbhip_partials_layout_get",
    "tsdbhip_run_partials", "tsdbhip_run_partials_multi", "tsdbhip_finalize", "tsdbhip_sync", "tsdbhip_rollup_interval_parse",
    "tsdbhip_rollup_basetime", "tsdbhip_rollup_qualifier", "tsdbhip_rollup_run", "tsdbhip_rollup_download",
    "tsdbhip_sel_layout", "tsdbhip_sel_run_values", "tsdbhip_sel_select", "tsdbhip_assemble", "tsdbhip_run_multi",
    "tsdbhip_debug_rows", "tsdbhip_debug_sel_window", "tsdbhip_shard_bounds", "tsdbhip_load_shard", "tsdbhip_synth_shard",
    "tsdbhip_load_rollup", "tsdbhip_load_cells", "tsdbhip_load_histograms", "tsdbhip_hist_run",
    "tsdbhip_hist_run_range", "tsdbhip_hist_result_free", "tsdbhip_expr_map", "tsdbhip_expr_zip", "tsdbhip_expr_topn",
    "tsdbhip_batch_range_sizes", "tsdbhip_batch_download_range", "tsdbhip_expr_sync", "tsdbhip_init_devices",
    "tsdbhip_md_shard_mode", "tsdbhip_md_info", "tsdbhip_host_alloc", "tsdbhip_host_free", "tsdbhip_md_stats",
    "tsdbhip_device_count", "tsdbhip_set_option", "tsdbhip_get_option",
]

# developer options (tsdbhip_set_option, opentsdb_amd/csrc/opts.h)
OPTIONS = ["FAST", "SHORT", "ROWS", "HWIN", "SEQ", "SEQ_ROWS", "SEQ_WAVE", "INDEX_GENERIC", "CMP_CHUNK", "CMP_ROWS",
           "CMP_ONEPASS", "PCT_ROWS", "PCT_KEYS", "PCT_VONLY", "PCT_V6", "SEL_FUSED", "SEL_COLS", "SEL_WIN", "SEL_WAVE",
           "SEL_REG", "SELOPS", "RAW_LERPW", "RAW_SEL_TOP", "RAW_SEL_REG", "RO_FUSE", "RO_RUNS", "MULTI_FUSE", "EMIT_HALF", "HIST_WINDOW",
           "HIST_WS", "HIST_LAYOUT", "TRACE", "DBG"]

SHARD_AUTO, SHARD_SERIES, SHARD_GROUPS, SHARD_SPANS = -1, 0, 1, 2   # tsdbhip.h TSDB_SHARD_*
MD_AUTO, MD_COPY, MD_RCCL = -1, 0, 1                               # tsdbhip.h TSDB_MD_*


class _PinnedBlock:
    """Page-locked host memory (tsdbhip_host_alloc) exposed through __array_interface__: numpy
    arrays over it keep this object as their base (views collapse to it), so the block is freed
    only when the last array over it is gone."""

    def __init__(self, nbytes: int, dtype, shape):
        p = C.c_void_p()
        _check(lib().tsdbhip_host_alloc(max(1, int(nbytes)), C.byref(p)))
        self.ptr = p.value
        self.__array_interface__ = {"data": (self.ptr, False), "shape": tuple(shape),
                                    "typestr": np.dtype(dtype).str, "version": 3}

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.tsdbhip_host_free(self.ptr)
            self.ptr = None


def pinned_copy(a: np.ndarray) -> np.ndarray:
    """`a` copied into page-locked host memory (uploads from it are DMA transfers)."""
    a = np.ascontiguousarray(a)
    out = np.asarray(_PinnedBlock(a.nbytes, a.dtype, a.shape))
    out[...] = a
    return out


class EngineError(Exception):
    def __init__(self, code: int, msg: str):
        self.code = code
        self.java = abi.ERROR_NAMES.get(code, str(code))
        super().__init__(f"{self.java}: {msg}")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-j8", "-C", CSRC], check=True)
    return LIB_PATH


_lib = None


def lib():
    """Loads libtsdbhip.so (fails loudly if it is not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libtsdbhip is not built ({LIB_PATH}); run `make -C {CSRC}`")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.tsdbhip_last_error.restype = C.c_char_p
        L.tsdbhip_aggregator_get.argtypes = [C.c_char_p]
        L.tsdbhip_parse_duration.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
        L.tsdbhip_parse_downsample.argtypes = [C.c_char_p, C.POINTER(abi.Query)]
        L.tsdbhip_scan_bounds.argtypes = [C.POINTER(abi.Query), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.tsdbhip_init.argtypes = [C.c_int, C.POINTER(vp)]
        L.tsdbhip_init_devices.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(vp)]
        L.tsdbhip_md_shard_mode.argtypes = [vp, C.c_int]
        L.tsdbhip_md_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_void_p]
        L.tsdbhip_device_count.argtypes = [C.POINTER(C.c_int)]
        L.tsdbhip_set_option.argtypes = [C.c_char_p, C.c_int64]
        L.tsdbhip_get_option.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
        L.tsdbhip_md_stats.argtypes = [vp, C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double)]
        L.tsdbhip_destroy.argtypes = [vp]
        L.tsdbhip_host_alloc.argtypes = [C.c_uint64, C.POINTER(vp)]
        L.tsdbhip_host_free.argtypes = [vp]
        L.tsdbhip_host_free.restype = None
        L.tsdbhip_load.argtypes = [vp, C.POINTER(abi.Batch)]
        L.tsdbhip_synth.argtypes = [vp, C.POINTER(abi.SynthSpec)]
        L.tsdbhip_batch_sizes.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64)]
        L.tsdbhip_batch_download.argtypes = [vp] + [C.c_void_p] * 7
        L.tsdbhip_batch_range_sizes.argtypes = [vp, C.c_int64, C.c_int64, C.POINTER(C.c_int64),
                                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.tsdbhip_batch_download_range.argtypes = [vp, C.c_int64, C.c_int64] + [C.c_void_p] * 7
        L.tsdbhip_run.argtypes = [vp, C.POINTER(abi.Query), C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_result_free.argtypes = [C.POINTER(abi.Result)]
        L.tsdbhip_last_timing.argtypes = [vp, C.POINTER(abi.Timing)]
        L.tsdbhip_partials_layout_get.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.POINTER(abi.PartialsLayout)]
        L.tsdbhip_run_partials.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p]
        L.tsdbhip_run_partials_multi.argtypes = [vp, C.POINTER(abi.Query), C.c_int, C.c_int64, C.c_void_p]
        L.tsdbhip_finalize.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p, C.c_int,
                                       C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_sync.argtypes = [vp]
        L.tsdbhip_run_multi.argtypes = [vp, C.POINTER(abi.Query), C.c_int, C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_sel_layout.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p, C.POINTER(C.c_int64)]
        L.tsdbhip_sel_run_values.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.tsdbhip_sel_select.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p]
        L.tsdbhip_assemble.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_rollup_interval_parse.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(abi.RollupInterval)]
        L.tsdbhip_rollup_basetime.argtypes = [C.c_int64, C.POINTER(abi.RollupInterval), C.POINTER(C.c_int32)]
        L.tsdbhip_rollup_qualifier.argtypes = [C.c_int64, C.c_int32, C.c_int16, C.c_int32,
                                               C.POINTER(abi.RollupInterval), C.c_void_p]
        L.tsdbhip_rollup_run.argtypes = [vp, C.POINTER(abi.RollupSpec), C.POINTER(C.c_int64), C.POINTER(C.c_uint64)]
        L.tsdbhip_rollup_download.argtypes = [vp] + [C.c_void_p] * 5
        L.tsdbhip_debug_rows.argtypes = [vp] + [C.c_void_p] * 4
        L.tsdbhip_debug_sel_window.argtypes = [vp, C.c_void_p, C.c_void_p]
        L.tsdbhip_shard_bounds.argtypes = [C.POINTER(abi.Batch), C.c_int, C.c_int, C.c_void_p]
        L.tsdbhip_load_shard.argtypes = [vp, C.POINTER(abi.Batch), C.c_int, C.c_int64, C.c_int64]
        L.tsdbhip_synth_shard.argtypes = [vp, C.POINTER(abi.SynthSpec), C.c_int64, C.c_int64]
        L.tsdbhip_load_rollup.argtypes = [vp, C.POINTER(abi.RollupBatch)]
        L.tsdbhip_load_cells.argtypes = [vp, C.POINTER(abi.CellBatch)]
        L.tsdbhip_load_histograms.argtypes = [vp, C.POINTER(H.HistBatch)]
        L.tsdbhip_hist_run.argtypes = [vp, C.POINTER(abi.Query), C.c_int, C.POINTER(C.c_float), C.c_int,
                                       C.POINTER(C.POINTER(H.HistResult))]
        L.tsdbhip_hist_run_range.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_int64, C.c_int,
                                             C.POINTER(C.c_float), C.c_int, C.POINTER(C.POINTER(H.HistResult))]
        L.tsdbhip_hist_result_free.argtypes = [C.POINTER(H.HistResult)]
        _lib = L
    return _lib


def _check(rc):
    if rc < 0:
        raise EngineError(rc, lib().tsdbhip_last_error().decode(errors="replace"))
    return rc


def device_count() -> int:
    """HIP devices visible to the library (tsdbhip_device_count).  Use this rather than
    torch.cuda.device_count() before building an RCCL context: torch's wheel carries its own
    HIP / HSA runtime, and initialising it beside the library's broke ncclCommInitAll here."""
    n = C.c_int()
    _check(lib().tsdbhip_device_count(C.byref(n)))
    return n.value


def set_option(name: str, value) -> None:
    """tsdbhip_set_option: a developer option (kernel choice for tests / A/B runs), process-wide;
    None or -1 resets it to the production choice."""
    _check(lib().tsdbhip_set_option(name.encode(), -1 if value is None else int(value)))


def get_option(name: str) -> int:
    v = C.c_int64()
    _check(lib().tsdbhip_get_option(name.encode(), C.byref(v)))
    return v.value


def reset_options() -> None:
    for n in OPTIONS:
        set_option(n, -1)


class options:
    """Context manager: developer options set for the block, reset after it."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        for k, v in self.kw.items():
            set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k in self.kw:
            set_option(k, -1)
        return False


def parse_downsample(spec: str) -> abi.Query:
    q = abi.new_query(0, 0)
    _check(lib().tsdbhip_parse_downsample(spec.encode(), C.byref(q)))
    return q


def scan_bounds(q: abi.Query):
    s, e = C.c_int64(), C.c_int64()
    _check(lib().tsdbhip_scan_bounds(C.byref(q), C.byref(s), C.byref(e)))
    return s.value, e.value


def shard_bounds(batch: abi.HostBatch, world: int, mode: int = SHARD_SERIES):
    """tsdbhip_shard_bounds: world + 1 byte-balanced boundaries (host logic, no GPU needed)."""
    b = np.zeros(world + 1, np.int64)
    _check(lib().tsdbhip_shard_bounds(C.byref(batch.c), world, mode, b.ctypes.data))
    return b


def rollup_interval(interval: str, row_span: str) -> abi.RollupInterval:
    """RollupInterval.builder().setInterval(interval).setRowSpan(row_span).build()."""
    iv = abi.RollupInterval()
    _check(lib().tsdbhip_rollup_interval_parse(interval.encode(), row_span.encode(), C.byref(iv)))
    return iv


def rollup_basetime(timestamp: int, iv: abi.RollupInterval) -> int:
    """RollupUtils.getRollupBasetime."""
    out = C.c_int32()
    _check(lib().tsdbhip_rollup_basetime(timestamp, C.byref(iv), C.byref(out)))
    return out.value


def rollup_qualifier(timestamp: int, basetime: int, flags: int, aggregator_id: int, iv: abi.RollupInterval) -> bytes:
    """RollupUtils.buildRollupQualifier."""
    out = (C.c_uint8 * 3)()
    _check(lib().tsdbhip_rollup_qualifier(timestamp, basetime, flags, aggregator_id, C.byref(iv), out))
    return bytes(out)


class RollupCells:
    """Cells of one rollup generation, in (function, series, time) order."""

    def __init__(self, series, base_time, qualifier, val_off, value):
        self.series = series          # int32 [n] batch series index
        self.base_time = base_time    # uint32 [n] row base time (s)
        self.qualifier = qualifier    # uint8 [n, 3]
        self.val_off = val_off        # uint64 [n + 1]
        self.value = value            # uint8 [val_off[-1]]

    def __len__(self):
        return len(self.series)

    def cell(self, i):
        """(series, base_time, qualifier bytes, value bytes) of cell i."""
        return (int(self.series[i]), int(self.base_time[i]), bytes(self.qualifier[i]),
                bytes(self.value[self.val_off[i]:self.val_off[i + 1]]))


class _ResultOwner:
    """Frees a tsdbhip_result when the numpy views into it are gone."""

    def __init__(self, res):
        self.res = res
        self.free = lib().tsdbhip_result_free

    def __del__(self):
        if self.res:
            self.free(self.res)
            self.res = None


class Engine:
    """One tsdbhip context bound to one GPU -- or, with `devices`, one multi-device context
    (tsdbhip_init_devices) that shards every load over those GPUs and answers queries as one GPU
    would."""

    def __init__(self, device: int = 0, devices=None, transport: int = MD_AUTO):
        self.ctx = C.c_void_p()
        if devices is None:
            _check(lib().tsdbhip_init(device, C.byref(self.ctx)))
        else:
            arr = np.ascontiguousarray(devices, dtype=np.int32)
            _check(lib().tsdbhip_init_devices(arr.ctypes.data, len(arr), transport, C.byref(self.ctx)))
            device = int(arr[0])
        self.device = device
        self.devices = None if devices is None else [int(d) for d in devices]
        self._batch = None
        self.last_call_ms = 0.0

    def shard_mode(self, mode: int):
        """tsdbhip_md_shard_mode: SHARD_AUTO / SHARD_SERIES / SHARD_GROUPS for the next loads."""
        _check(lib().tsdbhip_md_shard_mode(self.ctx, mode))

    def md_info(self):
        """tsdbhip_md_info -> (n_devices, transport, shard mode of the resident batch, series per device)."""
        nd, tr, mode = C.c_int(), C.c_int(), C.c_int()
        _check(lib().tsdbhip_md_info(self.ctx, C.byref(nd), C.byref(tr), C.byref(mode), None))
        per = np.zeros(nd.value, np.int64)
        _check(lib().tsdbhip_md_info(self.ctx, None, None, None, per.ctypes.data))
        return nd.value, tr.value, mode.value, per

    def md_stats(self):
        """tsdbhip_md_stats -> (per-device Timing list, RCCL communicator ranks, device-to-device
        bytes) of the last run on a multi-device context."""
        nd = C.c_int()   # (n_devices only: md_info's per-device series walks the shards)
        _check(lib().tsdbhip_md_info(self.ctx, C.byref(nd), None, None, None))
        nd = nd.value
        per = (abi.Timing * nd)()
        ranks, xb = C.c_int(), C.c_double()
        _check(lib().tsdbhip_md_stats(self.ctx, C.cast(per, C.c_void_p), C.byref(ranks), C.byref(xb)))
        return list(per), ranks.value, xb.value

    def close(self):
        if self.ctx:
            lib().tsdbhip_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, batch: abi.HostBatch):
        _check(lib().tsdbhip_load(self.ctx, C.byref(batch.c)))
        self._batch = batch

    def load_cells(self, cb: abi.HostCellBatch):
        """tsdbhip_load_cells: the scan's rows compacted on the GPU become the resident batch."""
        _check(lib().tsdbhip_load_cells(self.ctx, C.byref(cb.c)))
        self._batch = cb

    def load_histograms(self, hb: "H.HostHistBatch"):
        """tsdbhip_load_histograms: the resident histogram store."""
        _check(lib().tsdbhip_load_histograms(self.ctx, C.byref(hb.c)))

    def run_histogram(self, q: abi.Query, percentiles=(), show_buckets: bool = False, span_range=None):
        """TsdbQuery.runHistogram over the resident histogram store: per emitted group the list
        of its DataPoints (percentile series, then bucket series), see histogram.result_to_series.
        span_range=(start_ms, end_ms): HistogramAggregationIterator bounds given directly
        (tsdbhip_hist_run_range, every row)."""
        pct = (C.c_float * max(1, len(percentiles)))(*[float(x) for x in percentiles])
        res = C.POINTER(H.HistResult)()
        if span_range is None:
            _check(lib().tsdbhip_hist_run(self.ctx, C.byref(q), len(percentiles), pct, int(bool(show_buckets)),
                                          C.byref(res)))
        else:
            _check(lib().tsdbhip_hist_run_range(self.ctx, C.byref(q), int(span_range[0]), int(span_range[1]),
                                                len(percentiles), pct, int(bool(show_buckets)), C.byref(res)))
        try:
            return H.result_to_series(res.contents, [float(C.c_float(x).value) for x in percentiles])
        finally:
            lib().tsdbhip_hist_result_free(res)

    def load_rollup(self, rb: abi.HostRollupBatch):
        """tsdbhip_load_rollup: a rollup table's scan result as the resident batch; run()
        then answers rollup queries over it."""
        _check(lib().tsdbhip_load_rollup(self.ctx, C.byref(rb.c)))
        self._batch = rb

    def synth(self, n_series: int, start_s: int, n_points: int, period_ms: int, value_kind: int = 0,
              n_groups: int = 1, int_mod: int = 2000, seed: int = 0x5EED):
        sp = abi.SynthSpec(n_series, start_s, n_points, period_ms, value_kind, n_groups, int_mod, seed)
        _check(lib().tsdbhip_synth(self.ctx, C.byref(sp)))

    def synth_shard(self, pos_begin: int, pos_end: int, n_series: int, start_s: int, n_points: int,
                    period_ms: int, value_kind: int = 0, n_groups: int = 1, int_mod: int = 2000, seed: int = 0x5EED):
        """Batch positions [pos_begin, pos_end) of the n_series synthetic store (one rank's shard)."""
        sp = abi.SynthSpec(n_series, start_s, n_points, period_ms, value_kind, n_groups, int_mod, seed)
        _check(lib().tsdbhip_synth_shard(self.ctx, C.byref(sp), pos_begin, pos_end))

    def load_shard(self, batch: abi.HostBatch, mode: int, begin: int, end: int):
        """tsdbhip_load_shard: range [begin, end) of the batch under a TSDB_SHARD_* mode."""
        _check(lib().tsdbhip_load_shard(self.ctx, C.byref(batch.c), mode, begin, end))
        self._batch = batch

    def download(self) -> abi.HostBatch:
        ns, nr, qb, vb = C.c_int64(), C.c_int64(), C.c_uint64(), C.c_uint64()
        _check(lib().tsdbhip_batch_sizes(self.ctx, C.byref(ns), C.byref(nr), C.byref(qb), C.byref(vb)))
        srp = np.zeros(ns.value + 1, np.int64)
        base = np.zeros(max(1, nr.value), np.uint32)
        qo = np.zeros(nr.value + 1, np.uint64)
        vo = np.zeros(nr.value + 1, np.uint64)
        q = np.zeros(max(1, qb.value), np.uint8)
        v = np.zeros(max(1, vb.value), np.uint8)
        g = np.zeros(max(1, ns.value), np.int32)
        _check(lib().tsdbhip_batch_download(self.ctx, srp.ctypes.data, base.ctypes.data, qo.ctypes.data,
                                            vo.ctypes.data, q.ctypes.data, v.ctypes.data, g.ctypes.data))
        return abi.HostBatch(srp, base[:nr.value], qo, vo, q[:qb.value], v[:vb.value], g[:ns.value])

    def n_series(self) -> int:
        ns, nr, qb, vb = C.c_int64(), C.c_int64(), C.c_uint64(), C.c_uint64()
        _check(lib().tsdbhip_batch_sizes(self.ctx, C.byref(ns), C.byref(nr), C.byref(qb), C.byref(vb)))
        return ns.value

    def resident_groups(self) -> np.ndarray:
        """Group id of every resident series position (the resident order is group-sorted)."""
        n = self.n_series()
        g = np.zeros(max(1, n), np.int32)
        _check(lib().tsdbhip_batch_download_range(self.ctx, 0, n, None, None, None, None, None, None,
                                                  g.ctypes.data))
        return g[:n]

    def download_range(self, s0: int, s1: int) -> abi.HostBatch:
        """Resident series positions [s0, s1) as a host batch (group ids kept)."""
        nr, qb, vb = C.c_int64(), C.c_uint64(), C.c_uint64()
        _check(lib().tsdbhip_batch_range_sizes(self.ctx, s0, s1, C.byref(nr), C.byref(qb), C.byref(vb)))
        srp = np.zeros(s1 - s0 + 1, np.int64)
        base = np.zeros(max(1, nr.value), np.uint32)
        qo = np.zeros(nr.value + 1, np.uint64)
        vo = np.zeros(nr.value + 1, np.uint64)
        q = np.zeros(max(1, qb.value), np.uint8)
        v = np.zeros(max(1, vb.value), np.uint8)
        g = np.zeros(max(1, s1 - s0), np.int32)
        _check(lib().tsdbhip_batch_download_range(self.ctx, s0, s1, srp.ctypes.data, base.ctypes.data,
                                                  qo.ctypes.data, vo.ctypes.data, q.ctypes.data, v.ctypes.data,
                                                  g.ctypes.data))
        return abi.HostBatch(srp, base[:nr.value], qo, vo, q[:qb.value], v[:vb.value], g[:s1 - s0])

    def run(self, q: abi.Query):
        """tsdbhip_run -> [(group_id, ts, bits, is_int)]; the arrays are views into the
        library's result, freed when the last of them is garbage-collected."""
        res = C.POINTER(abi.Result)()
        t = time.perf_counter()
        _check(lib().tsdbhip_run(self.ctx, C.byref(q), C.byref(res)))
        self.last_call_ms = (time.perf_counter() - t) * 1000.0   # the C call alone (host wall time)
        return abi.result_to_groups(res.contents, owner=_ResultOwner(res))

    def run_multi(self, queries):
        """tsdbhip_run_multi: one decode + downsample pass shared by several queries."""
        n = len(queries)
        arr = (abi.Query * n)(*queries)
        outs = (C.POINTER(abi.Result) * n)()
        t = time.perf_counter()
        _check(lib().tsdbhip_run_multi(self.ctx, arr, n, outs))
        self.last_call_ms = (time.perf_counter() - t) * 1000.0   # the C call alone (host wall time)
        return [abi.result_to_groups(outs[i].contents, owner=_ResultOwner(outs[i])) for i in range(n)]

    def run_rollup_batch(self, rb: abi.HostRollupBatch, q: abi.Query):
        self.load_rollup(rb)
        return self.run(q)

    def run_batch(self, batch: abi.HostBatch, q: abi.Query):
        """Runner for TsdbQuery: load the query's spans, then run."""
        self.load(batch)
        return self.run(q)

    def timing(self) -> abi.Timing:
        t = abi.Timing()
        _check(lib().tsdbhip_last_timing(self.ctx, C.byref(t)))
        return t

    def sync(self):
        _check(lib().tsdbhip_sync(self.ctx))

    def debug_rows(self):
        """Test hook: k_index's per-row (ndp, flags, lsb, absmax) of the resident batch."""
        ns, nr, qb, vb = C.c_int64(), C.c_int64(), C.c_uint64(), C.c_uint64()
        _check(lib().tsdbhip_batch_sizes(self.ctx, C.byref(ns), C.byref(nr), C.byref(qb), C.byref(vb)))
        n = max(1, nr.value)
        ndp, flags = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        lsb, amax = np.zeros(n, np.int32), np.zeros(n, np.float64)
        _check(lib().tsdbhip_debug_rows(self.ctx, ndp.ctypes.data, flags.ctypes.data, lsb.ctypes.data,
                                        amax.ctypes.data))
        k = nr.value
        return ndp[:k], flags[:k], lsb[:k], amax[:k]

    def debug_sel_window(self):
        """Test hook: (runs, misses) of the sampled-window percentile group-by select."""
        runs, misses = C.c_int64(), C.c_int64()
        _check(lib().tsdbhip_debug_sel_window(self.ctx, C.byref(runs), C.byref(misses)))
        return runs.value, misses.value

    # ---- rollup generation (tsdbhip_rollup_run) ----
    def rollup_run(self, interval: abi.RollupInterval, start_s: int, end_s: int,
                   funcs=(("sum", 0), ("count", 1), ("max", 2), ("min", 3))):
        """Generates the rollup cells of the resident batch on the device; returns
        (n_cells, value_bytes).  funcs = [(downsample function, rollup aggregator id)]."""
        sp = abi.RollupSpec()
        sp.interval = interval
        sp.start_s = start_s
        sp.end_s = end_s
        sp.n_funcs = len(funcs)
        for i, (fn, aid) in enumerate(funcs):
            sp.func[i] = abi.AGG[fn] if isinstance(fn, str) else fn
            sp.agg_id[i] = aid
        n, b = C.c_int64(), C.c_uint64()
        _check(lib().tsdbhip_rollup_run(self.ctx, C.byref(sp), C.byref(n), C.byref(b)))
        return n.value, b.value

    def rollup_download(self, n_cells: int, value_bytes: int) -> RollupCells:
        series = np.zeros(max(1, n_cells), np.int32)
        base = np.zeros(max(1, n_cells), np.uint32)
        qual = np.zeros((max(1, n_cells), 3), np.uint8)
        voff = np.zeros(n_cells + 1, np.uint64)
        val = np.zeros(max(1, value_bytes), np.uint8)
        _check(lib().tsdbhip_rollup_download(self.ctx, series.ctypes.data, base.ctypes.data, qual.ctypes.data,
                                             voff.ctypes.data, val.ctypes.data))
        return RollupCells(series[:n_cells], base[:n_cells], qual[:n_cells], voff, val[:value_bytes])

    def rollup(self, interval: abi.RollupInterval, start_s: int, end_s: int,
               funcs=(("sum", 0), ("count", 1), ("max", 2), ("min", 3))) -> RollupCells:
        return self.rollup_download(*self.rollup_run(interval, start_s, end_s, funcs))

    # ---- multi-GPU exchange (see include/tsdbhip.h and opentsdb_amd/dist.py) ----
    def partials_layout(self, q: abi.Query, n_groups_global: int) -> abi.PartialsLayout:
        lay = abi.PartialsLayout()
        _check(lib().tsdbhip_partials_layout_get(self.ctx, C.byref(q), n_groups_global, C.byref(lay)))
        return lay

    def run_partials(self, q: abi.Query, n_groups_global: int, ptr: int):
        """This shard's per-(group, slot) partial states into `ptr` (device or host memory)."""
        _check(lib().tsdbhip_run_partials(self.ctx, C.byref(q), n_groups_global, C.c_void_p(ptr)))

    def run_partials_multi(self, queries, n_groups_global: int, ptr: int):
        """Partial states of several queries sharing the downsampling, from one fused pass: query
        i's buffer at ptr + i * partials_layout(queries[i]).bytes."""
        n = len(queries)
        arr = (abi.Query * n)(*queries)
        _check(lib().tsdbhip_run_partials_multi(self.ctx, arr, n, n_groups_global, C.c_void_p(ptr)))

    def finalize(self, q: abi.Query, n_groups_global: int, ptr: int, n_ranks: int):
        """Rank-ordered merge of n_ranks gathered partial buffers at `ptr` -> groups."""
        res = C.POINTER(abi.Result)()
        _check(lib().tsdbhip_finalize(self.ctx, C.byref(q), n_groups_global, C.c_void_p(ptr), n_ranks,
                                      C.byref(res)))
        try:
            return abi.result_to_groups(res.contents)
        finally:
            lib().tsdbhip_result_free(res)


    # ---- multi-GPU percentile / median group-by (values to the owning rank) ----
    def sel_layout(self, q: abi.Query, n_groups_global: int):
        """(local spans per group [n_groups_global] int64, slots K)."""
        counts = np.zeros(max(1, n_groups_global), np.int64)
        k = C.c_int64()
        _check(lib().tsdbhip_sel_layout(self.ctx, C.byref(q), n_groups_global, counts.ctypes.data, C.byref(k)))
        return counts[:n_groups_global], int(k.value)

    def sel_run_values(self, q: abi.Query, n_groups_global: int, vals: int, uni: int, act: int):
        """Local span contributions ([g][k][i] f64), emit flags [G][K] u8, group active [G] u32."""
        _check(lib().tsdbhip_sel_run_values(self.ctx, C.byref(q), n_groups_global, C.c_void_p(vals),
                                            C.c_void_p(uni), C.c_void_p(act)))

    def sel_select(self, q: abi.Query, n_groups_global: int, vals: int, counts: np.ndarray, uni: int,
                   out_val: int, out_flag: int):
        counts = np.ascontiguousarray(counts, np.int64)
        _check(lib().tsdbhip_sel_select(self.ctx, C.byref(q), n_groups_global, C.c_void_p(vals),
                                        C.c_void_p(counts.ctypes.data), C.c_void_p(uni), C.c_void_p(out_val),
                                        C.c_void_p(out_flag)))

    def assemble(self, q: abi.Query, n_groups_global: int, val: int, flag: int, act: int):
        res = C.POINTER(abi.Result)()
        _check(lib().tsdbhip_assemble(self.ctx, C.byref(q), n_groups_global, C.c_void_p(val), C.c_void_p(flag),
                                      C.c_void_p(act), C.byref(res)))
        try:
            return abi.result_to_groups(res.contents)
        finally:
            lib().tsdbhip_result_free(res)


_default = None


def default_engine() -> Engine:
    global _default
    if _default is None:
        _default = Engine(int(os.environ.get("TSDBHIP_DEVICE", "0")))
    return _default
