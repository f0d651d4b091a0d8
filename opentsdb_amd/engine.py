"""ctypes binding of libtsdbhip (the MI355X engine behind include/tsdbhip.h).

The shared library is built in-tree (opentsdb_amd/lib/libtsdbhip.so, see
opentsdb_amd/csrc/Makefile).  There is no CPU fallback: if the library or a HIP device
is missing, constructing an Engine raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSDBHIP_LIB") or os.path.join(HERE, "lib", "libtsdbhip.so")
CSRC = os.path.join(HERE, "csrc")

# every symbol include/tsdbhip.h declares
EXPORTS = [
    "tsdbhip_abi_version", "tsdbhip_last_error", "tsdbhip_aggregator_get", "tsdbhip_aggregator_interpolation",
    "tsdbhip_parse_duration", "tsdbhip_parse_downsample", "tsdbhip_scan_bounds", "tsdbhip_init",
    "tsdbhip_destroy", "tsdbhip_load", "tsdbhip_synth", "tsdbhip_batch_sizes", "tsdbhip_batch_download",
    "tsdbhip_run", "tsdbhip_result_free", "tsdbhip_last_timing", "tsdbhip_partials_layout_get",
    "tsdbhip_run_partials", "tsdbhip_finalize", "tsdbhip_sync",
]


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
        L.tsdbhip_destroy.argtypes = [vp]
        L.tsdbhip_load.argtypes = [vp, C.POINTER(abi.Batch)]
        L.tsdbhip_synth.argtypes = [vp, C.POINTER(abi.SynthSpec)]
        L.tsdbhip_batch_sizes.argtypes = [vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64)]
        L.tsdbhip_batch_download.argtypes = [vp] + [C.c_void_p] * 7
        L.tsdbhip_run.argtypes = [vp, C.POINTER(abi.Query), C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_result_free.argtypes = [C.POINTER(abi.Result)]
        L.tsdbhip_last_timing.argtypes = [vp, C.POINTER(abi.Timing)]
        L.tsdbhip_partials_layout_get.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.POINTER(abi.PartialsLayout)]
        L.tsdbhip_run_partials.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p]
        L.tsdbhip_finalize.argtypes = [vp, C.POINTER(abi.Query), C.c_int64, C.c_void_p, C.c_int,
                                       C.POINTER(C.POINTER(abi.Result))]
        L.tsdbhip_sync.argtypes = [vp]
        _lib = L
    return _lib


def _check(rc):
    if rc < 0:
        raise EngineError(rc, lib().tsdbhip_last_error().decode(errors="replace"))
    return rc


def parse_downsample(spec: str) -> abi.Query:
    q = abi.new_query(0, 0)
    _check(lib().tsdbhip_parse_downsample(spec.encode(), C.byref(q)))
    return q


def scan_bounds(q: abi.Query):
    s, e = C.c_int64(), C.c_int64()
    _check(lib().tsdbhip_scan_bounds(C.byref(q), C.byref(s), C.byref(e)))
    return s.value, e.value


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
    """One tsdbhip context bound to one GPU."""

    def __init__(self, device: int = 0):
        self.ctx = C.c_void_p()
        _check(lib().tsdbhip_init(device, C.byref(self.ctx)))
        self.device = device
        self._batch = None

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

    def synth(self, n_series: int, start_s: int, n_points: int, period_ms: int, value_kind: int = 0,
              n_groups: int = 1, int_mod: int = 2000, seed: int = 0x5EED):
        sp = abi.SynthSpec(n_series, start_s, n_points, period_ms, value_kind, n_groups, int_mod, seed)
        _check(lib().tsdbhip_synth(self.ctx, C.byref(sp)))

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

    def run(self, q: abi.Query):
        """tsdbhip_run -> [(group_id, ts, bits, is_int)]; the arrays are views into the
        library's result, freed when the last of them is garbage-collected."""
        res = C.POINTER(abi.Result)()
        _check(lib().tsdbhip_run(self.ctx, C.byref(q), C.byref(res)))
        return abi.result_to_groups(res.contents, owner=_ResultOwner(res))

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

    # ---- multi-GPU exchange (see include/tsdbhip.h and opentsdb_amd/dist.py) ----
    def partials_layout(self, q: abi.Query, n_groups_global: int) -> abi.PartialsLayout:
        lay = abi.PartialsLayout()
        _check(lib().tsdbhip_partials_layout_get(self.ctx, C.byref(q), n_groups_global, C.byref(lay)))
        return lay

    def run_partials(self, q: abi.Query, n_groups_global: int, ptr: int):
        """This shard's per-(group, slot) partial states into `ptr` (device or host memory)."""
        _check(lib().tsdbhip_run_partials(self.ctx, C.byref(q), n_groups_global, C.c_void_p(ptr)))

    def finalize(self, q: abi.Query, n_groups_global: int, ptr: int, n_ranks: int):
        """Rank-ordered merge of n_ranks gathered partial buffers at `ptr` -> groups."""
        res = C.POINTER(abi.Result)()
        _check(lib().tsdbhip_finalize(self.ctx, C.byref(q), n_groups_global, C.c_void_p(ptr), n_ranks,
                                      C.byref(res)))
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
