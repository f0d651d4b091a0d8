"""ctypes mirror of include/tsdbhip.h (the C ABI of libtsdbhip).

Pure declarations: enums, structs and the helpers that turn numpy arrays into a
``tsdbhip_batch``.  Shared by the engine binding (:mod:`opentsdb_amd.engine`) and by the
test-only oracle binding (oracle/oracle.py), which consumes the same boundary types.
"""
from __future__ import annotations

import ctypes as C
from collections.abc import Sequence

import numpy as np

# ---- error codes (tsdbhip.h) -------------------------------------------------
TSDB_OK = 0
TSDB_E_ILLEGAL_DATA = -2
TSDB_E_ILLEGAL_ARGUMENT = -3
TSDB_E_ILLEGAL_STATE = -4
TSDB_E_UNSUPPORTED = -5
TSDB_E_RUNTIME = -6
TSDB_E_NO_SUCH_ELEMENT = -7
TSDB_E_ASSERTION = -8
TSDB_E_CLASS_CAST = -9
TSDB_E_NULL_POINTER = -10
TSDB_E_HIP = -20
TSDB_E_NOMEM = -21
TSDB_E_NOT_IMPLEMENTED = -22

ERROR_NAMES = {
    TSDB_E_ILLEGAL_DATA: "IllegalDataException",
    TSDB_E_ILLEGAL_ARGUMENT: "IllegalArgumentException",
    TSDB_E_ILLEGAL_STATE: "IllegalStateException",
    TSDB_E_UNSUPPORTED: "UnsupportedOperationException",
    TSDB_E_RUNTIME: "RuntimeException",
    TSDB_E_NO_SUCH_ELEMENT: "NoSuchElementException",
    TSDB_E_ASSERTION: "AssertionError",
    TSDB_E_CLASS_CAST: "ClassCastException",
    TSDB_E_NULL_POINTER: "NullPointerException",
    TSDB_E_HIP: "HipError",
    TSDB_E_NOMEM: "OutOfMemory",
    TSDB_E_NOT_IMPLEMENTED: "NotImplemented",
}

# ---- aggregators (src/core/Aggregators.java:47-203) ---------------------------
AGGREGATOR_NAMES = [
    "sum", "pfsum", "min", "max", "avg", "median", "none", "mult", "dev", "diff",
    "zimsum", "mimmin", "mimmax", "squareSum", "count", "first", "last",
    "p999", "p99", "p95", "p90", "p75", "p50",
    "ep999r3", "ep99r3", "ep95r3", "ep90r3", "ep75r3", "ep50r3",
    "ep999r7", "ep99r7", "ep95r7", "ep90r7", "ep75r7", "ep50r7",
]
AGG = {n: i for i, n in enumerate(AGGREGATOR_NAMES)}

INTERP_LERP, INTERP_ZIM, INTERP_MAX, INTERP_MIN, INTERP_PREV = range(5)
FILL_NONE, FILL_ZERO, FILL_NAN, FILL_NULL, FILL_SCALAR = range(5)
FILL_NAMES = ["none", "zero", "nan", "null", "scalar"]

# calendar units of a 'c' downsampling interval (tsdbhip.h TSDB_CAL_*)
CAL_NONE, CAL_MS, CAL_S, CAL_M, CAL_H, CAL_D, CAL_W, CAL_N, CAL_Y = range(9)

QF_ORDERED = 0x1

LONG_MAX = (1 << 63) - 1


def interpolation_of(agg: int) -> int:
    """Aggregator.interpolationMethod() (src/core/Aggregators.java:47-173)."""
    name = AGGREGATOR_NAMES[agg]
    if name == "pfsum":
        return INTERP_PREV
    if name in ("none", "zimsum", "squareSum", "count", "first", "last"):
        return INTERP_ZIM
    if name == "mimmin":
        return INTERP_MAX
    if name == "mimmax":
        return INTERP_MIN
    return INTERP_LERP


class Batch(C.Structure):
    _fields_ = [
        ("n_series", C.c_int64),
        ("series_row_ptr", C.POINTER(C.c_int64)),
        ("n_rows", C.c_int64),
        ("row_base_time", C.POINTER(C.c_uint32)),
        ("row_qual_off", C.POINTER(C.c_uint64)),
        ("row_val_off", C.POINTER(C.c_uint64)),
        ("qual", C.POINTER(C.c_uint8)),
        ("val", C.POINTER(C.c_uint8)),
        ("group_id", C.POINTER(C.c_int32)),
    ]


class TZ(C.Structure):
    """tsdbhip_tz: a zone's UTC offset transition table (see opentsdb_amd/tz.py)."""
    _fields_ = [
        ("n", C.c_int32),
        ("utc_ms", C.POINTER(C.c_int64)),
        ("offset_ms", C.POINTER(C.c_int32)),
    ]


class Query(C.Structure):
    _fields_ = [
        ("start_time", C.c_int64),
        ("end_time", C.c_int64),
        ("aggregator", C.c_int32),
        ("ds_function", C.c_int32),
        ("ds_fill", C.c_int32),
        ("ds_all", C.c_int32),
        ("ds_calendar", C.c_int32),
        ("ds_interval_ms", C.c_int64),
        ("rate", C.c_int32),
        ("rate_counter", C.c_int32),
        ("rate_drop_resets", C.c_int32),
        ("flags", C.c_int32),
        ("rate_counter_max", C.c_int64),
        ("rate_reset_value", C.c_int64),
        ("ds_tz", C.POINTER(TZ)),
    ]


class Result(C.Structure):
    _fields_ = [
        ("n_groups", C.c_int64),
        ("group_id", C.POINTER(C.c_int32)),
        ("group_ptr", C.POINTER(C.c_int64)),
        ("ts_ms", C.POINTER(C.c_int64)),
        ("value_bits", C.POINTER(C.c_uint64)),
        ("is_int", C.POINTER(C.c_uint8)),
    ]


class Timing(C.Structure):
    _fields_ = [
        ("decode_downsample_ms", C.c_double),
        ("group_reduce_ms", C.c_double),
        ("total_ms", C.c_double),
        ("datapoints", C.c_int64),
        ("bytes", C.c_int64),
        ("tiles", C.c_int64),
        ("redo_tiles", C.c_int64),
        ("fast_ms", C.c_double),
        ("index_ms", C.c_double),
        ("compact_ms", C.c_double),
        ("fused_queries", C.c_int64),
        ("exchange_ms", C.c_double),
        ("devices_ms", C.c_double),
        ("xfer_ms", C.c_double),
        ("select_ms", C.c_double),
        ("assemble_ms", C.c_double),
    ]


class SynthSpec(C.Structure):
    _fields_ = [
        ("n_series", C.c_int64),
        ("start_s", C.c_int64),
        ("n_points", C.c_int64),
        ("period_ms", C.c_int64),
        ("value_kind", C.c_int32),
        ("n_groups", C.c_int32),
        ("int_mod", C.c_int64),
        ("seed", C.c_uint64),
    ]


class PartialsLayout(C.Structure):
    _fields_ = [
        ("n_groups", C.c_int64),
        ("n_slots", C.c_int64),
        ("bytes", C.c_int64),
    ]


class RollupInterval(C.Structure):
    """tsdbhip_rollup_interval (RollupInterval, src/rollup/RollupInterval.java)."""
    _fields_ = [
        ("interval_s", C.c_int32),
        ("intervals", C.c_int32),
        ("units", C.c_char),
        ("interval_units", C.c_char),
        ("unit_multiplier", C.c_int16),
    ]


class RollupSpec(C.Structure):
    _fields_ = [
        ("interval", RollupInterval),
        ("start_s", C.c_int64),
        ("end_s", C.c_int64),
        ("n_funcs", C.c_int32),
        ("func", C.c_int32 * 4),
        ("agg_id", C.c_int32 * 4),
    ]


def new_query(start_time: int, end_time: int, aggregator: str | int = "sum", *,
              ds_function: int = -1, ds_interval_ms: int = 0, ds_fill: int = FILL_NONE,
              ds_all: bool = False, rate: bool = False, counter: bool = False,
              counter_max: int = LONG_MAX, reset_value: int = 0, drop_resets: bool = False,
              flags: int = 0, tz=None) -> Query:
    q = Query()
    q.start_time = start_time
    q.end_time = end_time
    q.aggregator = AGG[aggregator] if isinstance(aggregator, str) else aggregator
    q.ds_function = ds_function
    q.ds_fill = ds_fill
    q.ds_all = int(ds_all)
    q.ds_calendar = 0
    q.ds_interval_ms = ds_interval_ms
    q.rate = int(rate)
    q.rate_counter = int(counter)
    q.rate_drop_resets = int(drop_resets)
    q.rate_counter_max = counter_max
    q.rate_reset_value = reset_value
    q.flags = flags
    if tz is not None:
        set_timezone(q, tz)
    return q


def set_timezone(q: Query, tz) -> None:
    """The calendar time zone of q: a zone id (tz.table) or a tz.TzTable; None = UTC."""
    if tz is None:
        q.ds_tz = C.POINTER(TZ)()
        return
    from . import tz as _tz
    t = tz if isinstance(tz, _tz.TzTable) else _tz.table(tz)
    q.ds_tz = C.pointer(t.struct)   # the struct keeps the table's arrays alive


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class HostBatch:
    """Owns the numpy arrays behind a :class:`Batch` (keeps them alive)."""

    def __init__(self, series_row_ptr, row_base_time, row_qual_off, row_val_off, qual, val, group_id):
        self.series_row_ptr = np.ascontiguousarray(series_row_ptr, dtype=np.int64)
        self.row_base_time = np.ascontiguousarray(row_base_time, dtype=np.uint32)
        self.row_qual_off = np.ascontiguousarray(row_qual_off, dtype=np.uint64)
        self.row_val_off = np.ascontiguousarray(row_val_off, dtype=np.uint64)
        self.qual = np.ascontiguousarray(qual, dtype=np.uint8)
        self.val = np.ascontiguousarray(val, dtype=np.uint8)
        self.group_id = np.ascontiguousarray(group_id, dtype=np.int32)
        if self.qual.size == 0:
            self.qual = np.zeros(1, np.uint8)
        if self.val.size == 0:
            self.val = np.zeros(1, np.uint8)
        n = len(self.series_row_ptr) - 1
        assert n >= 0 and len(self.group_id) == n
        assert len(self.row_qual_off) == len(self.row_base_time) + 1
        assert len(self.row_val_off) == len(self.row_base_time) + 1
        self.c = Batch(
            n, _ptr(self.series_row_ptr, C.c_int64), len(self.row_base_time),
            _ptr(self.row_base_time, C.c_uint32), _ptr(self.row_qual_off, C.c_uint64),
            _ptr(self.row_val_off, C.c_uint64), _ptr(self.qual, C.c_uint8),
            _ptr(self.val, C.c_uint8), _ptr(self.group_id, C.c_int32))

    @property
    def n_series(self) -> int:
        return len(self.series_row_ptr) - 1

    @property
    def n_rows(self) -> int:
        return len(self.row_base_time)


class CellBatch(C.Structure):
    """tsdbhip_cell_batch: a scan's rows before compaction (every column of every row)."""
    _fields_ = [
        ("n_series", C.c_int64),
        ("series_row_ptr", C.POINTER(C.c_int64)),
        ("n_rows", C.c_int64),
        ("row_base_time", C.POINTER(C.c_uint32)),
        ("row_col_ptr", C.POINTER(C.c_int64)),
        ("n_cols", C.c_int64),
        ("col_qual_off", C.POINTER(C.c_uint64)),
        ("col_val_off", C.POINTER(C.c_uint64)),
        ("col_timestamp", C.POINTER(C.c_int64)),
        ("qual", C.POINTER(C.c_uint8)),
        ("val", C.POINTER(C.c_uint8)),
        ("group_id", C.POINTER(C.c_int32)),
        ("fix_duplicates", C.c_int32),
        ("use_otsdb_timestamp", C.c_int32),
        ("use_max_value", C.c_int32),
    ]


class HostCellBatch:
    """Owns the arrays behind a :class:`CellBatch`."""

    def __init__(self, series_row_ptr, row_base_time, row_col_ptr, col_qual_off, col_val_off, qual, val, group_id,
                 col_timestamp=None, fix_duplicates=False, use_otsdb_timestamp=False, use_max_value=True):
        self.series_row_ptr = np.ascontiguousarray(series_row_ptr, dtype=np.int64)
        self.row_base_time = np.ascontiguousarray(row_base_time, dtype=np.uint32)
        self.row_col_ptr = np.ascontiguousarray(row_col_ptr, dtype=np.int64)
        self.col_qual_off = np.ascontiguousarray(col_qual_off, dtype=np.uint64)
        self.col_val_off = np.ascontiguousarray(col_val_off, dtype=np.uint64)
        self.qual = np.ascontiguousarray(qual, dtype=np.uint8)
        self.val = np.ascontiguousarray(val, dtype=np.uint8)
        self.group_id = np.ascontiguousarray(group_id, dtype=np.int32)
        self.col_timestamp = None if col_timestamp is None else np.ascontiguousarray(col_timestamp, dtype=np.int64)
        if self.qual.size == 0:
            self.qual = np.zeros(1, np.uint8)
        if self.val.size == 0:
            self.val = np.zeros(1, np.uint8)
        ns, nr, nc = len(self.series_row_ptr) - 1, len(self.row_base_time), len(self.col_qual_off) - 1
        assert len(self.group_id) == ns and len(self.row_col_ptr) == nr + 1 and len(self.col_val_off) == nc + 1
        self.c = CellBatch(ns, _ptr(self.series_row_ptr, C.c_int64), nr, _ptr(self.row_base_time, C.c_uint32),
                           _ptr(self.row_col_ptr, C.c_int64), nc, _ptr(self.col_qual_off, C.c_uint64),
                           _ptr(self.col_val_off, C.c_uint64),
                           C.POINTER(C.c_int64)() if self.col_timestamp is None else _ptr(self.col_timestamp, C.c_int64),
                           _ptr(self.qual, C.c_uint8), _ptr(self.val, C.c_uint8), _ptr(self.group_id, C.c_int32),
                           int(fix_duplicates), int(use_otsdb_timestamp), int(use_max_value))

    @classmethod
    def from_rows(cls, series, group_ids, fix_duplicates=False, use_otsdb_timestamp=False, use_max_value=True):
        """series: [[(base_time, [(qualifier bytes, value bytes, timestamp | None), ...]), ...], ...]"""
        srp, bases, rcp, qo, vo, ts = [0], [], [0], [0], [0], []
        qb, vb = bytearray(), bytearray()
        any_ts = False
        for rows in series:
            for base, cols in rows:
                bases.append(base)
                for col in cols:
                    q, v = col[0], col[1]
                    t = col[2] if len(col) > 2 else None
                    any_ts |= t is not None
                    ts.append(0 if t is None else t)
                    qb += q
                    vb += v
                    qo.append(len(qb))
                    vo.append(len(vb))
                rcp.append(len(qo) - 1)
            srp.append(len(bases))
        return cls(srp, bases, rcp, qo, vo, np.frombuffer(bytes(qb), np.uint8), np.frombuffer(bytes(vb), np.uint8),
                   group_ids, np.array(ts, np.int64) if any_ts else None, fix_duplicates, use_otsdb_timestamp,
                   use_max_value)


class RollupBatch(C.Structure):
    """tsdbhip_rollup_batch: RollupSeq rows of the queried aggregate (+ count cells)."""
    _fields_ = [
        ("cells", Batch),
        ("row_cqual_off", C.POINTER(C.c_uint64)),
        ("row_cval_off", C.POINTER(C.c_uint64)),
        ("cqual", C.POINTER(C.c_uint8)),
        ("cval", C.POINTER(C.c_uint8)),
        ("interval", RollupInterval),
        ("fix_duplicates", C.c_int32),
    ]


class HostRollupBatch:
    """Owns the arrays behind a :class:`RollupBatch`.  `counts` is None (no count cells:
    RollupSeq.need_count false) or (row_cqual_off, row_cval_off, cqual, cval)."""

    def __init__(self, cells: HostBatch, counts, interval: RollupInterval, fix_duplicates: bool = False):
        self.cells = cells
        self.interval = interval
        self.fix_duplicates = bool(fix_duplicates)
        self.c = RollupBatch()
        self.c.cells = cells.c
        self.c.interval = interval
        self.c.fix_duplicates = int(fix_duplicates)
        if counts is None:
            self.counts = None
        else:
            cq_off, cv_off, cq, cv = counts
            cq_off = np.ascontiguousarray(cq_off, dtype=np.uint64)
            cv_off = np.ascontiguousarray(cv_off, dtype=np.uint64)
            cq = np.ascontiguousarray(cq, dtype=np.uint8)
            cv = np.ascontiguousarray(cv, dtype=np.uint8)
            if cq.size == 0:
                cq = np.zeros(1, np.uint8)
            if cv.size == 0:
                cv = np.zeros(1, np.uint8)
            assert len(cq_off) == cells.n_rows + 1 and len(cv_off) == cells.n_rows + 1
            self.counts = (cq_off, cv_off, cq, cv)
            self.c.row_cqual_off = _ptr(cq_off, C.c_uint64)
            self.c.row_cval_off = _ptr(cv_off, C.c_uint64)
            self.c.cqual = _ptr(cq, C.c_uint8)
            self.c.cval = _ptr(cv, C.c_uint8)

    @property
    def need_count(self) -> bool:
        return self.counts is not None


def _view(ptr, n: int, dtype, owner):
    """numpy view of n elements at a ctypes pointer; `owner` is kept alive by the view."""
    nbytes = n * np.dtype(dtype).itemsize
    buf = (C.c_uint8 * nbytes).from_address(C.cast(ptr, C.c_void_p).value)
    buf._owner = owner
    return np.frombuffer(buf, dtype)


class Groups(Sequence):
    """The groups of a tsdbhip_result as a sequence of (group_id, ts, bits, is_int) tuples over
    the result arrays (numpy views; the library's memory stays owned by `owner` while any view
    is alive).  The tuples are built when a group is accessed -- the arrays are already complete
    on the host -- as a JVM caller wraps the arrays as DataPoints without copying."""

    def __init__(self, gid, gp, ts, bits, isi):
        self._gid, self._gp, self._ts, self._bits, self._isi = gid, gp, ts, bits, isi

    def __len__(self):
        return len(self._gid)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        n = len(self._gid)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        a, b = int(self._gp[i]), int(self._gp[i + 1])
        return (int(self._gid[i]), self._ts[a:b], self._bits[a:b], self._isi[a:b])

    def __add__(self, other):
        return list(self) + list(other)

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return f"Groups({len(self)} groups, {int(self._gp[-1]) if len(self._gp) else 0} points)"


def result_to_groups(res: Result, owner=None):
    """A tsdbhip_result / ref_result as a sequence of (group_id, ts[int64], bits[uint64],
    is_int[uint8]) numpy tuples.  Without `owner` a list of copies; with it a lazy :class:`Groups`
    of views into the result memory, which `owner` frees when the last view is gone."""
    groups = []
    n = res.n_groups
    if n == 0:
        return groups
    gp = np.ctypeslib.as_array(res.group_ptr, shape=(n + 1,)).copy()
    gid = np.ctypeslib.as_array(res.group_id, shape=(n,)).copy()
    tot = int(gp[-1])
    if tot and owner is not None:
        ts = _view(res.ts_ms, tot, np.int64, owner)
        bits = _view(res.value_bits, tot, np.uint64, owner)
        isi = _view(res.is_int, tot, np.uint8, owner)
    elif tot:
        ts = np.ctypeslib.as_array(res.ts_ms, shape=(tot,)).copy()
        bits = np.ctypeslib.as_array(res.value_bits, shape=(tot,)).copy()
        isi = np.ctypeslib.as_array(res.is_int, shape=(tot,)).copy()
    else:
        ts = np.zeros(0, np.int64)
        bits = np.zeros(0, np.uint64)
        isi = np.zeros(0, np.uint8)
    if owner is not None:
        return Groups(gid, gp, ts, bits, isi)
    for g in range(n):
        a, b = int(gp[g]), int(gp[g + 1])
        groups.append((int(gid[g]), ts[a:b], bits[a:b], isi[a:b]))
    return groups
