"""In-memory data store with OpenTSDB's on-disk cell format (the MockBase analogue).

Producer side of the format the engine decodes.  Restates, for building inputs:
  * TSDB.addPoint(long / float / double)        src/core/TSDB.java:1012-1110
  * Internal.buildQualifier                     src/core/Internal.java:848-862
  * storeIntoDB base-time computation           src/core/TSDB.java:1164-1175
  * CompactionQueue compaction of a row         src/core/CompactionQueue.java:340-626
  * the HBase scan's row-key range              src/query/QueryUtil.java:323-344
and flattens the scanned Spans into the CSR ``tsdbhip_batch`` of include/tsdbhip.h.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

from . import abi

SECOND_MASK = 0xFFFFFFFF00000000
MAX_TIMESPAN = 3600
MS_MIXED_COMPACT = 1


class IllegalDataException(Exception):
    pass


# ---- value / qualifier encoding (TSDB.addPoint*, Internal.buildQualifier) -----

def encode_long(value: int) -> tuple[bytes, int]:
    """TSDB.addPoint(long): smallest of 1/2/4/8 bytes, flags = len-1 (TSDB.java:1012-1027)."""
    if -128 <= value <= 127:
        v = struct.pack(">b", value)
    elif -32768 <= value <= 32767:
        v = struct.pack(">h", value)
    elif -(1 << 31) <= value <= (1 << 31) - 1:
        v = struct.pack(">i", value)
    else:
        v = struct.pack(">q", value)
    return v, len(v) - 1


def encode_float(value: float) -> tuple[bytes, int]:
    """TSDB.addPoint(float): 4 bytes, flags FLAG_FLOAT|0x3 (TSDB.java:1097-1110)."""
    return struct.pack(">f", value), 0x8 | 0x3


def encode_double(value: float) -> tuple[bytes, int]:
    """TSDB.addPoint(double): 8 bytes, flags FLAG_FLOAT|0x7 (TSDB.java:1057-1070)."""
    return struct.pack(">d", value), 0x8 | 0x7


def base_time_of(ts: int) -> int:
    if ts & SECOND_MASK:
        s = ts // 1000
        return s - s % MAX_TIMESPAN
    return ts - ts % MAX_TIMESPAN


def build_qualifier(ts: int, flags: int) -> bytes:
    """Internal.buildQualifier (Internal.java:848-862)."""
    if ts & SECOND_MASK:
        base = base_time_of(ts)
        q = (((ts - base * 1000) << 6) | flags) | 0xF0000000
        return struct.pack(">I", q & 0xFFFFFFFF)
    base = base_time_of(ts)
    return struct.pack(">H", (((ts - base) << 4) | flags) & 0xFFFF)


def qualifier_offset_ms(q: bytes) -> int:
    if (q[0] & 0xF0) == 0xF0:
        return (struct.unpack(">I", q)[0] & 0x0FFFFFC0) >> 6
    return (struct.unpack(">H", q)[0] >> 4) * 1000


# ---- store ---------------------------------------------------------------------

class UidTable:
    """Mocked UniqueId: names get UIDs 1, 2, ... in first-use order (3-byte width)."""

    def __init__(self, preset: dict[str, int] | None = None):
        self.ids: dict[str, int] = dict(preset or {})

    def get(self, name: str) -> int:
        if name not in self.ids:
            self.ids[name] = max(self.ids.values(), default=0) + 1
        return self.ids[name]


@dataclass
class SeriesKey:
    metric: str
    tags: tuple  # sorted ((tagk, tagv), ...)


@dataclass
class _Row:
    cells: dict = field(default_factory=dict)  # qualifier bytes -> value bytes (latest put wins)
    order: list = field(default_factory=list)  # insertion order of qualifiers (newest last)


class MockStore:
    """Rows keyed by (metric uid, tags uids, base_time).  Cells are stored un-compacted,
    exactly like MockBase with write-back compaction disabled; compaction happens at
    scan time (SaltScanner.processRow -> TSDB.compact)."""

    def __init__(self, fix_duplicates: bool = False):
        self.metrics = UidTable()
        self.tagk = UidTable()
        self.tagv = UidTable()
        self.rows: dict[tuple, _Row] = {}
        self.fix_duplicates = fix_duplicates

    # TSDB.addPoint overloads
    def add_long(self, metric: str, ts: int, value: int, tags: dict):
        v, f = encode_long(int(value))
        self._put(metric, ts, v, f, tags)

    def add_float(self, metric: str, ts: int, value: float, tags: dict):
        if value != value or value in (float("inf"), float("-inf")):
            raise ValueError("value is NaN or Infinite")
        v, f = encode_float(value)
        self._put(metric, ts, v, f, tags)

    def add_double(self, metric: str, ts: int, value: float, tags: dict):
        if value != value or value in (float("inf"), float("-inf")):
            raise ValueError("value is NaN or Infinite")
        v, f = encode_double(value)
        self._put(metric, ts, v, f, tags)

    def _series_uids(self, metric: str, tags: dict):
        m = self.metrics.get(metric)
        t = tuple(sorted((self.tagk.get(k), self.tagv.get(v)) for k, v in tags.items()))
        return m, t

    def _put(self, metric, ts, value, flags, tags):
        if ts < 0 or (ts & SECOND_MASK and ts > 9999999999999):
            raise ValueError(f"invalid timestamp {ts}")
        m, t = self._series_uids(metric, tags)
        base = base_time_of(ts)
        key = (m, t, base)
        row = self.rows.setdefault(key, _Row())
        q = build_qualifier(ts, flags)
        row.cells[q] = value
        if q in row.order:
            row.order.remove(q)
        row.order.append(q)

    # CompactionQueue.Compaction (defaultMergeDataPoints + buildCompactedColumn)
    def compact(self, key) -> tuple[bytes, bytes]:
        row = self.rows[key]
        # heap order: by time offset; ties broken newest-first (ColumnDatapointIterator.compareTo)
        entries = []
        for age, q in enumerate(reversed(row.order)):
            entries.append((qualifier_offset_ms(q), age, q, row.cells[q]))
        entries.sort(key=lambda e: (e[0], e[1]))
        if len(entries) == 1:
            return entries[0][2], entries[0][3]
        quals, vals = [], []
        prev = -1
        ms_in_row = s_in_row = False
        for off, _, q, v in entries:
            if off == prev:
                if vals[-1] != v and not self.fix_duplicates:
                    raise IllegalDataException(f"Duplicate timestamp for key={key}, ms_offset={off}")
                continue
            prev = off
            quals.append(q)
            vals.append(v)
            if len(q) == 4:
                ms_in_row = True
            else:
                s_in_row = True
        meta = MS_MIXED_COMPACT if (ms_in_row and s_in_row) else 0
        if len(quals) > 1:
            return b"".join(quals), b"".join(vals) + bytes([meta])
        return quals[0], vals[0]

    # ---- scan (findSpans) --------------------------------------------------------
    def series(self, metric: str):
        """All series keys of a metric in SpanCmp order (metric uid, then tag uids)."""
        if metric not in self.metrics.ids:
            return []
        m = self.metrics.ids[metric]
        keys = sorted({(k[0], k[1]) for k in self.rows if k[0] == m}, key=lambda k: _tag_bytes(k[1]))
        return keys

    def scan(self, metric: str, scan_start_s: int, scan_end_s: int, tag_pred=None):
        """Rows of metric with base_time in [scan_start_s, scan_end_s), grouped per series
        in SpanCmp order.  Returns [(series_key, [(base_time, qual, val), ...]), ...]."""
        out = []
        for sk in self.series(metric):
            if tag_pred is not None and not tag_pred(sk[1]):
                continue
            rows = []
            for base in sorted(b for (m, t, b) in self.rows if (m, t) == sk):
                if scan_start_s <= base < scan_end_s:
                    q, v = self.compact((sk[0], sk[1], base))
                    rows.append((base, q, v))
            if rows:
                out.append((sk, rows))
        return out


def _tag_bytes(tags: tuple) -> bytes:
    return b"".join(k.to_bytes(3, "big") + v.to_bytes(3, "big") for k, v in tags)


def make_batch(spans, group_ids) -> abi.HostBatch:
    """Flatten [(key, [(base, qual, val), ...]), ...] into a tsdbhip_batch."""
    row_ptr = [0]
    bases, qoff, voff = [], [0], [0]
    qbuf, vbuf = bytearray(), bytearray()
    for _, rows in spans:
        for base, q, v in rows:
            bases.append(base)
            qbuf += q
            vbuf += v
            qoff.append(len(qbuf))
            voff.append(len(vbuf))
        row_ptr.append(len(bases))
    return abi.HostBatch(np.array(row_ptr, np.int64), np.array(bases, np.uint32),
                         np.array(qoff, np.uint64), np.array(voff, np.uint64),
                         np.frombuffer(bytes(qbuf), np.uint8), np.frombuffer(bytes(vbuf), np.uint8),
                         np.array(group_ids, np.int32))
