"""Host side of the rollup read path: the caller half of
tsdbhip_load_rollup.

The reference keeps this above the aggregation path, and so does this mirror:

  * RollupConfig -- aggregator ids and the configured intervals, with the best-match rule a
    downsampling interval picks its table by (src/rollup/RollupConfig.java:166-200,279-289);
  * RollupStore  -- the rollup tables as TSDB.addAggregatePoint writes them
    (src/core/TSDB.java:1322-1588): one cell per (row key, aggregator, timestamp) with the
    qualifier [aggregator id][offset << 4 | flags] (RollupUtils.buildRollupQualifier
    :143-171), or an old "<agg>:" string prefix; a row key's cells come back from a scan in
    qualifier byte order, one version per qualifier;
  * scan_cells() -- TsdbQuery's rollup scan (src/core/TsdbQuery.java:1415-1460: the
    qualifier filter of the rollup aggregator, or of sum and count for avg) and
    RollupSeq.setRow / addRow's classification of each cell as the aggregate's value or a
    count (src/rollup/RollupSeq.java:122-230, the prefix stripped), flattened into the
    tsdbhip_rollup_batch of include/tsdbhip.h.

The engine then restates RollupSpan / RollupSeq iteration and the Downsampler's rollup
branches on the device (opentsdb_amd/csrc/engine.cpp tsdbhip_load_rollup / run_rollup).
"""
from __future__ import annotations

import struct

import numpy as np

from . import abi
from .store import MockStore, encode_long

SECOND_MASK = 0xFFFFFFFF00000000
AGGREGATOR_MASK = 0x7F   # RollupUtils.AGGREGATOR_MASK


class NoSuchRollupForIntervalException(Exception):
    pass


class RollupConfig:
    """RollupConfig: aggregator name -> id, interval name -> RollupInterval."""

    def __init__(self, agg_ids: dict, intervals):
        """intervals: (interval, row_span) or (interval, row_span, is_default) -- the default
        interval is the raw table (RollupInterval.isDefaultInterval); at most one (:93-103)."""
        from . import engine
        self.ids = {k.lower(): int(v) for k, v in agg_ids.items()}
        self.intervals = {}
        self.default = None
        for item in intervals:
            iv, span = item[0], item[1]
            if iv in self.intervals:
                raise ValueError(f"Only one interval of each type can be configured: {iv}")
            if len(item) > 2 and item[2]:
                if self.default is not None:
                    raise ValueError(f"Multiple default intervals configured. Only one is allowed: {iv}")
                self.default = iv
            self.intervals[iv] = engine.rollup_interval(iv, span)

    def isDefaultInterval(self, name: str) -> bool:   # RollupInterval.isDefaultInterval :298-300
        return name == self.default

    def getIdForAggregator(self, agg: str) -> int:   # :279-289
        if not agg:
            raise ValueError("Aggregator cannot be null or empty.")
        if agg.lower() not in self.ids:
            raise ValueError(f"No ID found mapping to aggregator: {agg}")
        return self.ids[agg.lower()]

    def getRollupInterval(self, interval_s: int, str_interval: str = ""):   # :166-200
        """Configured intervals equal to or dividing interval_s, largest first."""
        if interval_s <= 0:
            raise ValueError("Interval cannot be null or empty")
        found = [(iv.interval_s, name) for name, iv in self.intervals.items()
                 if iv.interval_s == interval_s or interval_s % iv.interval_s == 0]
        if not found:
            raise NoSuchRollupForIntervalException(str(interval_s))
        return [name for _, name in sorted(found, reverse=True)]


def normalize_agg(agg: str) -> str:
    """RollupQuery ctor :69-80: zimsum / mimmax / mimmin read the sum / max / min columns."""
    return {"zimsum": "sum", "mimmax": "max", "mimmin": "min"}.get(agg, agg)


class RollupStore:
    """Rollup tables keyed by interval name; uids shared with a raw MockStore."""

    def __init__(self, config: RollupConfig, raw: MockStore | None = None):
        self.config = config
        self.raw = raw if raw is not None else MockStore()
        self.tables = {name: {} for name in config.intervals}   # name -> {(m, tags, base): {qual: value}}

    # TSDB.addAggregatePoint (long / float / double overloads) :1322-1440
    def add_aggregate_point(self, metric: str, ts: int, value, tags: dict, interval: str, aggregator: str,
                            kind: str | None = None):
        if kind is None:
            kind = "long" if isinstance(value, int) else "float"
        if kind == "long":
            v, flags = encode_long(int(value))
        else:
            if value != value or value in (float("inf"), float("-inf")):
                raise ValueError(f"value is NaN or Infinite: {value}")
            v, flags = (struct.pack(">f", value), 0x8 | 0x3) if kind == "float" else (struct.pack(">d", value), 0x8 | 0x7)
        if ts < 0 or (ts & SECOND_MASK) != 0:   # :1463-1469: rollups take seconds only
            raise ValueError(f"{'negative' if ts < 0 else 'bad'} timestamp={ts}")
        from . import engine
        iv = self.config.intervals[interval]
        agg_id = self.config.getIdForAggregator(aggregator)
        base = engine.rollup_basetime(ts, iv)
        qual = engine.rollup_qualifier(ts, base, flags, agg_id, iv)
        m, t = self.raw._series_uids(metric, tags)
        self.tables[interval].setdefault((m, t, base), {})[qual] = v

    def add_column(self, interval: str, metric: str, tags: dict, base: int, qualifier: bytes, value: bytes):
        """A raw cell (e.g. the old "sum:" string-prefixed qualifier, TestTsdbQueryRollup.oldStringPrefix)."""
        m, t = self.raw._series_uids(metric, tags)
        self.tables[interval].setdefault((m, t, base), {})[bytes(qualifier)] = bytes(value)

    def series(self, interval: str, metric: str):
        m = self.raw.metrics.ids.get(metric)
        if m is None:
            return []
        from .store import _tag_bytes
        return sorted({(k[0], k[1]) for k in self.tables[interval] if k[0] == m}, key=lambda k: _tag_bytes(k[1]))

    def scan_cells(self, interval: str, metric: str, ds_function: str, group_by: str, tag_pred=None):
        """The scan of a rollup query (TsdbQuery.java:1415-1460) and RollupSeq's cell
        classification (RollupSeq.java:122-230).  Returns [(series_key, [(base, values,
        counts)])] in row key order, values / counts lists of (2-byte qualifier, value
        bytes), and whether the query reads counts (RollupSeq.need_count)."""
        rollup_agg = normalize_agg(ds_function)
        gb = normalize_agg(group_by)
        need_count = gb in ("avg", "dev")
        cfg = self.config
        # scanner qualifier filter
        if rollup_agg != "avg":
            prefixes = [rollup_agg.encode(), bytes([cfg.getIdForAggregator(rollup_agg) & 0xFF])]
        else:
            prefixes = [b"sum", b"count", bytes([cfg.getIdForAggregator("sum") & 0xFF]),
                        bytes([cfg.getIdForAggregator("count") & 0xFF])]
        if need_count:
            agg_id, count_id = cfg.getIdForAggregator("sum"), cfg.getIdForAggregator("count")
            agg_prefix = b"sum:"   # RollupQuery.agg_prefix of an avg group-by
        else:
            agg_id = cfg.getIdForAggregator(rollup_agg)   # RollupSeq ctor: throws if unmapped
            count_id = None
            agg_prefix = (gb + ":").encode()   # RollupQuery.getRollupAggPrefix (the group-by's name)
        out = []
        for sk in self.series(interval, metric):
            if tag_pred is not None and not tag_pred(sk[1]):
                continue
            rows = []
            for base in sorted(b for (m, t, b) in self.tables[interval] if (m, t) == sk):
                cells = self.tables[interval][(sk[0], sk[1], base)]
                vals, cnts = [], []
                for q in sorted(cells):   # HBase returns a row's columns in qualifier order
                    if not any(q.startswith(p) for p in prefixes):
                        continue
                    v = cells[q]
                    if need_count:
                        if (q[0] & AGGREGATOR_MASK) == agg_id:
                            vals.append((q[1:3], v))
                        elif (q[0] & AGGREGATOR_MASK) == count_id:
                            cnts.append((q[1:3], v))
                        elif q.startswith(b"sum:"):
                            vals.append((q[4:6], v))
                        elif q.startswith(b"count:"):
                            cnts.append((q[6:8], v))
                        else:
                            raise ValueError("IllegalDataException: Attempt to add a different aggregate cell, "
                                             "expected aggregator either SUM or COUNT")
                    else:
                        if (q[0] & AGGREGATOR_MASK) == agg_id:
                            vals.append((q[1:3], v))
                        elif q.startswith(agg_prefix):
                            vals.append((q[len(agg_prefix):len(agg_prefix) + 2], v))
                        else:
                            raise ValueError("IllegalDataException: Attempt to add a different aggregate cell")
                if vals or cnts:
                    rows.append((base, vals, cnts))
            if rows:
                out.append((sk, rows))
        return out, need_count


def make_rollup_batch(spans, group_ids, interval: abi.RollupInterval, need_count: bool,
                      fix_duplicates: bool = False) -> abi.HostRollupBatch:
    """Flatten scan_cells() output into a tsdbhip_rollup_batch."""
    row_ptr, bases = [0], []
    qoff, voff, cqoff, cvoff = [0], [0], [0], [0]
    qb, vb, cqb, cvb = bytearray(), bytearray(), bytearray(), bytearray()
    for _, rows in spans:
        for base, vals, cnts in rows:
            bases.append(base)
            for q, v in vals:
                qb += q
                vb += v
            for q, v in cnts:
                cqb += q
                cvb += v
            qoff.append(len(qb))
            voff.append(len(vb))
            cqoff.append(len(cqb))
            cvoff.append(len(cvb))
        row_ptr.append(len(bases))
    cells = abi.HostBatch(np.array(row_ptr, np.int64), np.array(bases, np.uint32), np.array(qoff, np.uint64),
                          np.array(voff, np.uint64), np.frombuffer(bytes(qb), np.uint8),
                          np.frombuffer(bytes(vb), np.uint8), np.array(group_ids, np.int32))
    counts = None
    if need_count:
        counts = (np.array(cqoff, np.uint64), np.array(cvoff, np.uint64), np.frombuffer(bytes(cqb), np.uint8),
                  np.frombuffer(bytes(cvb), np.uint8))
    return abi.HostRollupBatch(cells, counts, interval, fix_duplicates)
