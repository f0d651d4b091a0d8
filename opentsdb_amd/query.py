"""Host-side mirror of the reference query API for the aggregation path.

The Java host keeps these classes unchanged and binds libtsdbhip through JNI
(INTEGRATION.md).  No JDK exists in this pipeline, so this module restates the pieces
of them that feed the C ABI, with the same names, argument meaning and exceptions, so
the parity tests read like the reference's own tests:

  * TsdbQuery.setStartTime / setEndTime / setTimeSeries / downsample / run
      (src/core/TsdbQuery.java:262-319, 434-560, 716-1049)
  * DownsamplingSpecification(String)    (src/core/DownsamplingSpecification.java:116-191)
  * RateOptions                          (src/core/RateOptions.java:27-97)
  * DataPoints / DataPoint views of a result (src/core/DataPoints.java, DataPoint.java)

run() does what findSpans + GroupByAndAggregateCB do on the host (scan the store for
the metric, filter tags, group spans by the group-by tag values in ByteMap order) and
hands the flattened Spans to a runner -- libtsdbhip on the GPU by default.
"""
from __future__ import annotations

import struct
import time
from dataclasses import dataclass

import numpy as np

from . import abi
from .store import MockStore, make_batch

SECOND_MASK = 0xFFFFFFFF00000000


class QueryException(Exception):
    """A reference exception surfaced through the C ABI (Java class in .java)."""

    def __init__(self, code: int, msg: str = ""):
        self.code = code
        self.java = abi.ERROR_NAMES.get(code, str(code))
        super().__init__(f"{self.java}: {msg}")


@dataclass
class RateOptions:
    counter: bool = False
    counter_max: int = abi.LONG_MAX
    reset_value: int = 0
    drop_resets: bool = False


def parse_duration(duration: str) -> int:
    """DateTime.parseDuration (src/utils/DateTime.java:186-226)."""
    unit = 0
    while unit < len(duration) and duration[unit].isdigit():
        unit += 1
        if unit >= len(duration):
            raise ValueError(f"Invalid duration, must have an integer and unit: {duration}")
    if unit == 0:
        raise ValueError(f"Invalid duration (number): {duration}")
    interval = int(duration[:unit])
    if interval <= 0:
        raise ValueError(f"Zero or negative duration: {duration}")
    c = duration[-1].lower()
    if c == "s":
        if len(duration) >= 2 and duration[-2] == "m":
            return interval
        mult = 1
    else:
        mult = {"m": 60, "h": 3600, "d": 86400, "w": 604800, "n": 2592000, "y": 31536000}.get(c)
        if mult is None:
            raise ValueError(f"Invalid duration (suffix): {duration}")
    return interval * mult * 1000


@dataclass
class DownsamplingSpecification:
    """new DownsamplingSpecification(String) / (interval, function, fill)."""
    interval: int = 0
    function: str | None = None
    fill_policy: str = "none"
    run_all: bool = False
    use_calendar: bool = False
    calendar_unit: int = 0     # abi.CAL_* of a 'c' interval (DateTime.unitsToCalendarType)
    timezone: str | None = None   # setTimezone (DownsamplingSpecification.java:199-207); None = UTC

    def setTimezone(self, tz: str) -> None:
        if tz is None:
            raise ValueError("Timezone cannot be null")
        self.timezone = tz

    @classmethod
    def parse(cls, spec: str) -> "DownsamplingSpecification":
        parts = spec.split("-")
        while parts and parts[-1] == "":
            parts.pop()
        if len(parts) < 2:
            raise ValueError(f"Invalid downsampling specifier '{spec}': must provide at least interval and function")
        if len(parts) > 3:
            raise ValueError(f"Invalid downsampling specifier '{spec}': must consist of interval, function, and optional fill policy")
        ds = cls()
        if "all" in parts[0]:
            ds.run_all = True
        elif parts[0].endswith("c"):
            ds.interval = parse_duration(parts[0][:-1])
            ds.use_calendar = True
            d = parts[0][:-1]
            ds.calendar_unit = abi.CAL_MS if d.lower().endswith("ms") else \
                {"s": abi.CAL_S, "m": abi.CAL_M, "h": abi.CAL_H, "d": abi.CAL_D, "w": abi.CAL_W, "n": abi.CAL_N,
                 "y": abi.CAL_Y}[d[-1]]
        else:
            ds.interval = parse_duration(parts[0])
        if parts[1] not in abi.AGG:
            raise ValueError(f"No such downsampling function: {parts[1]}")
        if parts[1] == "none":
            raise ValueError("cannot use the NONE aggregator for downsampling")
        ds.function = parts[1]
        if len(parts) == 3:
            if parts[2].lower() not in abi.FILL_NAMES:
                raise ValueError(f"Unrecognized fill policy: {parts[2]}")
            ds.fill_policy = parts[2].lower()
        return ds


class DataPoint:
    __slots__ = ("_ts", "_int", "_v")

    def __init__(self, ts: int, is_int: bool, v):
        self._ts, self._int, self._v = ts, is_int, v

    def timestamp(self) -> int:
        return self._ts

    def isInteger(self) -> bool:
        return self._int

    def longValue(self) -> int:
        if not self._int:
            raise TypeError("ClassCastException: value is a double")
        return self._v

    def doubleValue(self) -> float:
        if self._int:
            raise TypeError("ClassCastException: value is a long")
        return self._v

    def toDouble(self) -> float:
        return float(self._v)


class DataPoints:
    """One SpanGroup's materialised output (arrays from tsdbhip_result)."""

    def __init__(self, group_id: int, ts: np.ndarray, bits: np.ndarray, is_int: np.ndarray,
                 metric: str = "", group_key: tuple = ()):
        self.group_id = group_id
        self.ts = np.asarray(ts, np.int64)
        self.bits = np.asarray(bits, np.uint64)
        self.is_int = np.asarray(is_int, np.uint8)
        self.metric = metric
        self.group_key = group_key

    def size(self) -> int:
        return len(self.ts)

    def timestamp(self, i: int) -> int:
        return int(self.ts[i])

    def isInteger(self, i: int) -> bool:
        return bool(self.is_int[i])

    def longValue(self, i: int) -> int:
        return int(self.bits[i].astype(np.int64))

    def doubleValue(self, i: int) -> float:
        return struct.unpack("<d", struct.pack("<Q", int(self.bits[i])))[0]

    def values(self) -> np.ndarray:
        """float64 view of every point (longs converted like toDouble())."""
        d = self.bits.view(np.float64).copy()
        ints = self.is_int.astype(bool)
        d[ints] = self.bits[ints].view(np.int64).astype(np.float64)
        return d

    def __iter__(self):
        for i in range(len(self.ts)):
            if self.is_int[i]:
                yield DataPoint(int(self.ts[i]), True, self.longValue(i))
            else:
                yield DataPoint(int(self.ts[i]), False, self.doubleValue(i))

    def metricName(self) -> str:
        return self.metric


UNSET = -1
ROLLUP_USAGES = ("ROLLUP_RAW", "ROLLUP_NOFALLBACK", "ROLLUP_FALLBACK", "ROLLUP_FALLBACK_RAW")


class TsdbQuery:
    """Mirror of net.opentsdb.core.TsdbQuery for the aggregation path."""

    def __init__(self, store: MockStore, runner=None, rollups=None, rollup_runner=None, fix_duplicates=False):
        self.store = store
        self.runner = runner
        self.rollups = rollups              # rollup_read.RollupStore (tsdb.getRollupConfig() + tables)
        self.rollup_runner = rollup_runner  # (HostRollupBatch, Query) -> groups; libtsdbhip by default
        self.fix_duplicates = fix_duplicates
        self.start_time = UNSET
        self.end_time = UNSET
        self.metric = None
        self.tags = {}
        self.aggregator = None
        self.rate = False
        self.rate_options = RateOptions()
        self.downsampler: DownsamplingSpecification | None = None
        self.flags = 0
        self.rollup_usage = "ROLLUP_NOFALLBACK"   # TsdbQuery.java:150

    def setRollupUsage(self, usage: str | None):
        """TSSubQuery.setRollupUsage / ROLLUP_USAGE.parse (TsdbQuery.java:207-222): an unknown
        name means ROLLUP_NOFALLBACK."""
        u = (usage or "").upper()
        self.rollup_usage = u if u in ROLLUP_USAGES else "ROLLUP_NOFALLBACK"

    # TsdbQuery.java:262-319
    def setStartTime(self, timestamp: int):
        if timestamp < 0 or ((timestamp & SECOND_MASK) != 0 and timestamp > 9999999999999):
            raise ValueError(f"Invalid timestamp: {timestamp}")
        if self.end_time != UNSET and timestamp >= self.getEndTime():
            raise ValueError(f"new start time ({timestamp}) is greater than or equal to end time")
        self.start_time = timestamp

    def setEndTime(self, timestamp: int):
        if timestamp < 0 or ((timestamp & SECOND_MASK) != 0 and timestamp > 9999999999999):
            raise ValueError(f"Invalid timestamp: {timestamp}")
        if self.start_time != UNSET and timestamp <= self.getStartTime():
            raise ValueError(f"new end time ({timestamp}) is less than or equal to start time")
        self.end_time = timestamp

    def getStartTime(self) -> int:
        if self.start_time == UNSET:
            raise RuntimeError("IllegalStateException: setStartTime was never called!")
        return self.start_time

    def getEndTime(self) -> int:
        if self.end_time == UNSET:
            self.setEndTime(int(time.time() * 1000))
        return self.end_time

    def setTimeSeries(self, metric: str, tags: dict, function: str, rate: bool,
                      rate_options: RateOptions | None = None):
        if function not in abi.AGG:
            raise KeyError(f"No such aggregator: {function}")
        self.metric = metric
        self.tags = dict(tags)
        self.aggregator = function
        self.rate = rate
        self.rate_options = rate_options or RateOptions()

    def downsample(self, interval, function: str | None = None, fill_policy: str = "none"):
        """downsample(interval_ms, Aggregator[, FillPolicy]) or downsample("1m-avg")."""
        if isinstance(interval, str):
            self.downsampler = DownsamplingSpecification.parse(interval)
            return
        if function is None:
            raise ValueError("downsampling function cannot be null")
        if interval <= 0:
            raise ValueError(f"interval not > 0: {interval}")
        if function == "none":
            raise ValueError("cannot use the NONE aggregator for downsampling")
        self.downsampler = DownsamplingSpecification(interval=interval, function=function,
                                                     fill_policy=fill_policy)

    def setOrdered(self, ordered: bool = True):
        """Engine option: cross-series float reductions in SpanGroup index order."""
        self.flags = (self.flags | abi.QF_ORDERED) if ordered else (self.flags & ~abi.QF_ORDERED)

    # -- C ABI structs -----------------------------------------------------------
    def to_abi(self) -> abi.Query:
        ds = self.downsampler
        q = abi.new_query(
            self.getStartTime(), self.getEndTime(), self.aggregator,
            ds_function=abi.AGG[ds.function] if ds else -1,
            ds_interval_ms=ds.interval if ds else 0,
            ds_fill=abi.FILL_NAMES.index(ds.fill_policy) if ds else abi.FILL_NONE,
            ds_all=bool(ds and ds.run_all), rate=self.rate, counter=self.rate_options.counter,
            counter_max=self.rate_options.counter_max, reset_value=self.rate_options.reset_value,
            drop_resets=self.rate_options.drop_resets, flags=self.flags)
        if ds and ds.use_calendar:
            q.ds_calendar = ds.calendar_unit
            if ds.timezone is not None:
                abi.set_timezone(q, ds.timezone)
        return q

    def scan_bounds(self):
        """getScanStartTimeSeconds / getScanEndTimeSeconds (TsdbQuery.java:1506-1606)."""
        start = self.getStartTime()
        if start & SECOND_MASK:
            start //= 1000
        ds = self.downsampler
        aligned = start
        if ds and ds.interval > 0:
            aligned -= ((1000 * start) % ds.interval) // 1000
        s = aligned - aligned % 3600
        s = s if s > 0 else 0
        end = self.getEndTime()
        if end & SECOND_MASK:
            end //= 1000
            if end - end * 1000 < 1:
                end += 1
        if ds and ds.interval > 0:
            ia = end + (ds.interval - (1000 * end) % ds.interval) // 1000
            off = ia % 3600
            e = ia if off == 0 else ia + (3600 - off)
        else:
            e = end + (3600 - end % 3600)
        return s, e

    def rollup_interval_name(self):
        """transformDownSamplerToRollupQuery (TsdbQuery.java:1665-1700): the best-match rollup
        table of the downsampling interval, or None (a raw scan) -- also when the best match is
        the default interval, the raw table itself (:1694-1697)."""
        best = self._best_rollups()
        if not best or self.rollups.config.isDefaultInterval(best[0]):
            return None
        return best[0]

    def _filters(self):
        """Tag filters and group-by tag uids of setTimeSeries' tags (None: no series match)."""
        tagk_ids = self.store.tagk.ids
        tagv_ids = self.store.tagv.ids
        filters = []   # (tagk uid, allowed tagv uid set or None)
        group_bys = []
        for k, v in self.tags.items():
            if k not in tagk_ids:
                return None
            ku = tagk_ids[k]
            if v == "*":
                group_bys.append(ku)
                filters.append((ku, None))
            elif "|" in v:
                allowed = {tagv_ids[x] for x in v.split("|") if x in tagv_ids}
                group_bys.append(ku)
                filters.append((ku, allowed))
            else:
                if v not in tagv_ids:
                    return None
                filters.append((ku, {tagv_ids[v]}))
        group_bys.sort()

        def pred(tags):
            d = dict(tags)
            for ku, allowed in filters:
                if ku not in d:
                    return False
                if allowed is not None and d[ku] not in allowed:
                    return False
            return True
        return pred, group_bys

    @staticmethod
    def _groups(spans, group_bys):
        if not group_bys:
            return [()], [0] * len(spans)
        key_of = []
        for sk, _ in spans:
            d = dict(sk[1])
            key_of.append(tuple(d.get(ku, -1) for ku in group_bys))
        keys = sorted({k for k in key_of if -1 not in k})  # ByteMap order of the uid bytes
        index = {k: i for i, k in enumerate(keys)}
        return keys, [index.get(k, -1) for k in key_of]

    def build_rollup_batch(self, name: str):
        """The rollup scan of table `name` grouped like build_batch: (HostRollupBatch, keys)."""
        from .rollup_read import make_rollup_batch
        iv = self.rollups.config.intervals[name]
        f = self._filters()
        ds = self.downsampler
        if f is None:
            spans, need_count = [], False
        else:
            spans, need_count = self.rollups.scan_cells(name, self.metric, ds.function, self.aggregator, f[0])
        keys, gids = self._groups(spans, f[1] if f else [])
        return make_rollup_batch(spans, gids, iv, need_count, self.fix_duplicates), keys

    def build_batch(self):
        """findSpans + GroupByAndAggregateCB grouping (TsdbQuery.java:795-1049).
        Returns (HostBatch, group keys in emission order)."""
        s, e = self.scan_bounds()
        tagk_ids = self.store.tagk.ids
        tagv_ids = self.store.tagv.ids
        filters = []   # (tagk uid, allowed tagv uid set or None)
        group_bys = []
        for k, v in self.tags.items():
            if k not in tagk_ids:
                return make_batch([], []), []
            ku = tagk_ids[k]
            if v == "*":
                group_bys.append(ku)
                filters.append((ku, None))
            elif "|" in v:
                allowed = {tagv_ids[x] for x in v.split("|") if x in tagv_ids}
                group_bys.append(ku)
                filters.append((ku, allowed))
            else:
                if v not in tagv_ids:
                    return make_batch([], []), []
                filters.append((ku, {tagv_ids[v]}))
        group_bys.sort()

        def pred(tags):
            d = dict(tags)
            for ku, allowed in filters:
                if ku not in d:
                    return False
                if allowed is not None and d[ku] not in allowed:
                    return False
            return True

        spans = self.store.scan(self.metric, s, e, pred)
        if not group_bys:
            keys = [()]
            gids = [0] * len(spans)
        else:
            key_of = []
            for sk, _ in spans:
                d = dict(sk[1])
                key_of.append(tuple(d.get(ku, -1) for ku in group_bys))
            keys = sorted({k for k in key_of if -1 not in k})  # ByteMap order of the uid bytes
            index = {k: i for i, k in enumerate(keys)}
            gids = [index.get(k, -1) for k in key_of]
        return make_batch(spans, gids), keys

    def _best_rollups(self):
        """getRollupInterval's match list for the downsampling interval, best first ([] = none;
        ROLLUP_RAW never builds a rollup query, TsdbQuery.java:480-483)."""
        ds = self.downsampler
        if self.rollups is None or ds is None or ds.interval <= 0 or self.rollup_usage == "ROLLUP_RAW":
            return []
        from .rollup_read import NoSuchRollupForIntervalException
        try:
            return list(self.rollups.config.getRollupInterval(ds.interval // 1000))
        except NoSuchRollupForIntervalException:
            return []

    def _run_rollup(self, name):
        rb, keys = self.build_rollup_batch(name)
        q = self.to_abi()
        runner = self.rollup_runner
        if runner is None:
            from .engine import default_engine
            runner = default_engine().run_rollup_batch
        if rb.cells.n_series == 0:
            return []
        out = []
        for gid, ts, bits, isi in runner(rb, q):
            key = keys[gid] if (self.aggregator != "none" and 0 <= gid < len(keys)) else ()
            out.append(DataPoints(gid, ts, bits, isi, self.metric, key))
        return out

    def _run_raw(self, aggregator_override):
        batch, keys = self.build_batch()
        q = self.to_abi()
        if aggregator_override:
            q.aggregator = abi.AGG[aggregator_override]
        runner = self.runner
        if runner is None:
            from .engine import default_engine
            runner = default_engine().run_batch
        if batch.n_series == 0:
            return []
        groups = runner(batch, q)
        out = []
        for gid, ts, bits, isi in groups:
            key = keys[gid] if (self.aggregator != "none" and 0 <= gid < len(keys)) else ()
            out.append(DataPoints(gid, ts, bits, isi, self.metric, key))
        return out

    def _rollup_to_downsampler(self, name):
        """transformRollupQueryToDownSampler (TsdbQuery.java:1706-1717): the raw scan downsamples
        at the failed rollup table's interval with the rollup aggregator (zimsum / mimmax /
        mimmin read as sum / max / min, RollupQuery.java:69-80)."""
        from .rollup_read import normalize_agg
        ds = self.downsampler
        self.downsampler = DownsamplingSpecification(
            interval=self.rollups.config.intervals[name].interval_s * 1000,
            function=normalize_agg(ds.function), fill_policy=ds.fill_policy if ds else "zero")

    def run(self):
        """TsdbQuery.run(): DataPoints[] of the query (one per SpanGroup).  With a rollup config
        the downsampler becomes a rollup query on the best-match table
        (transformDownSamplerToRollupQuery, :1665-1700; a count group-by turns into sum there);
        the default interval is the raw table.  Under ROLLUP_FALLBACK / ROLLUP_FALLBACK_RAW an
        empty result re-runs on the next best match or on raw data
        (FallbackRollupOnEmptyResult, :1293-1354).  The query's downsampler is restored after."""
        best = self._best_rollups()
        if not best:
            return self._run_raw(None)
        override = "sum" if self.aggregator == "count" else None
        cur = best.pop(0)
        if self.rollups.config.isDefaultInterval(cur):
            return self._run_raw(override)
        saved = self.downsampler
        try:
            while True:
                out = self._run_rollup(cur)
                if out or self.rollup_usage not in ("ROLLUP_FALLBACK", "ROLLUP_FALLBACK_RAW"):
                    return out
                if self.rollup_usage == "ROLLUP_FALLBACK_RAW":
                    self._rollup_to_downsampler(cur)
                    return self._run_raw(override)
                if not best:
                    return []
                nxt = best.pop(0)
                if self.rollups.config.isDefaultInterval(nxt):
                    self._rollup_to_downsampler(cur)
                    return self._run_raw(override)
                # (the next table's interval divides the sample interval: the downsampler keeps
                # its interval, :1331-1340)
                cur = nxt
        finally:
            self.downsampler = saved
