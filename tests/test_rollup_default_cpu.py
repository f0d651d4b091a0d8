"""transformDownSamplerToRollupQuery's default interval (src/core/TsdbQuery.java:1665-1700): a best
match that is the default interval (the raw table, RollupInterval.isDefaultInterval) drops the
rollup query -- a raw scan -- but a count group-by was already turned into sum (:1681-1683).
RollupConfig allows one default interval (src/rollup/RollupConfig.java:93-103).  No reference
test covers the default interval on the query path: these cases restate that code, unpinned."""
from __future__ import annotations

import pytest

from opentsdb_amd import abi
from opentsdb_amd.query import TsdbQuery
from opentsdb_amd.rollup_read import RollupConfig, RollupStore
from opentsdb_amd.store import MockStore

T0 = 1356998400
IDS = {"sum": 1, "count": 2, "max": 3, "min": 4}


def make(intervals):
    st = MockStore()
    for i in range(10):
        st.add_long("sys.cpu", T0 + i * 60, i, {"host": "a"})
    rs = RollupStore(RollupConfig(IDS, intervals), st)
    for iv in intervals:
        if len(iv) < 3:
            for agg in ("sum", "count"):
                rs.add_aggregate_point("sys.cpu", T0, 5, {"host": "a"}, iv[0], agg)
    return st, rs


def query(st, rs, agg, seen):
    def runner(batch, q):
        seen.append((q.aggregator, "raw"))
        return []

    def rollup_runner(rb, q):
        seen.append((q.aggregator, "rollup"))
        return []

    q = TsdbQuery(st, runner=runner, rollups=rs, rollup_runner=rollup_runner)
    q.setStartTime(T0)
    q.setEndTime(T0 + 3600)
    q.setTimeSeries("sys.cpu", {"host": "*"}, agg, False)
    q.downsample("10m-sum")
    return q


def test_default_interval_is_a_raw_scan():
    st, rs = make([("1m", "1h", True), ("10m", "1d")])
    seen = []
    query(st, rs, "sum", seen).run()
    assert seen == [(abi.AGG["sum"], "rollup")]   # 10m matches exactly: the rollup table
    st, rs = make([("1m", "1h", True), ("1h", "1d")])
    seen = []
    q = query(st, rs, "sum", seen)
    assert q.rollup_interval_name() is None       # best match 1m is the default interval
    q.run()
    assert seen == [(abi.AGG["sum"], "raw")]


def test_count_on_the_default_interval_scans_raw_with_sum():
    st, rs = make([("1m", "1h", True)])
    seen = []
    query(st, rs, "count", seen).run()
    assert seen == [(abi.AGG["sum"], "raw")]
    st, rs = make([("1m", "1h")])                  # not the default: a rollup query (count -> sum there)
    seen = []
    query(st, rs, "count", seen).run()
    assert seen == [(abi.AGG["count"], "rollup")]


def test_one_default_interval_only():
    with pytest.raises(ValueError, match="Multiple default intervals"):
        RollupConfig(IDS, [("1m", "1h", True), ("1h", "1d", True)])
    with pytest.raises(ValueError, match="Only one interval of each type"):
        RollupConfig(IDS, [("1m", "1h"), ("1m", "1d")])
