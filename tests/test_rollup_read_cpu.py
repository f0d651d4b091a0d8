"""Rollup read path on the CPU: the oracle's RollupSpan / RollupSeq /
Downsampler restatement pinned by the known answers of test/core/TestTsdbQueryRollup.java
(tests/golden/rollup_queries.json, transcribed by tests/golden/make_rollup_query_golden.py),
the host scan mirror (opentsdb_amd/rollup_read.py) and the RollupSeq corner cases the
reference's code defines (sync, duplicates, seek in lock step)."""
import ctypes as C
import struct

import numpy as np
import pytest

from opentsdb_amd import abi, engine
from opentsdb_amd.query import QueryException
from opentsdb_amd.rollup_read import make_rollup_batch
from oracle import oracle as O
from tests import golden_util as gu

DOC = gu.load("rollup_queries.json")
CASES = {c["name"]: c for c in DOC["cases"]}


def oracle_runners():
    def raw(batch, q):
        return O.run_query(batch, q)

    def rollup(rb, q):
        return O.run_rollup_query(rb, q)
    return raw, rollup


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_known_answers(name):
    case = CASES[name]
    exp = case["expect"]
    if "write_error" in exp:
        with pytest.raises(ValueError):
            gu.rollup_stores(DOC, case)
        return
    q = gu.rollup_query(DOC, case, *oracle_runners())
    if "error" in exp:
        with pytest.raises(O.OracleError) as e:
            q.run()
        assert abi.ERROR_NAMES[e.value.code] == exp["error"]
        return
    gu.check_rollup_expect(case, q.run())


def test_every_test_method_transcribed():
    import os
    src = "/root/reference/test/core/TestTsdbQueryRollup.java"
    if not os.path.exists(src):
        pytest.skip("reference absent")
    import re
    names = set(re.findall(r"public void (\w+)\(\) throws", open(src).read())) - {"beforeLocal"}
    assert names <= set(CASES), names - set(CASES)


def test_table_choice():
    """RollupConfig.getRollupInterval: exact match or the largest dividing interval."""
    raw, rs = gu.rollup_stores(DOC, CASES["run10mSumLongSingleTS"])
    cfg = rs.config
    assert cfg.getRollupInterval(600) == ["10m"]
    assert cfg.getRollupInterval(1800) == ["10m"]
    assert cfg.getRollupInterval(7200) == ["1h", "10m"]
    from opentsdb_amd.rollup_read import NoSuchRollupForIntervalException
    with pytest.raises(NoSuchRollupForIntervalException):
        cfg.getRollupInterval(900)


def _iv():
    return engine.rollup_interval("10m", "6h")


def _batch(rows, counts=True, fix=False, groups=None):
    """rows: per series [(base, [(off, flags, bytes)], [(off, flags, bytes)])]."""
    spans = []
    for s in rows:
        rr = []
        for base, vals, cnts in s:
            rr.append((base, [(struct.pack(">H", (o << 4) | f), v) for o, f, v in vals],
                       [(struct.pack(">H", (o << 4) | f), v) for o, f, v in cnts]))
        spans.append((None, rr))
    return make_rollup_batch(spans, groups or [0] * len(spans), _iv(), counts, fix)


def _l(v):
    return (0x7, struct.pack(">q", v))


def _q(ds="10m-avg", agg="avg", start=1356998400, end=1357041600, rate=False):
    q = abi.new_query(start, end, agg, rate=rate)
    assert O.lib().ref_parse_downsample(ds.encode(), C.byref(q)) == 0
    return q


def _pts(groups):
    return [[(int(t), float(np.array([b], np.uint64).view(np.float64)[0])) for t, b in zip(ts, bits)]
            for _, ts, bits, _ in groups]


B = 1356998400


def test_sync_skips_unpaired_cells():
    """RollupIterator.sync: only offsets present in both streams are datapoints."""
    rb = _batch([[(B, [(0, *_l(20)), (1, *_l(40)), (3, *_l(60))], [(0, *_l(2)), (2, *_l(9)), (3, *_l(3))])]])
    assert _pts(O.run_rollup_query(rb, _q())) == [[(B * 1000, 10.0), ((B + 1800) * 1000, 20.0)]]


def test_count_downsampling_sums_counts():
    rb = _batch([[(B, [(0, *_l(20)), (1, *_l(40))], [(0, *_l(2)), (1, *_l(5))])]])
    assert _pts(O.run_rollup_query(rb, _q("20m-count", "avg"))) == [[(B * 1000, 7.0)]]
    # without count cells valueCount() is 1
    rb = _batch([[(B, [(0, *_l(20)), (1, *_l(40))], [])]], counts=False)
    assert _pts(O.run_rollup_query(rb, _q("20m-count", "sum"))) == [[(B * 1000, 2.0)]]


def test_avg_zero_count_is_zero():
    rb = _batch([[(B, [(0, *_l(20))], [(0, *_l(0))])]])
    assert _pts(O.run_rollup_query(rb, _q())) == [[(B * 1000, 0.0)]]


def test_offsets_must_increase():
    rb = _batch([[(B, [(2, *_l(1)), (1, *_l(2))], [])]], counts=False)
    with pytest.raises(O.OracleError) as e:
        O.run_rollup_query(rb, _q("10m-sum", "sum"))
    assert e.value.code == abi.TSDB_E_ILLEGAL_DATA
    rb = _batch([[(B, [(1, *_l(1)), (2, *_l(2))], [(2, *_l(1)), (1, *_l(2))])]])
    with pytest.raises(O.OracleError) as e:
        O.run_rollup_query(rb, _q())
    assert e.value.code == abi.TSDB_E_ILLEGAL_ARGUMENT


def test_duplicate_offsets_keep_the_later_cell():
    rb = _batch([[(B, [(1, *_l(1)), (1, *_l(7))], [])]], counts=False, fix=True)
    assert _pts(O.run_rollup_query(rb, _q("10m-sum", "sum"))) == [[((B + 600) * 1000, 7.0)]]


def test_dev_downsampling_unsupported():
    rb = _batch([[(B, [(0, *_l(20))], [(0, *_l(2))])]])
    with pytest.raises(O.OracleError) as e:
        O.run_rollup_query(rb, _q("10m-dev", "avg"))
    assert e.value.code == abi.TSDB_E_UNSUPPORTED


def test_rollup_query_needs_downsampling():
    rb = _batch([[(B, [(0, *_l(20))], [])]], counts=False)
    q = abi.new_query(B, B + 3600, "sum")
    with pytest.raises(O.OracleError):
        O.run_rollup_query(rb, q)


def test_rollup_scan_bounds():
    """getScanStart/EndTimeSeconds with a RollupQuery (TsdbQuery.java:1515-1526,1562-1567)."""
    iv = _iv()
    q = _q("10m-sum", "sum", start=1357000000, end=1357041600)
    assert O.rollup_scan_bounds(q, iv) == (1356998400, engine.rollup_basetime(1357041600 + 600 * 36, iv))
    assert O.rollup_scan_bounds(q, iv) == (1356998400, 1357063200)
    q = _q("10m-sum", "sum", start=1357000000, end=1357041600, rate=True)
    assert O.rollup_scan_bounds(q, iv)[0] == 1356998400 - 21600
