"""Cells of one series with the same base time (salt-bucket duplicates) merge like
Span.addRow / RowSeq.addRow (src/core/Span.java:177-220, src/core/RowSeq.java:91-222; SURVEY.md
8a row a4): ordered merge by qualifier offset, the later cell's duplicate timestamps dropped.
The engine merges at load; the oracle restates the reference's addRow (pinned by
TestRowSeq's addRowMerge* known answers in test_oracle_golden.py)."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def dup_batch(seed, n_series=24, n_groups=3, single=False):
    """Each series' points split into two overlapping subsets, each encoded as its own cells
    (two cells per hour); the overlap repeats some timestamps with different values."""
    rng = np.random.default_rng(seed)
    series, gids = [], []
    for s in range(n_series):
        t = np.sort(rng.choice(np.arange(0, 7200), size=int(rng.integers(4, 300)), replace=False))
        pick = rng.random(len(t))
        a = t[pick < 0.6]
        b = t[pick > 0.3]   # 0.3 < pick < 0.6: in both cells
        rows = []
        for part, off in ((a, 0), (b, 1000)):
            if single:
                part = part[:1]
            if len(part) == 0:
                continue
            ts = T0 * 1000 + part * 1000
            kind = np.full(len(part), 0 if s % 2 == 0 else 2)
            lv = rng.integers(-1000, 1000, len(part)) + off
            fv = rng.normal(50, 10, len(part)) + off
            rows += synth.encode_rows(ts, lv, fv, kind, np.zeros(len(part), bool))
        series.append(rows)
        gids.append(s % n_groups)
    order = sorted(range(n_series), key=lambda i: gids[i])
    return synth.from_series([series[i] for i in order], [gids[i] for i in order])


@pytest.mark.parametrize("agg", ["sum", "max", "min", "count", "avg"])
def test_merged_cells_downsampled(eng, agg):
    b = dup_batch(1)
    q = abi.new_query(T0, T0 + 7199, agg, ds_function=abi.AGG["sum"], ds_interval_ms=60000)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, ctx=agg)


@pytest.mark.parametrize("agg", ["sum", "max", "first", "last"])
def test_merged_cells_raw(eng, agg):
    b = dup_batch(2)
    q = abi.new_query(T0, T0 + 7199, agg)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, tol=0.0, ctx=agg)


def test_merged_single_datapoint_cells(eng):
    b = dup_batch(3, single=True)
    for agg in ["sum", "count"]:
        q = abi.new_query(T0, T0 + 7199, agg, ds_function=abi.AGG["max"], ds_interval_ms=600000)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, ctx=agg)
