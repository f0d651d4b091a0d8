"""GPU parity of rollup generation (tsdbhip_rollup_run) against the
CPU restatement oracle/rollup.generate: every cell -- series, row base time, the 3-byte
qualifier [agg id][BE16 offset<<4|flags] and the value bytes -- must be byte-identical.
The codec itself is pinned by tests/test_rollup_cpu.py (reference known answers)."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from oracle import rollup as R

pytestmark = pytest.mark.gpu

T0 = 1356998400
FUNCS = (("sum", 0), ("count", 1), ("max", 2), ("min", 3))


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def engine_cells(eng, batch, interval, span, start, end, funcs=FUNCS):
    from opentsdb_amd import engine
    eng.load(batch)
    cells = eng.rollup(engine.rollup_interval(interval, span), start, end, funcs)
    return [cells.cell(i) for i in range(len(cells))]


def check(eng, batch, interval, span, start, end, funcs=FUNCS):
    exp = R.generate(batch, R.Interval(interval, span), start, end, funcs)
    got = engine_cells(eng, batch, interval, span, start, end, funcs)
    assert len(got) == len(exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g == e, (i, g, e)
    return got


@pytest.mark.parametrize("interval,span", [("1h", "1d"), ("1d", "1n"), ("10m", "1d"), ("6h", "1y"), ("10m", "2h")])
def test_rollup_config1_shape(eng, interval, span):
    # 40 series x 1 day @10 s; even series vle ints, odd series float32 (configs 3 / 5 mix)
    b = synth.generate(40, T0, 8640, 10000, value_kind=2, n_groups=4, int_mod=30000)
    got = check(eng, b, interval, span, T0, T0 + 86400)
    assert got


def test_rollup_partial_range(eng):
    b = synth.generate(10, T0, 8640, 10000, value_kind=2, n_groups=2)
    check(eng, b, "1h", "1d", T0 + 3 * 3600 + 1200, T0 + 9 * 3600)


def test_rollup_function_subset_and_ids(eng):
    b = synth.generate(8, T0, 2000, 10000, value_kind=0)
    check(eng, b, "1h", "1d", T0, T0 + 86400, (("min", 7), ("sum", 42)))


def rows_mixed(seed):
    rng = np.random.default_rng(seed)
    series, gids = [], []
    for s in range(12):
        n = int(rng.integers(1, 400))
        ts = np.sort(rng.choice(np.arange(0, 2 * 86400 * 1000, 250), n, replace=False)) + T0 * 1000
        ms = (ts % 1000) != 0
        if s % 3 == 0:   # ints of every vle width, negative too
            kind = np.zeros(n, np.int64)
            lv = rng.integers(-(1 << 40), 1 << 40, n) >> rng.integers(0, 40, n)
            fv = np.zeros(n)
        elif s % 3 == 1:   # float64 values that do not fit a float32
            kind = np.full(n, 2)
            lv = np.zeros(n, np.int64)
            fv = rng.normal(0, 1e6, n)
        else:   # mixed int / float32 / float64 points
            kind = rng.integers(0, 3, n)
            lv = rng.integers(-1000, 1000, n)
            fv = np.round(rng.normal(0, 100, n), 2)
        series.append(synth.encode_rows(ts, lv, fv, kind, ms))
        gids.append(-1 if s == 5 else s % 4)
    return synth.from_series(series, gids)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("interval,span", [("1h", "1d"), ("15m", "1d"), ("1d", "1n")])
def test_rollup_mixed_rows(eng, seed, interval, span):
    check(eng, rows_mixed(seed), interval, span, T0, T0 + 2 * 86400)


def test_rollup_month_boundaries(eng):
    # daily rollups in monthly rows across Feb of a leap year and a year end
    starts = [1330473600 - 5 * 86400, 1356998400 - 3 * 86400]   # 2012-02-24, 2012-12-29
    series = []
    for st in starts:
        ts = (st + np.arange(0, 10 * 86400, 3600)) * 1000
        series.append(synth.encode_rows(ts, np.arange(len(ts)), None, np.zeros(len(ts), int), np.zeros(len(ts), bool)))
    b = synth.from_series(series, [0, 1])
    got = check(eng, b, "1d", "1n", starts[0], starts[1] + 10 * 86400)
    assert len({c[1] for c in got}) >= 4


def test_rollup_infinite_sum_rejected(eng):
    """addAggregatePoint(double) rejects an infinite value (src/core/TSDB.java:1426-1428)."""
    from opentsdb_amd import engine
    ts = (T0 + np.arange(0, 7200, 60)) * 1000
    fv = np.full(len(ts), 1.5e308)
    b = synth.from_series([synth.encode_rows(ts, None, fv, np.full(len(ts), 2), np.zeros(len(ts), bool))], [0])
    with pytest.raises(R.RollupError):
        R.generate(b, R.Interval("1h", "1d"), T0, T0 + 7200, (("sum", 0),))
    eng.load(b)
    with pytest.raises(engine.EngineError) as ei:
        eng.rollup(engine.rollup_interval("1h", "1d"), T0, T0 + 7200, (("sum", 0),))
    assert ei.value.java == "IllegalArgumentException"


def test_rollup_count_property_device_synth(eng):
    """Size-independent property at a larger size: the count cells of a 1h rollup add up to
    the datapoints of the window, and every series contributes its 24 buckets."""
    from opentsdb_amd import engine
    n = 200_000
    eng.synth(n, T0, 8640, 10000, value_kind=2, n_groups=1000, int_mod=30000)
    nc, nb = eng.rollup_run(engine.rollup_interval("1h", "1d"), T0, T0 + 86400, (("count", 1),))
    cells = eng.rollup_download(nc, nb)
    assert nc == n * 24
    # 360 points per bucket: vle 2-byte longs 0x0168
    assert np.all(cells.val_off[1:] - cells.val_off[:-1] == 2)
    v = cells.value.reshape(-1, 2)
    assert np.all((v[:, 0].astype(int) << 8 | v[:, 1]) == 360)
    assert np.all(cells.qualifier[:, 0] == 1)
    offs = (cells.qualifier[:, 1].astype(int) << 8 | cells.qualifier[:, 2]) >> 4
    np.testing.assert_array_equal(offs.reshape(n, 24), np.tile(np.arange(24), (n, 1)))
    np.testing.assert_array_equal(cells.series.reshape(n, 24)[:, 0], np.arange(n))
