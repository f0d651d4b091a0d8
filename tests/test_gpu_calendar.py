"""GPU parity of calendar ('c') downsampling in UTC:
DateTime.previousInterval / the calendar Downsampler and FillingDownsampler
(src/utils/DateTime.java:445-606, src/core/Downsampler.java:131-147,336-432,
src/core/FillingDownsampler.java:113-135,280-286).  The oracle's calendar arithmetic is
pinned by tests/golden/calendar.json (TestDownsampler's UTC cases); here the engine is
checked against the oracle on multi-series stores.  The engine takes the intervals whose
UTC grid is one global sequence (ms / s / m / h dividing their unit, 1d, 1w) and refuses
months, years and per-span anchored intervals with NOT_IMPLEMENTED."""
from __future__ import annotations

import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import parse_downsample
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400          # 2013-01-01 00:00 UTC (a Tuesday)


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def week_batch():
    # 3 weeks @10 min, series starting 5 h apart, mixed int / float
    return synth.generate(24, T0 + 3 * 86400, 3 * 7 * 144, 600000, value_kind=2, n_groups=3, int_mod=1000, seed=2)


@pytest.fixture(scope="module")
def hour_batch():
    return synth.generate(30, T0, 720, 5000, value_kind=2, n_groups=4, int_mod=30000, seed=4)


def q_of(spec, start, end, agg):
    q = abi.new_query(start, end, agg)
    p = parse_downsample(spec)
    for f in ("ds_function", "ds_fill", "ds_all", "ds_calendar", "ds_interval_ms"):
        setattr(q, f, getattr(p, f))
    return q


@pytest.mark.parametrize("spec", ["1mc-avg", "5mc-sum", "15mc-max", "30sc-avg", "1hc-sum", "20sc-min", "500msc-count",
                                  "1mc-p99", "10mc-dev"])
@pytest.mark.parametrize("agg", ["sum", "max", "avg"])
def test_calendar_small_units(eng, hour_batch, spec, agg):
    q = q_of(spec, T0, T0 + 3599, agg)
    assert_groups_match(eng.run_batch(hour_batch, q), O.run_query(hour_batch, q), agg, ctx=spec)


@pytest.mark.parametrize("spec", ["1dc-sum", "1wc-sum", "1wc-avg", "6hc-max", "1dc-p50", "1wc-count"])
def test_calendar_days_weeks(eng, week_batch, spec):
    q = q_of(spec, T0 + 3 * 86400, T0 + 24 * 86400, "sum")
    assert_groups_match(eng.run_batch(week_batch, q), O.run_query(week_batch, q), "sum", ctx=spec)


@pytest.mark.parametrize("spec", ["1dc-sum-nan", "1hc-avg-zero", "15mc-max-null", "1dc-count-zero"])
def test_calendar_fill(eng, week_batch, spec):
    q = q_of(spec, T0 + 3 * 86400, T0 + 10 * 86400 - 1, "sum")
    assert_groups_match(eng.run_batch(week_batch, q), O.run_query(week_batch, q), "sum", ctx=spec)


def test_calendar_rate(eng, hour_batch):
    q = q_of("5mc-avg", T0, T0 + 3599, "sum")
    q.rate = 1
    assert_groups_match(eng.run_batch(hour_batch, q), O.run_query(hour_batch, q), "sum", ctx="rate")


@pytest.mark.parametrize("spec", ["1nc-sum", "1yc-sum", "7sc-sum", "2wc-sum", "2dc-sum"])
def test_calendar_without_global_grid_not_implemented(eng, hour_batch, spec):
    q = q_of(spec, T0, T0 + 3599, "sum")
    with pytest.raises(Exception) as ei:
        eng.run_batch(hour_batch, q)
    assert "NotImplemented" in str(ei.value)
