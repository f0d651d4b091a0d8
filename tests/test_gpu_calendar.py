"""GPU parity of calendar ('c') downsampling in UTC:
DateTime.previousInterval / the calendar Downsampler and FillingDownsampler
(src/utils/DateTime.java:445-606, src/core/Downsampler.java:131-147,336-432,
src/core/FillingDownsampler.java:113-135,280-286).  The oracle's calendar arithmetic is
pinned by tests/golden/calendar.json (TestDownsampler's UTC cases); here the engine is
checked against the oracle on multi-series stores.  Intervals whose UTC grid is one global
sequence run on the fixed grid (ms / s / m / h dividing their unit, 1d, 1w) or a boundary
table (n months with 12 % n == 0, 1 year); intervals anchored per span run on the union table
of the spans' anchors when those agree (tests/test_gpu_calendar_tz.py covers time zones and
disagreeing anchors)."""
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


@pytest.mark.parametrize("spec", ["1dc-sum-nan", "1hc-avg-zero", "15mc-max-null", "1dc-count-zero", "1wc-sum-nan",
                                  "1wc-avg-zero"])
def test_calendar_fill(eng, week_batch, spec):
    q = q_of(spec, T0 + 3 * 86400, T0 + 10 * 86400 - 1, "sum")
    assert_groups_match(eng.run_batch(week_batch, q), O.run_query(week_batch, q), "sum", ctx=spec)


def test_calendar_rate(eng, hour_batch, week_batch):
    q = q_of("5mc-avg", T0, T0 + 3599, "sum")
    q.rate = 1
    assert_groups_match(eng.run_batch(hour_batch, q), O.run_query(hour_batch, q), "sum", ctx="rate")
    for spec in ["1wc-avg-zero", "1wc-sum-nan", "1dc-max-zero"]:   # leading filled week feeds the first rate
        q = q_of(spec, T0 + 3 * 86400, T0 + 20 * 86400 - 1, "sum")
        q.rate = 1
        assert_groups_match(eng.run_batch(week_batch, q), O.run_query(week_batch, q), "sum", ctx=f"rate {spec}")


@pytest.fixture(scope="module")
def year_batch():
    # 14 months @6 h from 2012-12-01 (leap-year February 2012 is before; 2013 is not leap)
    return synth.generate(12, T0 - 31 * 86400, 14 * 30 * 4, 6 * 3600000, value_kind=2, n_groups=2, int_mod=1000,
                          seed=8)


@pytest.mark.parametrize("spec", ["1nc-sum", "1nc-avg", "2nc-max", "3nc-count", "6nc-sum", "1yc-sum", "1nc-dev",
                                  "1nc-sum-nan", "1nc-avg-zero"])
@pytest.mark.parametrize("agg", ["sum", "p90", "min"])
def test_calendar_months_years(eng, year_batch, spec, agg):
    q = q_of(spec, T0 - 31 * 86400, T0 + 400 * 86400, agg)
    assert_groups_match(eng.run_batch(year_batch, q), O.run_query(year_batch, q), agg, ctx=f"{spec} {agg}")


def test_calendar_months_rate(eng, year_batch):
    q = q_of("1nc-avg", T0 - 31 * 86400, T0 + 400 * 86400, "sum")
    q.rate = 1
    assert_groups_match(eng.run_batch(year_batch, q), O.run_query(year_batch, q), "sum", ctx="rate")


@pytest.mark.parametrize("spec", ["7sc-sum", "2wc-sum", "2dc-sum", "5nc-sum", "2yc-sum", "7mc-avg", "5hc-max"])
def test_calendar_anchored_per_span(eng, hour_batch, spec):
    # every span's first datapoint is T0: one anchor, one grid (engine.cpp plan_calendar)
    q = q_of(spec, T0, T0 + 3599, "sum")
    assert_groups_match(eng.run_batch(hour_batch, q), O.run_query(hour_batch, q), "sum", ctx=spec)


@pytest.mark.parametrize("spec", ["1nc-p99", "1wc-p99-nan"])
def test_calendar_pct_over_table(eng, hour_batch, spec):
    """Percentile downsampling over a calendar slot table (k_pct's MODE_TABLE slot lookup)."""
    q = q_of(spec, T0, T0 + 3599, "sum")
    assert_groups_match(eng.run_batch(hour_batch, q), O.run_query(hour_batch, q), "sum", ctx=spec)
