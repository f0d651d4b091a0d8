"""GPU parity of calendar downsampling in a time zone and of intervals anchored per span
(SURVEY.md 8f row f3): DateTime.previousInterval in the query's zone and the calendar
Downsampler / FillingDownsampler (src/utils/DateTime.java:445-606,
src/core/Downsampler.java:131-147,336-432, src/core/FillingDownsampler.java:113-135).  The
oracle's zone-aware Calendar is pinned by the EST / America/Denver / Pacific/Funafuti /
Asia/Kabul / Pacific/Fiji cases of TestDownsampler and TestFillingDownsampler
(tests/golden/calendar.json, tests/test_oracle_golden.py); here the engine (engine.cpp
plan_calendar + the MODE_TABLE kernels) is checked against the oracle on multi-series stores
whose ranges cross daylight-saving transitions.  Zone tables come from opentsdb_amd.tz."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import parse_downsample
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

# 2016-01-10 .. 2016-03-20: Fiji leaves DST on Jan 17, Denver enters it on Mar 13
TA = 1452384000
ZONES = ["EST", "America/Denver", "Asia/Kabul", "Pacific/Funafuti", "Pacific/Fiji"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def merge(*batches):
    """Batches concatenated series-wise and regrouped (series in group order, as SpanCmp /
    the group-by keys order them)."""
    series = []
    for b in batches:
        for s in range(b.n_series):
            r0, r1 = int(b.series_row_ptr[s]), int(b.series_row_ptr[s + 1])
            rows = []
            for r in range(r0, r1):
                q = b.qual[int(b.row_qual_off[r]):int(b.row_qual_off[r + 1])].tobytes()
                v = b.val[int(b.row_val_off[r]):int(b.row_val_off[r + 1])].tobytes()
                rows.append((int(b.row_base_time[r]), q, v))
            series.append((int(b.group_id[s]), rows))
    series.sort(key=lambda x: x[0])
    srp, base, qo, vo, qual, val, gid = [0], [], [0], [0], bytearray(), bytearray(), []
    for g, rows in series:
        for bt, q, v in rows:
            base.append(bt)
            qual += q
            val += v
            qo.append(len(qual))
            vo.append(len(val))
        srp.append(len(base))
        gid.append(g)
    return abi.HostBatch(srp, base, qo, vo, np.frombuffer(bytes(qual), np.uint8), np.frombuffer(bytes(val), np.uint8),
                         gid)


@pytest.fixture(scope="module")
def dst_batch():
    # 10 series x 70 days @20 min, mixed int / float, 3 groups
    return synth.generate(10, TA, 70 * 72, 1200000, value_kind=2, n_groups=3, int_mod=5000, seed=11)


def q_of(spec, start, end, agg, tz):
    q = abi.new_query(start, end, agg, tz=tz)
    p = parse_downsample(spec)
    for f in ("ds_function", "ds_fill", "ds_all", "ds_calendar", "ds_interval_ms"):
        setattr(q, f, getattr(p, f))
    return q


def check(eng, batch, q, agg, ctx):
    assert_groups_match(eng.run_batch(batch, q), O.run_query(batch, q), agg, ctx=ctx)


@pytest.mark.parametrize("tz", ZONES)
@pytest.mark.parametrize("spec", ["1dc-sum", "1wc-avg", "1nc-sum", "1hc-max", "30mc-avg", "1yc-count", "6hc-sum",
                                  "2dc-min", "3nc-sum"])
def test_tz_query(eng, dst_batch, tz, spec):
    q = q_of(spec, TA + 2 * 86400 + 1234, TA + 66 * 86400, "sum", tz)
    check(eng, dst_batch, q, "sum", f"{tz} {spec}")


@pytest.mark.parametrize("tz", ["America/Denver", "Pacific/Fiji", "Asia/Kabul"])
@pytest.mark.parametrize("agg", ["avg", "max", "p90", "none", "dev"])
def test_tz_aggregators(eng, dst_batch, tz, agg):
    q = q_of("1dc-avg", TA + 86400, TA + 60 * 86400, agg, tz)
    check(eng, dst_batch, q, agg, f"{tz} {agg}")


@pytest.mark.parametrize("tz", ZONES)
@pytest.mark.parametrize("spec", ["1dc-sum-nan", "1wc-avg-zero", "1hc-sum-null", "1nc-max-nan"])
def test_tz_fill(eng, dst_batch, tz, spec):
    q = q_of(spec, TA + 3 * 86400 + 500, TA + 40 * 86400 - 1, "sum", tz)
    check(eng, dst_batch, q, "sum", f"{tz} {spec}")


@pytest.mark.parametrize("tz", ["America/Denver", "Pacific/Fiji"])
def test_tz_rate(eng, dst_batch, tz):
    q = q_of("1dc-avg", TA + 86400, TA + 60 * 86400, "sum", tz)
    q.rate = 1
    check(eng, dst_batch, q, "sum", f"{tz} rate")


def test_tz_utc_table_equals_utc(eng, dst_batch):
    # a zone without transitions at offset 0 gives the UTC answers
    from opentsdb_amd import tz as T
    for spec in ["1dc-sum", "1wc-avg", "1nc-sum"]:
        q0 = q_of(spec, TA + 86400, TA + 60 * 86400, "sum", None)
        q1 = q_of(spec, TA + 86400, TA + 60 * 86400, "sum", T.fixed("UTC0", 0))
        a, b = eng.run_batch(dst_batch, q0), eng.run_batch(dst_batch, q1)
        assert_groups_match(a, b, "sum", ctx=spec)


@pytest.fixture(scope="module")
def staggered():
    """Spans whose first datapoints lie in different hours: 7sc anchors each span at the top of
    its first hour and 3600 % 7 != 0, so the spans sit on different 7 s grids."""
    T0 = 1356998400
    return merge(synth.generate(3, T0, 720, 5000, value_kind=2, n_groups=2, int_mod=900, seed=1),
                 synth.generate(2, T0 + 3600 + 1234, 700, 5000, value_kind=0, n_groups=2, seed=2),
                 synth.generate(3, T0 + 2 * 3600 + 17, 500, 7000, value_kind=1, n_groups=2, int_mod=300, seed=5))


@pytest.mark.parametrize("agg", ["sum", "avg", "min", "max", "dev", "count", "zimsum", "mimmax", "first", "last",
                                 "p90", "median", "none"])
def test_anchors_disagree_union_evaluation(eng, staggered, agg):
    """Per-span grids that disagree: each span's Downsampler output, aggregated over the union
    of their timestamps (run_anchored -> the raw union evaluator)."""
    T0 = 1356998400
    for spec in ["7sc-sum", "11sc-avg", "7sc-max"]:
        q = q_of(spec, T0, T0 + 3 * 3600, agg, None)
        check(eng, staggered, q, agg, f"anchored {spec} {agg}")


def test_anchors_disagree_rate_percentile_zone(eng, staggered):
    T0 = 1356998400
    q = q_of("7sc-avg", T0, T0 + 3 * 3600, "sum", None)
    q.rate = 1
    check(eng, staggered, q, "sum", "anchored rate")
    q = q_of("13sc-p95", T0 + 100, T0 + 3 * 3600 - 50, "sum", None)
    check(eng, staggered, q, "sum", "anchored p95 downsampling")
    q = q_of("7sc-sum", T0, T0 + 3 * 3600, "sum", "Asia/Kabul")
    check(eng, staggered, q, "sum", "anchored Kabul")


@pytest.mark.parametrize("tz", [None, "America/Denver", "Pacific/Fiji"])
@pytest.mark.parametrize("spec", ["1nc-p95", "1dc-p99", "1dc-median", "2dc-p50", "1wc-ep90r7", "1dc-p75-nan"])
def test_percentile_downsampling_over_calendar_slots(eng, dst_batch, tz, spec):
    """Percentile / median downsampling over variable-width calendar slots (k_pct with the
    MODE_TABLE slot lookup), across Denver's DST start and Fiji's DST end."""
    for agg in ["sum", "max"]:
        q = q_of(spec, TA + 2 * 86400 + 1234, TA + 66 * 86400, agg, tz)
        check(eng, dst_batch, q, agg, f"{tz} {spec} {agg}")


@pytest.mark.parametrize("tz", [None, "America/Denver"])
@pytest.mark.parametrize("spec", ["3wc-sum", "5wc-avg", "4wc-max-nan", "3wc-p90"])
def test_week_intervals_wider_than_two(eng, dst_batch, tz, spec):
    """n > 2 weeks: previousInterval's January-week resolution, which still lands on the Sunday
    of the span's first week (DateTime.java:559-571, TestDateTime.previousIntervalWeeks)."""
    q = q_of(spec, TA + 2 * 86400 + 1234, TA + 66 * 86400, "sum", tz)
    check(eng, dst_batch, q, "sum", f"{tz} {spec}")


def test_anchors_agree_across_spans(eng):
    # 5nc anchors at the top of the year: spans starting months apart share the grid
    T0 = 1356998400
    b = merge(synth.generate(3, T0, 200, 86400000, value_kind=2, n_groups=2, seed=3),
              synth.generate(3, T0 + 40 * 86400, 150, 86400000, value_kind=2, n_groups=2, seed=4))
    for tz in [None, "Pacific/Fiji"]:
        q = q_of("5nc-sum", T0, T0 + 200 * 86400, "sum", tz)
        check(eng, b, q, "sum", f"5nc {tz}")


@pytest.mark.parametrize("agg", ["sum", "avg", "max", "dev", "p90", "none"])
def test_anchors_disagree_with_fill(eng, staggered, agg):
    """A fill policy over per-span grids that disagree: each span's FillingDownsampler emits on its
    own calendar sequence (previousInterval(start) .. previousInterval(end)) -- its bucket where one
    has that timestamp, else the fill -- and the union evaluator aggregates those points."""
    T0 = 1356998400
    for spec in ["7sc-sum-nan", "11sc-avg-zero", "7sc-max-null"]:
        q = q_of(spec, T0 + 5, T0 + 3 * 3600 - 7, agg, None)
        check(eng, staggered, q, agg, f"anchored fill {spec} {agg}")


@pytest.mark.parametrize("tz", ["America/Denver", "Asia/Kabul"])
@pytest.mark.parametrize("spec", ["2dc-sum-zero", "5nc-sum-nan", "3wc-avg-nan", "7hc-max-null"])
def test_fill_grid_against_span_anchors(eng, dst_batch, tz, spec):
    q = q_of(spec, TA + 2 * 86400 + 1234, TA + 66 * 86400, "sum", tz)
    check(eng, dst_batch, q, "sum", f"{tz} {spec}")
