"""GPU parity of the raw path (queries without downsampling): AggregationIterator over the
timestamp union with LERP / ZIM / MAX / MIN / PREV, rate / counters, isInteger switching,
spans that start late or end early, and the NONE aggregator -- all against the CPU oracle,
BIT-EXACTLY: the raw kernel feeds every aggregator its span values in SpanGroup order, so
float sums follow the reference's association as well."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import set_option
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400
ALL_AGGS = ["sum", "avg", "min", "max", "count", "dev", "zimsum", "mimmin", "mimmax", "squareSum", "first",
            "last", "diff", "pfsum", "mult"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def exact(got, want, agg, ctx):
    assert_groups_match(got, want, agg, tol=0.0, ctx=ctx)


def random_batch(seed, n_series=40, n_groups=3, ms=False, mixed=True, span_h=2):
    """Series with random point sets inside [T0, T0 + span_h h): late starts, early ends,
    int / float32 / float64 values (mixed within a series when `mixed`)."""
    rng = np.random.default_rng(seed)
    rows, gids = [], []
    for s in range(n_series):
        lo = int(rng.integers(0, span_h * 3600 // 2))
        hi = int(rng.integers(lo + 1, span_h * 3600))
        n = int(rng.integers(1, 120))
        if ms:
            t = np.sort(rng.choice(np.arange(lo * 1000, hi * 1000, 7), size=min(n, (hi - lo) * 1000 // 7), replace=False))
        else:
            t = np.sort(rng.choice(np.arange(lo, hi), size=min(n, hi - lo), replace=False)) * 1000
        ts = T0 * 1000 + t
        m = len(ts)
        if mixed:
            kind = rng.integers(0, 3, m)
        else:
            kind = np.full(m, 0 if s % 2 == 0 else 1)
        lv = rng.integers(-50000, 50000, m)
        fv = rng.normal(100, 40, m)
        msf = np.full(m, ms) if not mixed else (ts % 1000 != 0) | (rng.random(m) < 0.3 if ms else False)
        rows.append(synth.encode_rows(ts, lv, fv, kind, msf))
        gids.append(s % n_groups)
    order = sorted(range(n_series), key=lambda i: gids[i])
    return synth.from_series([rows[i] for i in order], [gids[i] for i in order])


@pytest.mark.parametrize("agg", ALL_AGGS)
def test_raw_aggregators_int_series(eng, agg):
    b = synth.generate(30, T0 + 3, 300, 11000, value_kind=1, n_groups=3, int_mod=20000, seed=5)
    q = abi.new_query(T0, T0 + 3599, agg)
    exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"int {agg}")


@pytest.mark.parametrize("agg", ALL_AGGS)
def test_raw_aggregators_random_mixed(eng, agg):
    b = random_batch(11)
    q = abi.new_query(T0, T0 + 7199, agg)
    exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"mixed {agg}")


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("agg", ["sum", "avg", "dev", "mimmin", "mimmax", "zimsum"])
def test_raw_ms_and_mixed_rows(eng, seed, agg):
    b = random_batch(seed, n_series=25, ms=True)
    q = abi.new_query(T0, T0 + 7199, agg)
    exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"ms seed={seed} {agg}")


def test_raw_pure_float_groups(eng):
    b = random_batch(21, mixed=False)
    for agg in ["sum", "avg", "squareSum", "dev", "mult"]:
        q = abi.new_query(T0, T0 + 7199, agg)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, agg)


@pytest.mark.parametrize("opts", [dict(), dict(counter=True), dict(counter=True, drop_resets=True),
                                  dict(counter=True, counter_max=1 << 32, reset_value=1000000),
                                  dict(counter=True, reset_value=5)])
def test_raw_rate_counters(eng, opts):
    b = synth.generate_counters(48, T0, 360, n_groups=4, reset_p=1 / 40, seed=9)
    for agg in ["sum", "avg", "max", "pfsum"]:
        q = abi.new_query(T0, T0 + 3599, agg, rate=True, **opts)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"{agg} {opts}")


def test_raw_rate_mixed_random(eng):
    b = random_batch(31)
    for agg in ["sum", "dev", "min"]:
        q = abi.new_query(T0, T0 + 7199, agg, rate=True)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, agg)


def test_raw_config4_shape(eng):
    """BASELINE config 4 at 1/500 scale: 200 jittered counters x 1 h, 64 groups, sum (long LERP)."""
    b = synth.generate_counters(200, T0, 360, n_groups=64, seed=0x5EED)
    q = abi.new_query(T0, T0 + 3599, "sum")
    exact(eng.run_batch(b, q), O.run_query(b, q), "sum", "config4 sum")
    q = abi.new_query(T0, T0 + 3599, "sum", rate=True, counter=True, counter_max=1 << 32, reset_value=1000000)
    exact(eng.run_batch(b, q), O.run_query(b, q), "sum", "config4 rate")


def test_raw_none_aggregator(eng):
    b = random_batch(41, n_series=12)
    q = abi.new_query(T0, T0 + 7199, "none")
    exact(eng.run_batch(b, q), O.run_query(b, q), "none", "none")


def test_raw_large_group_global_cursors(eng):
    """More spans in a group than fit the LDS cursor table (RAW_LDS_SPANS = 4096)."""
    b = synth.generate(5000, T0, 40, 90000, value_kind=1, n_groups=1, int_mod=1000, seed=3)
    q = abi.new_query(T0, T0 + 3599, "sum")
    exact(eng.run_batch(b, q), O.run_query(b, q), "sum", "5000 spans")


def test_raw_long_overflow_wraps(eng):
    """Long LERP and sums wrap like Java longs (8-byte values near Long.MAX_VALUE)."""
    big = (1 << 62) + 12345
    rows = [synth.encode_rows([T0 * 1000, (T0 + 100) * 1000], [big, -big], None, [0, 0], [False, False]),
            synth.encode_rows([(T0 + 30) * 1000, (T0 + 70) * 1000], [big, big], None, [0, 0], [False, False])]
    b = synth.from_series(rows, [0, 0])
    for agg in ["sum", "avg", "squareSum", "mult", "diff", "dev"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, agg)


def test_raw_spans_outside_scan_range(eng):
    """Series whose rows all lie outside the scan range sit in the group with no points."""
    rows = [synth.encode_rows([T0 * 1000 + 5000, T0 * 1000 + 65000], [3, 9], None, [0, 0], [False, False]),
            synth.encode_rows([(T0 + 7200) * 1000 + 1000], [7], None, [0], [False]),
            synth.encode_rows([T0 * 1000 + 20000, T0 * 1000 + 80000], [1.5, 2.5], [1.5, 2.5], [1, 1], [False, False])]
    b = synth.from_series(rows, [0, 0, 0])
    for agg in ["sum", "min", "count"]:
        for rate in (False, True):
            q = abi.new_query(T0, T0 + 3599, agg, rate=rate)
            exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"{agg} rate={rate}")


@pytest.mark.parametrize("lerpw", ["0", "1"])
def test_raw_strip_window_lerp(eng, monkeypatch, lerpw):
    """k_raw_eval's strip-wide long LERP (lerpw_*: reciprocal quotient + exact remainder) and the
    general 64-bit path (option RAW_LERPW = 0) give the oracle's answer: counters, large-slope
    integers that leave the fast window (|dy| (x1 - x0) >= 2^51), negative slopes, mixed groups."""
    set_option("RAW_LERPW", lerpw)
    b = synth.generate_counters(300, T0, 360, n_groups=16, seed=0xC4)
    for agg in ["sum", "avg", "min", "max", "dev"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"counters {agg}")
    rng = np.random.default_rng(3)
    rows = []
    for s in range(24):
        ts = T0 * 1000 + np.sort(rng.choice(np.arange(0, 3600000, 13), 40, replace=False))
        scale = [10, 1 << 30, 1 << 45, 1 << 61][s % 4]
        lv = rng.integers(-scale, scale, 40)
        rows.append(synth.encode_rows(ts, lv, None, np.zeros(40, np.int64), np.ones(40, bool)))
    b = synth.from_series(rows, [s // 6 for s in range(24)])
    for agg in ["sum", "max", "mult"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"wide {agg}")
    b = random_batch(77, n_series=60, n_groups=2)
    q = abi.new_query(T0, T0 + 7199, "sum")
    exact(eng.run_batch(b, q), O.run_query(b, q), "sum", "mixed")
