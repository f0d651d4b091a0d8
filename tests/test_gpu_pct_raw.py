"""GPU parity of percentiles / median as the group-by aggregator WITHOUT a downsampler (the
raw timestamp-union path).  At every union point
AggregationIterator hands the aggregator one operand per active span -- the exact value or
its LERP (src/core/AggregationIterator.java:667-797) -- and isInteger (:612-625) picks
  runLong:   Median sorted[n / 2]; PercentileAgg with its estimation type (LEGACY / R_3 /
             R_7), then (long) of the estimate (src/core/Aggregators.java:403-413, :675-686);
  runDouble: NaNs dropped, LEGACY always (:416-430, :689-706).
k_raw_vals stores the operands, k_raw_sel selects.  Order statistics of exactly computed
operands: the bar is bit-exact against the oracle."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import set_option
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match
from tests.test_gpu_raw import random_batch

pytestmark = pytest.mark.gpu

T0 = 1356998400
GSEL = ["p999", "p99", "p95", "p90", "p75", "p50", "ep999r3", "ep99r3", "ep50r3", "ep999r7", "ep95r7", "ep50r7",
        "median"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def exact(got, want, agg, ctx):
    assert_groups_match(got, want, agg, tol=0.0, ctx=ctx)


@pytest.mark.parametrize("agg", GSEL)
def test_raw_pct_int_series(eng, agg):
    """All-integer groups: runLong with the estimation type honoured."""
    b = synth.generate(30, T0 + 3, 300, 11000, value_kind=1, n_groups=3, int_mod=20000, seed=5)
    q = abi.new_query(T0, T0 + 3599, agg)
    exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"int {agg}")


@pytest.mark.parametrize("agg", GSEL)
def test_raw_pct_random_mixed(eng, agg):
    """Late starts, early ends, int / float32 / float64 mixed: isInteger switches per point."""
    b = random_batch(11)
    q = abi.new_query(T0, T0 + 7199, agg)
    exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"mixed {agg}")


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("agg", ["p90", "ep75r3", "ep75r7", "median"])
def test_raw_pct_ms_rows(eng, seed, agg):
    b = random_batch(seed, n_series=25, ms=True)
    q = abi.new_query(T0, T0 + 7199, agg)
    exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"ms {seed} {agg}")


@pytest.mark.parametrize("opts", [dict(), dict(counter=True), dict(counter=True, drop_resets=True)])
def test_raw_pct_rate(eng, opts):
    """Rates are doubles: runDouble (LEGACY) even for the ep* aggregators."""
    b = synth.generate_counters(48, T0, 360, n_groups=4, reset_p=1 / 40, seed=9)
    for agg in ["p99", "ep99r3", "median"]:
        q = abi.new_query(T0, T0 + 3599, agg, rate=True, **opts)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"{agg} {opts}")


def test_raw_pct_ties_one_group(eng):
    """One group of 400 integer series over 50 distinct values: many ties, one block per
    union point staging 400 operands."""
    b = synth.generate(400, T0, 120, 10000, value_kind=1, n_groups=1, int_mod=50, seed=3)
    for agg in ["p99", "p50", "median", "ep999r3", "ep50r7"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, agg)


def test_raw_pct_nan_members(eng):
    """Float series with NaN values: runDouble drops them; a point whose operands are all NaN
    yields NaN."""
    rng = np.random.default_rng(5)
    rows, gids = [], []
    for s in range(12):
        ts = T0 * 1000 + np.sort(rng.choice(np.arange(0, 3600), 200, replace=False)) * 1000
        f = rng.normal(0, 10, 200)
        f[rng.random(200) < 0.2] = np.nan
        if s in (3, 4, 5):
            f[:] = np.nan
        rows.append(synth.encode_rows(ts, np.zeros(200, np.int64), f, np.full(200, 2), np.zeros(200, bool)))
        gids.append(0 if s < 6 else 1)
    b = synth.from_series(rows, gids)
    for agg in ["p90", "median", "ep90r7"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, agg)


@pytest.mark.parametrize("kind", [1, 2])
def test_raw_pct_group_beyond_lds(eng, kind):
    """A group of 5000 spans exceeds the per-wave LDS stage of k_raw_sel (4096 keys): the keys
    are built in place over the strided operands (int: compacted present longs; float: all)."""
    eng.synth(5000, T0, 6, 10000, kind, 1, 1000, 0x5EED)
    b = eng.download()
    for agg in ["p99", "ep50r3", "median"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run(q), O.run_query(b, q), agg, f"kind {kind} {agg}")


@pytest.mark.parametrize("ops", ["1", "70000"])
def test_raw_pct_strip_batches(eng, ops, monkeypatch):
    """Operands are staged per strip (RAW_STRIP points x the group's spans) in batches of at
    most option SELOPS  operands: one strip per batch, and several strips per batch."""
    set_option("SELOPS", ops)
    b = random_batch(7, n_series=60, n_groups=2, span_h=3)
    for agg in ["p95", "ep50r3", "median"]:
        q = abi.new_query(T0, T0 + 3 * 3600 - 1, agg)
        exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"ops {ops} {agg}")


@pytest.mark.parametrize("reg", ["0", "1"])
@pytest.mark.parametrize("n_spans", [40, 700, 1600, 2000])
def test_raw_pct_register_select(eng, monkeypatch, reg, n_spans):
    """k_raw_sel_reg (keys in registers, 8 / 16 / 26 / 32 a lane by group size) and the
    LDS-staged k_raw_sel (option RAW_SEL_REG = 0) against the oracle: long points with absent
    operands (spans not started or ended), double points with NaN members, ties."""
    set_option("RAW_SEL_REG", reg)
    eng.synth(n_spans, T0, 4, 10000, 1, 1, 40, 0xA5 + n_spans)
    b = eng.download()
    for agg in ["p99", "median", "ep75r7"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run(q), O.run_query(b, q), agg, f"int {n_spans} {agg}")
    for mixed in (False, True):
        b = random_batch(n_spans, n_series=n_spans, n_groups=1, mixed=mixed, span_h=1)
        for agg in ["p95", "median"]:
            q = abi.new_query(T0, T0 + 3599, agg)
            exact(eng.run_batch(b, q), O.run_query(b, q), agg, f"random {mixed} {n_spans} {agg}")


@pytest.mark.parametrize("top", ["0", "1"])
@pytest.mark.parametrize("n_spans", [12, 33, 300, 1563, 2900])
def test_raw_pct_top_select(eng, monkeypatch, top, n_spans):
    """k_raw_sel_top (lane = union point, the T largest keys streamed into registers; used when
    every requested rank lies within T of the top) against the oracle and against the per-point
    kernels (option RAW_SEL_TOP = 0): long and double points, absent operands, NaN members, ties,
    every estimation type, small groups for the median."""
    set_option("RAW_SEL_TOP", top)
    eng.synth(n_spans, T0, 4, 10000, 1, 1, 25, 0x77 + n_spans)
    b = eng.download()
    for agg in ["p99", "p999", "ep99r3", "ep99r7", "p95", "median", "p50"]:
        q = abi.new_query(T0, T0 + 3599, agg)
        exact(eng.run(q), O.run_query(b, q), agg, f"int {n_spans} {agg}")
    for mixed in (False, True):
        rb = random_batch(n_spans, n_series=min(n_spans, 150), n_groups=1, mixed=mixed, span_h=1)
        for agg in ["p99", "ep999r7", "median"]:
            q = abi.new_query(T0, T0 + 3599, agg)
            exact(eng.run_batch(rb, q), O.run_query(rb, q), agg, f"random {mixed} {n_spans} {agg}")

