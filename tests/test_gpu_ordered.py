"""GPU parity of TSDB_QF_ORDERED: cross-series float reductions folded in SpanGroup index
order (AggregationIterator hands Aggregator.runDouble one value per span in span order,
src/core/AggregationIterator.java:735-797; Sum :237-259, SquareSum :269-293, Avg :371-393,
StdDev :504-569, Multiply :470-485).  The default path sums tiles in a tree (relative error
<= 1e-12); with the flag every aggregator is BIT-EXACT against the
oracle."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.query import TsdbQuery
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400
ORD = ["sum", "avg", "squareSum", "dev", "zimsum", "pfsum"]


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def float_batch():
    # 500 float series over 2 groups: long enough sums for the association to matter
    return synth.generate(500, T0, 360, 10000, value_kind=0, n_groups=2, seed=21)


@pytest.mark.parametrize("agg", ORD)
def test_ordered_bit_exact(eng, float_batch, agg):
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000, flags=abi.QF_ORDERED)
    assert_groups_match(eng.run_batch(float_batch, q), O.run_query(float_batch, q), agg, tol=0.0, ctx=agg)


def test_ordered_mult_small_and_overflow(eng, float_batch):
    b = synth.generate(20, T0, 360, 10000, value_kind=0, n_groups=2, seed=22)
    q = abi.new_query(T0, T0 + 3599, "mult", ds_function=abi.AGG["avg"], ds_interval_ms=60000, flags=abi.QF_ORDERED)
    assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), "mult", tol=0.0, ctx="mult")
    # 250 factors of ~50 overflow: doubleValue's Inf check throws on both sides
    with pytest.raises(Exception) as e1:
        eng.run_batch(float_batch, q)
    with pytest.raises(Exception) as e2:
        O.run_query(float_batch, q)
    assert e1.value.java == e2.value.java == "IllegalStateException"


@pytest.mark.parametrize("kw", [dict(ds_fill=abi.FILL_NAN), dict(ds_fill=abi.FILL_ZERO), dict(rate=True),
                                dict(ds_all=True)])
def test_ordered_fill_rate_all(eng, float_batch, kw):
    for agg in ["sum", "dev"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["sum"], ds_interval_ms=0 if "ds_all" in kw else 300000,
                          flags=abi.QF_ORDERED, **kw)
        assert_groups_match(eng.run_batch(float_batch, q), O.run_query(float_batch, q), agg, tol=0.0, ctx=f"{agg} {kw}")


def test_ordered_sparse_lerp(eng):
    rng = np.random.default_rng(23)
    from opentsdb_amd.store import MockStore
    st = MockStore()
    for s in range(60):
        ts = np.sort(rng.choice(np.arange(0, 7200, 7), size=rng.integers(3, 200), replace=False))
        for t in ts:
            st.add_float("m", T0 + int(t), float(rng.normal(10, 5)), {"h": f"h{s}", "g": f"g{s % 3}"})
    for agg in ["sum", "avg", "dev", "squareSum"]:
        q = TsdbQuery(st, runner=eng.run_batch)
        q.setStartTime(T0)
        q.setEndTime(T0 + 7199)
        q.setTimeSeries("m", {"g": "*"}, agg, False)
        q.downsample("2m-avg")
        batch, _ = q.build_batch()
        qa = q.to_abi()
        qa.flags = abi.QF_ORDERED
        assert_groups_match(eng.run_batch(batch, qa), O.run_query(batch, qa), agg, tol=0.0, ctx=agg)


def test_ordered_config3_shape(eng):
    # one-row int / float series (k_short in dense_out mode) through the ordered fold
    b = synth.generate(3000, T0, 360, 10000, value_kind=2, n_groups=5, int_mod=30000, seed=5)
    for agg in ["sum", "avg", "dev"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000, flags=abi.QF_ORDERED)
        assert_groups_match(eng.run_batch(b, q), O.run_query(b, q), agg, tol=0.0, ctx=agg)
