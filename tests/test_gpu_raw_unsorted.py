"""GPU parity of the raw path (no downsampler) over cells whose datapoints are NOT in time
order.  RowSeq.Iterator walks a cell in stored order (src/core/RowSeq.java:552-568) and
AggregationIterator.next emits the smallest next timestamp of the group's spans, advancing
every span that has it (src/core/AggregationIterator.java:514-567): the emitted sequence is
the greedy merge of the stored orders, not the sorted union -- timestamps may repeat or go
back, a span's window may have its point on either end or x1 <= x0 (:682-797), and a long
LERP over x1 == x0 divides by zero (ArithmeticException).  k_raw_merge walks those steps on
the GPU; everything else is the sorted path's evaluation.  The bar is the oracle, bit-exact,
or the same Java exception."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
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


def unsorted_batch(seed, n_series=30, n_groups=3, swap_p=0.15, dup_p=0.0, ms=False, kinds=(0, 1, 2), span_h=2):
    """Random series as tests/test_gpu_raw.random_batch builds them, then, inside each hour
    row, neighbouring points swapped with probability swap_p and a point given its
    predecessor's timestamp with probability dup_p."""
    rng = np.random.default_rng(seed)
    rows, gids = [], []
    for s in range(n_series):
        lo = int(rng.integers(0, span_h * 3600 // 2))
        hi = int(rng.integers(lo + 1, span_h * 3600))
        n = int(rng.integers(1, 90))
        if ms:
            t = np.sort(rng.choice(np.arange(lo * 1000, hi * 1000, 7), size=min(n, (hi - lo) * 1000 // 7),
                                   replace=False))
        else:
            t = np.sort(rng.choice(np.arange(lo, hi), size=min(n, hi - lo), replace=False)) * 1000
        ts = T0 * 1000 + t
        base = (ts // 1000) - (ts // 1000) % 3600
        for j in range(1, len(ts)):
            if base[j] != base[j - 1]:
                continue
            r = rng.random()
            if r < swap_p:
                ts[j - 1], ts[j] = ts[j], ts[j - 1]
            elif r < swap_p + dup_p:
                ts[j] = ts[j - 1]
        m = len(ts)
        kind = rng.choice(np.asarray(kinds), m)
        lv = rng.integers(-50000, 50000, m)
        fv = rng.normal(100, 40, m)
        msf = (ts % 1000 != 0) | (rng.random(m) < 0.3 if ms else False)
        rows.append(synth.encode_rows(ts, lv, fv, kind, msf))
        gids.append(s % n_groups)
    order = sorted(range(n_series), key=lambda i: gids[i])
    return synth.from_series([rows[i] for i in order], [gids[i] for i in order])


def outcome(fn):
    from opentsdb_amd.engine import EngineError
    try:
        return fn(), None
    except (EngineError, O.OracleError) as e:
        return None, e.java


def check(eng, b, q, agg, ctx, tol=0.0):
    """Same result bit for bit (tol None: the downsampled path's group-by tolerance),
    or the same Java exception; returns whether a result came back."""
    want, werr = outcome(lambda: O.run_query(b, q))
    got, gerr = outcome(lambda: eng.run_batch(b, q))
    assert gerr == werr, f"{ctx}: engine {gerr} vs oracle {werr}"
    if werr is None:
        assert_groups_match(got, want, agg, tol=tol, ctx=ctx)
    return werr is None


def test_unsorted_rows_are_flagged():
    """The batches below do hold cells out of time order (the merge path is the one taken)."""
    b = unsorted_batch(1)
    flat = []
    for r in range(len(b.row_base_time)):
        q = b.qual[b.row_qual_off[r]:b.row_qual_off[r + 1]]
        offs = [((int(q[i]) << 8 | int(q[i + 1])) >> 4) for i in range(0, len(q), 2)]
        flat.append(any(x >= y for x, y in zip(offs, offs[1:])))
    assert any(flat)


@pytest.mark.parametrize("agg", ALL_AGGS)
def test_unsorted_swaps_all_aggregators(eng, agg):
    """Swapped neighbours (no repeated timestamps): results for every aggregator."""
    b = unsorted_batch(11)
    q = abi.new_query(T0, T0 + 7199, agg)
    assert check(eng, b, q, agg, f"swaps {agg}")


@pytest.mark.parametrize("agg", ["sum", "avg", "min", "max", "count", "zimsum", "mimmin", "mimmax", "pfsum", "dev"])
def test_unsorted_integer_long_lerp(eng, agg):
    """All-integer series: nextLongValue's LERP with x outside (x0, x1) and x1 < x0."""
    b = unsorted_batch(12, kinds=(0,), swap_p=0.3)
    q = abi.new_query(T0, T0 + 7199, agg)
    assert check(eng, b, q, agg, f"long {agg}")


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("agg", ["sum", "avg", "mimmax", "count"])
def test_unsorted_ms_rows(eng, seed, agg):
    b = unsorted_batch(seed, n_series=20, ms=True)
    q = abi.new_query(T0, T0 + 7199, agg)
    check(eng, b, q, agg, f"ms {seed} {agg}")


@pytest.mark.parametrize("seed", [4, 5, 6, 7])
@pytest.mark.parametrize("agg", ["sum", "avg", "min", "count", "zimsum", "first", "last"])
def test_unsorted_repeated_timestamps(eng, seed, agg):
    """Repeated timestamps: a window with x1 == x0 (long: / by zero; double: Inf / NaN, then
    'Got Infinity'), or the same result."""
    b = unsorted_batch(seed, swap_p=0.15, dup_p=0.1)
    q = abi.new_query(T0, T0 + 7199, agg)
    check(eng, b, q, agg, f"dups {seed} {agg}")


def test_unsorted_none_aggregator(eng):
    b = unsorted_batch(21, n_series=12, dup_p=0.05)
    q = abi.new_query(T0, T0 + 7199, "none")
    assert check(eng, b, q, "none", "none")


@pytest.mark.parametrize("agg", ["p99", "p50", "ep90r3", "ep75r7", "median"])
def test_unsorted_percentile_group_by(eng, agg):
    b = unsorted_batch(31)
    q = abi.new_query(T0, T0 + 7199, agg)
    assert check(eng, b, q, agg, f"pct {agg}")
    b = unsorted_batch(32, kinds=(0,), dup_p=0.1)
    check(eng, b, q, agg, f"pct dups {agg}")


def test_unsorted_rate_raises(eng):
    """RateSpan: 'Next timestamp ... is supposed to be strictly greater' (RateSpan.java:129-134)."""
    b = unsorted_batch(41)
    q = abi.new_query(T0, T0 + 7199, "sum", rate=True)
    assert not check(eng, b, q, "sum", "rate")


def test_unsorted_long_division_by_zero(eng):
    """Span A = [5 s, 5 s] (a repeated timestamp) and B = [5 s, 3 s]: after the joint step at
    5 s, B's point at 3 s makes A interpolate between two points at 5 s -- / by zero in
    nextLongValue (ArithmeticException); with a double in the slots the LERP gives NaN / Inf
    instead."""
    ta = [(T0 + 5) * 1000, (T0 + 5) * 1000]
    tb = [(T0 + 5) * 1000, (T0 + 3) * 1000]
    z = [False, False]
    b = synth.from_series([synth.encode_rows(ta, [7, 9], None, [0, 0], z),
                           synth.encode_rows(tb, [1, 2], None, [0, 0], z)], [0, 0])
    for agg in ["sum", "dev", "p50", "median"]:   # LERP interpolation: nextLongValue divides
        assert not check(eng, b, abi.new_query(T0, T0 + 3599, agg), agg, f"long / 0 {agg}")
    for agg in ["count", "zimsum", "mimmin"]:      # ZIM / MIN interpolation: no division
        assert check(eng, b, abi.new_query(T0, T0 + 3599, agg), agg, f"long, no LERP {agg}")
    b = synth.from_series([synth.encode_rows(ta, [7, 9], [7.0, 9.0], [0, 2], z),
                           synth.encode_rows(tb, [1, 2], None, [0, 0], z)], [0, 0])
    for agg in ["sum", "count", "min", "p50"]:
        check(eng, b, abi.new_query(T0, T0 + 3599, agg), agg, f"double / 0 {agg}")


@pytest.mark.parametrize("seed", [51, 52])
@pytest.mark.parametrize("agg,ds,iv", [("sum", "sum", 60), ("sum", "avg", 60), ("max", "min", 600), ("avg", "count", 300),
                                       ("sum", "last", 60), ("p99", "avg", 60), ("none", "sum", 60)])
def test_unsorted_downsampled(eng, seed, agg, ds, iv):
    """With a downsampler the cells' stored order decides the intervals: ValuesInInterval takes
    every next value below the current interval's end (Downsampler.java:464-471), so a point
    that recedes joins the interval it follows, not its own (RowSeq.Iterator does not sort)."""
    b = unsorted_batch(seed, swap_p=0.25, dup_p=0.05)
    q = abi.new_query(T0 + 600, T0 + 6599, agg, ds_function=abi.AGG[ds], ds_interval_ms=iv * 1000)
    # timestamps and the per-span buckets exact; float sums across spans in any order (the
    # partials path) within REL_TOL unless the aggregator is order-free
    assert check(eng, b, q, agg, f"ds {seed} {agg} {iv}s-{ds}", tol=None)


def test_unsorted_downsampled_known(eng):
    """One series stored [70 s, 10 s, 130 s, 125 s] under 1m-sum: intervals 60 (70 + 10) and
    120 (130 + 125), not 0 / 60 / 120."""
    z = [False] * 4
    b = synth.from_series([synth.encode_rows([(T0 + t) * 1000 for t in (70, 10, 130, 125)], [1, 2, 4, 8], None,
                                             [0] * 4, z)], [0])
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["sum"], ds_interval_ms=60000)
    got = eng.run_batch(b, q)
    assert_groups_match(got, O.run_query(b, q), "sum", tol=0.0, ctx="known ds")
    (_, ts, bits, _), = got
    assert list(ts) == [(T0 + 60) * 1000, (T0 + 120) * 1000]
    assert [float(v) for v in bits.view(np.float64)] == [3.0, 12.0]


@pytest.mark.parametrize("pts,want", [([12930, 12890], 7.0), ([12890, 12930], 9.0), ([12930, 12890, 12940], 15.0)])
def test_unsorted_seek_row_skip(eng, pts, want):
    """A 3h1m interval puts the Downsampler's seek point S = T0 + 12900 s inside the scan's first
    hour row.  Span.seekRow passes over a row whose LAST cell is before S (Span.java:360-380): row
    [S + 30, S - 10] yields nothing (7 = the next row's 3 + 4), row [S - 10, S + 30] is entered at
    its first cell at or past S (9), and row [S + 30, S - 10, S + 40] from S + 30 on, the receding
    S - 10 included (15)."""
    n = len(pts) + 2
    b = synth.from_series([synth.encode_rows([(T0 + t) * 1000 for t in pts + [14500, 14600]], list(range(1, n + 1)),
                                             None, [0] * n, [False] * n)], [0])
    q = abi.new_query(T0 + 4 * 3600, T0 + 30 * 3600, "sum", ds_function=abi.AGG["sum"], ds_interval_ms=10860 * 1000)
    got = eng.run_batch(b, q)
    assert_groups_match(got, O.run_query(b, q), "sum", tol=0.0, ctx=f"seek {pts}")
    (_, ts, bits, _), = got
    assert list(ts) == [(T0 + 12900) * 1000] and float(bits.view(np.float64)[0]) == want


def _row(base, pts):
    """One hour row of 2-byte second qualifiers and 1-byte integers, offsets as given (up to
    4095 s: Internal.java's 12-bit offset)."""
    q = b"".join(((off << 4) | 0x0).to_bytes(2, "big") for off, _ in pts)
    v = b"".join(int(x).to_bytes(1, "big", signed=True) for _, x in pts)
    return (base, q, v)


@pytest.mark.parametrize("agg,ds", [("sum", "sum"), ("sum", "avg"), ("count", "count"), ("sum", None), ("p50", None),
                                    ("avg", None), ("sum", "last")])
def test_rows_recede_across_hour(eng, agg, ds):
    """Row T0 holds an offset past its hour (3700 s, a 2-byte qualifier reaches 4095 s); the next
    row's first datapoint (3650 s) lies before it.  Span.Iterator yields rows in order, so the
    stream goes back in time across the rows: k_recede flags the second row, and the downsampled
    path (stored order: 3650 joins the interval of 3700) and the raw greedy walk take it.  A
    second span keeps the group-by honest."""
    a = [_row(T0, [(100, 1), (3700, 2)]), _row(T0 + 3600, [(50, 4), (200, 8)])]
    b = [_row(T0, [(30, 16), (3000, 32)]), _row(T0 + 3600, [(60, 64), (300, 96)])]
    batch = synth.from_series([a, b], [0, 0])
    if ds:
        q = abi.new_query(T0, T0 + 7199, agg, ds_function=abi.AGG[ds], ds_interval_ms=60000)
    else:
        q = abi.new_query(T0, T0 + 7199, agg)
    assert check(eng, batch, q, agg, f"recede {agg} {ds}", tol=None if ds else 0.0)


def test_unsorted_known_walk(eng):
    """A = [10 s, 5 s], B = [5 s, 20 s] (long values): steps 5 (B), 10 (A), 5 (A), 20 (B).  At
    the third step B's window is (5 s, 20 s) with x == x0: B's own value 2, not a LERP."""
    z = [False, False]
    b = synth.from_series([synth.encode_rows([(T0 + 10) * 1000, (T0 + 5) * 1000], [100, 50], None, [0, 0], z),
                           synth.encode_rows([(T0 + 5) * 1000, (T0 + 20) * 1000], [2, 32], None, [0, 0], z)], [0, 0])
    q = abi.new_query(T0, T0 + 3599, "sum")
    got = eng.run_batch(b, q)
    want = O.run_query(b, q)
    assert_groups_match(got, want, "sum", tol=0.0, ctx="walk")
    (_, ts, bits, isint), = got
    assert list(ts) == [(T0 + 5) * 1000, (T0 + 10) * 1000, (T0 + 5) * 1000, (T0 + 20) * 1000]
    assert isint.all()
    # 5: B alone (A not started); 10: A's 100 + B's LERP 2 + 5*30/15 = 12; 5: A's 50 + B's 2
    # (x == x0); 20: A ended, B's 32
    assert [int(v) for v in bits.view(np.int64)] == [2, 112, 52, 32]
