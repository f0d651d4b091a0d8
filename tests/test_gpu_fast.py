"""GPU parity of the streaming kernel (k_fast) against the general kernel (k_grid) and the
CPU oracle.

k_fast reduces each bucket in an order-free way that is only taken when the exactness
certificate proves every association order gives Java's bit pattern, and it accumulates
series into the tile partials in the same order as k_grid.  So the two GPU paths must
agree BIT-EXACTLY on every query, and both must match the oracle (tolerance of
test_gpu_parity for cross-series float sums).  Tiles k_fast cannot take (NaN rows, other
row classes, failed certificate) are handed back to k_grid: those cases are covered too,
and the redo counters show which path ran."""
from __future__ import annotations

import os

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd.engine import get_option, set_option
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match, T0

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def run_path(eng, batch, q, fast: bool):
    old = get_option("FAST")
    set_option("FAST", 1 if fast else 0)
    try:
        got = eng.run_batch(batch, q) if batch is not None else eng.run(q)
        return got, eng.timing()
    finally:
        set_option("FAST", old)


def assert_bit_equal(a, b, ctx):
    assert len(a) == len(b), ctx
    for (g1, t1, v1, i1), (g2, t2, v2, i2) in zip(a, b):
        assert g1 == g2, ctx
        np.testing.assert_array_equal(t1, t2, err_msg=ctx)
        np.testing.assert_array_equal(v1, v2, err_msg=f"{ctx}: fast vs general value bits")
        np.testing.assert_array_equal(i1, i2, err_msg=ctx)


def check(eng, batch, q, agg, ctx, expect_fast=True, expect_redo=None):
    fast, tf = run_path(eng, batch, q, True)
    gen, tg = run_path(eng, batch, q, False)
    assert tg.redo_tiles == tg.tiles
    if expect_fast:
        assert tf.fast_ms > 0, f"{ctx}: streaming kernel not used"
        if expect_redo is False:
            assert tf.redo_tiles == 0, f"{ctx}: {tf.redo_tiles} tiles redone"
        elif expect_redo is True:
            assert tf.redo_tiles > 0, f"{ctx}: expected tiles handed back"
    assert_bit_equal(fast, gen, ctx)
    host = batch if batch is not None else eng.download()
    assert_groups_match(fast, O.run_query(host, q), agg, ctx=ctx)
    return tf


@pytest.fixture(scope="module")
def f32():
    return synth.generate(192, T0, 7200, 1000, value_kind=0, n_groups=3, seed=11)


DS = ["avg", "sum", "count", "squareSum", "min", "max"]


@pytest.mark.parametrize("ds", DS)
@pytest.mark.parametrize("interval", [10000, 15000, 60000, 90000, 3600000])
def test_fast_ds_intervals(eng, f32, ds, interval):
    q = abi.new_query(T0 + 1000, T0 + 6000, "sum", ds_function=abi.AGG[ds], ds_interval_ms=interval)
    # squares of float32 values carry ~48 significant bits: their sums are rarely
    # certified exact, those tiles are handed back
    check(eng, f32, q, "sum", f"{ds}-{interval}", expect_redo=None if ds == "squareSum" else False)


@pytest.mark.parametrize("period,interval", [(2000, 10000), (5000, 30000), (3000, 7000)])
def test_fast_lanes_spanning_many_buckets(eng, period, interval):
    """8 datapoints per lane cover more than two buckets: the per-datapoint fold."""
    b = synth.generate(96, T0, 3600 * 1000 // period, period, value_kind=0, n_groups=3, seed=17)
    for ds in ["avg", "max", "count"]:
        q = abi.new_query(T0 + 100, T0 + 3000, "sum", ds_function=abi.AGG[ds], ds_interval_ms=interval)
        check(eng, b, q, "sum", f"{period}/{interval} {ds}", expect_redo=False)


def test_fast_large_k_uses_general_kernel(eng, f32):
    q = abi.new_query(T0, T0 + 7199, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=1000)
    check(eng, f32, q, "sum", "K=7200", expect_fast=False)


@pytest.mark.parametrize("window", [(17, 3000), (1800, 5400), (3599, 3601), (0, 7199), (-600, 9000), (3000, 3059)])
def test_fast_edge_rows(eng, f32, window):
    a, b = window
    q = abi.new_query(T0 + a, T0 + b, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    check(eng, f32, q, "sum", f"window {window}", expect_redo=False)


@pytest.mark.parametrize("agg", ["sum", "avg", "min", "max", "count", "dev", "zimsum", "mimmin", "mimmax",
                                 "first", "last", "diff", "none", "squareSum"])
def test_fast_aggregators(eng, f32, agg):
    q = abi.new_query(T0 + 100, T0 + 7000, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    check(eng, f32, q, agg, agg, expect_redo=False)


@pytest.mark.parametrize("fill", [abi.FILL_NAN, abi.FILL_ZERO, abi.FILL_NULL])
def test_fast_fill(eng, fill):
    # query window wider than the data: leading and trailing slots are filled
    b = synth.generate(64, T0, 600, 7000, value_kind=0, n_groups=2, seed=5)
    q = abi.new_query(T0 - 300, T0 + 5400, "avg", ds_function=abi.AGG["max"], ds_interval_ms=30000, ds_fill=fill)
    check(eng, b, q, "avg", f"fill {fill}", expect_redo=False)


@pytest.mark.parametrize("opts", [dict(), dict(counter=True), dict(counter=True, drop_resets=True)])
def test_fast_rate(eng, f32, opts):
    q = abi.new_query(T0, T0 + 7199, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000, rate=True, **opts)
    check(eng, f32, q, "sum", f"rate {opts}", expect_redo=False)


def test_fast_ms_qualifiers(eng):
    b = synth.generate(96, T0, 4000, 1500, value_kind=0, n_groups=4, seed=3)
    for iv, span in [(15000, 5999), (16500, 5999), (60000, 5999), (61500, 5999)]:
        q = abi.new_query(T0, T0 + span, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=iv)
        check(eng, b, q, "sum", f"ms {iv}", expect_redo=False)


def test_fast_float64_certified(eng):
    b = synth.generate(96, T0, 3600, 1000, value_kind=3, n_groups=4, seed=9)
    for ds in ["avg", "sum", "min"]:
        q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG[ds], ds_interval_ms=60000)
        check(eng, b, q, "sum", f"f64 {ds}", expect_redo=False)


def test_fast_float64_certificate_fails(eng, monkeypatch):
    """Full-mantissa doubles: the certificate fails, every tile is redone sequentially (k_grid; the
    one-pass k_seq_dense route is switched off here, see test_float64_sequential_sums)."""
    set_option("SEQ", "0")
    b = synth.generate(96, T0, 3600, 1000, value_kind=4, n_groups=4, seed=9)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    check(eng, b, q, "sum", "f64 uncertified", expect_redo=True)
    # min/max need no certificate
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["max"], ds_interval_ms=60000)
    check(eng, b, q, "sum", "f64 max", expect_redo=False)


def test_fast_nan_and_int_rows_handed_back(eng):
    b = synth.generate(128, T0, 3600, 1000, value_kind=0, n_groups=4, seed=21)
    val = b.val.copy()
    # a NaN in the first row of series 5 (float32 big-endian quiet NaN)
    off = int(b.row_val_off[b.series_row_ptr[5]]) + 4 * 100
    val[off:off + 4] = np.frombuffer(np.array([np.nan], ">f4").tobytes(), np.uint8)
    nb = abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, val, b.group_id)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    t = check(eng, nb, q, "sum", "nan row", expect_redo=True)
    assert t.redo_tiles < t.tiles
    m = synth.generate(64, T0, 720, 5000, value_kind=2, n_groups=2, seed=4)
    check(eng, m, q, "sum", "mixed int/float", expect_redo=True)


def test_fast_device_bench_shape(eng):
    eng.synth(4096, T0, 3600, 1000, 0, 64, 1, 0x5EED)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    t = check(eng, None, q, "sum", "config2 4096 series", expect_redo=False)
    assert t.datapoints == 4096 * 3600


# ---- vle-integer class (k_fast<F, 2, 0>): 1-2 byte integers in one-chunk rows ----------
@pytest.mark.parametrize("ds", DS)
@pytest.mark.parametrize("interval", [10000, 60000, 90000, 3600000])
def test_fast_vle_ints_config1_shape(eng, ds, interval):
    b = synth.generate(96, T0, 360, 10000, value_kind=1, n_groups=3, int_mod=2000, seed=13)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG[ds], ds_interval_ms=interval)
    check(eng, b, q, "sum", f"vle {ds}-{interval}", expect_redo=False)


@pytest.mark.parametrize("agg", ["sum", "avg", "min", "max", "count", "dev"])
def test_fast_config3_shape_two_classes(eng, agg):
    """Even series int [0, 30000), odd series float32 (config 3).  With an even number of
    groups every tile is one class: the float class runs first, the vle class takes the
    tiles it hands back, nothing is left for k_grid."""
    b = synth.generate(256, T0, 360, 10000, value_kind=2, n_groups=4, int_mod=30000, seed=0x5EED)
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    check(eng, b, q, agg, f"config3 {agg}", expect_redo=False)


def test_fast_mixed_tiles_fall_through_to_grid(eng):
    # 20000 series -> tiles of 2 series; 3 groups -> each tile holds an int and a float series
    eng.synth(20000, T0, 360, 10000, 2, 3, 30000, 1)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    check(eng, None, q, "sum", "mixed tiles", expect_redo=True)
    # 4-byte integers are outside the vle class
    b = synth.generate(96, T0, 360, 10000, value_kind=1, n_groups=2, int_mod=1 << 20, seed=2)
    check(eng, b, q, "sum", "4-byte ints", expect_fast=False)


def test_fast_vle_rate_and_fill(eng):
    b = synth.generate(64, T0 + 900, 200, 10000, value_kind=1, n_groups=2, int_mod=30000, seed=8)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000, rate=True)
    check(eng, b, q, "sum", "vle rate", expect_redo=False)
    q = abi.new_query(T0, T0 + 7199, "avg", ds_function=abi.AGG["sum"], ds_interval_ms=60000, ds_fill=abi.FILL_ZERO)
    check(eng, b, q, "avg", "vle fill", expect_redo=False)


def test_fast_device_config3_shape(eng):
    eng.synth(20000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    t = check(eng, None, q, "sum", "config3 20000 series", expect_redo=False)
    assert t.datapoints == 20000 * 360


def test_fast_full_tiles_config3_shape(eng):
    """>= 524288 series: full 64-series tiles (64 rows in the walker's LDS window); both
    k_fast classes against the general kernel, bit for bit."""
    eng.synth(600000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    fast, tf = run_path(eng, None, q, True)
    gen, tg = run_path(eng, None, q, False)
    assert tf.redo_tiles == 0 and tf.fast_ms > 0
    assert_bit_equal(fast, gen, "config3 600k")


def test_fast_multi_row_series_window_refill(eng):
    """Tiles of 64 series x 24 rows: the descriptor window refills every 64 rows."""
    eng.synth(600000, T0, 24 * 36, 100000, 0, 64, 1, 7)
    q = abi.new_query(T0, T0 + 86399, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=3600000)
    fast, tf = run_path(eng, None, q, True)
    gen, tg = run_path(eng, None, q, False)
    assert tf.redo_tiles == 0 and tf.fast_ms > 0
    assert_bit_equal(fast, gen, "24 rows per series")


def run_short(eng, batch, q, short: bool):
    old = get_option("SHORT")
    set_option("SHORT", 1 if short else 0)
    try:
        return run_path(eng, batch, q, True)
    finally:
        set_option("SHORT", old)


@pytest.mark.parametrize("agg,ds", [("sum", "avg"), ("avg", "sum"), ("dev", "avg"), ("min", "max"), ("max", "min"),
                                    ("count", "count"), ("sum", "squareSum")])
def test_short_kernel_matches_walker(eng, agg, ds):
    """k_short (one row per series, descriptors up front) against k_fast's row walker and
    k_grid, bit for bit, on the config 3 shape."""
    eng.synth(40000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG[ds], ds_interval_ms=60000)
    s, ts = run_short(eng, None, q, True)
    w, tw = run_short(eng, None, q, False)
    g, tg = run_path(eng, None, q, False)
    assert ts.redo_tiles == 0 and ts.fast_ms > 0
    assert_bit_equal(s, w, f"short vs walker {agg}:{ds}")
    assert_bit_equal(s, g, f"short vs general {agg}:{ds}")


def test_short_kernel_mixed_row_counts(eng):
    """Tiles mixing one-row and two-row series, and rows outside the scan range: k_short
    hands those tiles to k_fast; results identical to the general kernel and the oracle."""
    rng = np.random.default_rng(3)
    series, gids = [], []
    for s in range(300):
        start = T0 + (1800 if s % 7 == 0 else 0) + (7200 if s % 11 == 0 else 0)
        ts = (start + np.arange(360) * 10) * 1000
        fv = np.round(rng.normal(50, 5, 360), 3)
        series.append(synth.encode_rows(ts, None, fv, np.ones(360, int), np.zeros(360, bool)))
        gids.append(s % 3)
    b = synth.from_series(series, gids)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    s, ts = run_short(eng, b, q, True)
    g, tg = run_path(eng, b, q, False)
    assert_bit_equal(s, g, "mixed row counts")
    assert_groups_match(s, O.run_query(b, q), "sum", ctx="mixed row counts vs oracle")


@pytest.mark.parametrize("ds,iv,span", [("sum", 60000, 3 * 3600 - 1), ("avg", 420000, 3 * 3600 - 1),
                                        ("squareSum", 60000, 3599), ("avg", 86400000, 3 * 3600 - 1),
                                        ("sum", 1000, 1799), ("avg", 60000, 3 * 3600 - 1)])
@pytest.mark.parametrize("seqwave", ["1", "0"])
def test_float64_sequential_sums(eng, monkeypatch, seqwave, ds, iv, span):
    """k_seq_wave (one wave a series, K <= 64) and k_seq_dense (option SEQ_WAVE = 0).  Full-mantissa doubles over three hour rows: the rows carry ROW_NOCERT (two of their values
    cannot add exactly).  Sum / avg downsampling then runs k_seq_dense (each bucket in Java's
    order, one pass, then the group-by step over the stored buckets); with it switched off the
    streaming kernels hand the tiles to k_grid, which sums them in order in one pass (slow_chunk).
    Both equal the general path bit for bit and the oracle -- buckets inside a row, across rows
    (7m), one a day and one a datapoint; squareSum keeps the certificate check at series end."""
    set_option("SEQ_WAVE", seqwave)
    b = synth.generate(70, T0, 3 * 3600, 1000, value_kind=4, n_groups=3, seed=17)
    for agg in ("sum", "max", "none"):
        q = abi.new_query(T0, T0 + span, agg, ds_function=abi.AGG[ds], ds_interval_ms=iv)
        seq, ts = run_path(eng, b, q, True)
        gen, _ = run_path(eng, b, q, False)
        set_option("SEQ", 0)
        try:
            grid, _ = run_path(eng, b, q, True)
        finally:
            set_option("SEQ", None)
        if ds in ("sum", "avg"):
            assert ts.fast_ms == 0, "k_seq_dense expected (no streaming pass)"
        ctx = f"f64 seq {ds} {iv} {agg}"
        assert_bit_equal(seq, gen, ctx)
        assert_bit_equal(grid, gen, ctx + " (k_grid)")
        assert_groups_match(seq, O.run_query(b, q), agg, ctx=ctx)


@pytest.mark.parametrize("seqwave", ["1", "0"])
def test_float64_sequential_sums_mixed_rows(eng, monkeypatch, seqwave):
    """Both sequential kernels (option SEQ_WAVE).  k_seq_dense over a scan mixing full-mantissa doubles (ROW_NOCERT), vle integers and
    millisecond rows: the non-uniform rows are walked datapoint by datapoint (width from the
    qualifier, length from its flags); bit-exact against the general path and the oracle."""
    set_option("SEQ_WAVE", seqwave)
    from tests.test_gpu_calendar_tz import merge
    b = merge(synth.generate(20, T0, 7200, 1000, value_kind=4, n_groups=3, seed=5),
              synth.generate(20, T0, 7200, 1000, value_kind=1, n_groups=3, int_mod=70000, seed=6),
              synth.generate(10, T0, 3000, 2500, value_kind=4, n_groups=3, seed=7))
    for ds, iv in (("sum", 60000), ("avg", 300000)):
        for agg in ("sum", "avg"):
            q = abi.new_query(T0, T0 + 7199, agg, ds_function=abi.AGG[ds], ds_interval_ms=iv)
            seq, ts = run_path(eng, b, q, True)
            gen, _ = run_path(eng, b, q, False)
            assert ts.fast_ms == 0
            assert_bit_equal(seq, gen, f"mixed {ds} {agg}")
            assert_groups_match(seq, O.run_query(b, q), agg, ctx=f"mixed {ds} {agg}")


@pytest.fixture(scope="module")
def tiny_rows():
    return synth.generate(100_000, T0, 8, 450000, value_kind=2, n_groups=16, int_mod=900, seed=23)


@pytest.mark.parametrize("ds", ["sum", "avg", "min", "max", "count", "dev", "first", "last", "diff", "squareSum"])
def test_tiny_rows_at_scale_sequential(eng, tiny_rows, ds):
    """100k series of one 8-point row (the shape of rollup tables read as hour rows): every
    downsampling function runs k_seq_dense (one series a thread, Java's order), bit-exact against
    the streaming / k_grid path and the oracle."""
    b = tiny_rows
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG[ds], ds_interval_ms=900000)
    seq, ts = run_path(eng, b, q, True)
    set_option("SEQ", 0)
    try:
        other, _ = run_path(eng, b, q, True)
    finally:
        set_option("SEQ", None)
    assert ts.fast_ms == 0, "k_seq_dense expected"
    assert_bit_equal(seq, other, f"tiny {ds}")
    assert_groups_match(seq, O.run_query(b, q), "sum", ctx=f"tiny {ds}")


def _short_rows_with_breaks():
    """300 series of full-mantissa doubles in short hour rows (6 points an hour, 24 hours) -- the
    shape of a rollup table read as hour rows -- plus rows k_seq_rows must hand back: series 3's
    sixth row reaches 160 s past its hour (2-byte qualifiers go to 4095 s), series 7 holds two
    cells of one hour (a repeated base), series 11 mixes 2-byte integers into its rows."""
    rng = np.random.default_rng(31)
    rows, gids = [], []
    for s in range(300):
        ts = T0 * 1000 + np.arange(24 * 6, dtype=np.int64) * 600000 + rng.integers(0, 599, 24 * 6) * 1000
        f = rng.normal(50, 10, len(ts)) * (1 + 1e-9 * s)
        kind = np.full(len(ts), 2)
        lv = np.zeros(len(ts), np.int64)
        if s == 11:
            kind[::5] = 0
            lv[::5] = rng.integers(-30000, 30000, len(lv[::5]))
        r = synth.encode_rows(ts, lv, f, kind, np.zeros(len(ts), bool))
        if s == 3:
            base, q, v = r[5]
            extra = [(3600 + 40 * k, float(rng.normal(50, 10))) for k in range(5)]   # (< 3840: 0xF0.. is a ms qualifier)
            q += b"".join(((off << 4) | 0xF).to_bytes(2, "big") for off, _ in extra)
            v = v[:-1] + b"".join(np.array([x], ">f8").tobytes() for _, x in extra) + v[-1:]
            r[5] = (base, q, v)
        if s == 7:
            base, q, v = r[8]
            r.insert(9, (base, ((3599 << 4) | 0xF).to_bytes(2, "big"), np.array([12.375], ">f8").tobytes()))
        rows.append(r)
        gids.append(s % 5)
    order = sorted(range(300), key=lambda i: gids[i])
    return synth.from_series([rows[i] for i in order], [gids[i] for i in order])


@pytest.mark.parametrize("ds,iv", [("sum", 600000), ("avg", 3600000), ("dev", 1200000), ("first", 600000),
                                   ("sum", 420000), ("avg", 86400000)])
def test_sequential_rows_kernel(eng, monkeypatch, ds, iv):
    """k_seq_rows (one thread a short hour row, Java's order inside each bucket) against
    k_seq_dense (option SEQ_ROWS = 0) bit for bit and the oracle, including the series it hands
    back (a row past its hour, two cells of one hour, mixed value kinds) and intervals it does not
    take (7m buckets crossing rows, 1d)."""
    b = _short_rows_with_breaks()
    res = {}
    for mode in ("1", "0"):
        set_option("SEQ_ROWS", mode)
        for agg in ("sum", "none"):
            q = abi.new_query(T0, T0 + 86399, agg, ds_function=abi.AGG[ds], ds_interval_ms=iv)
            got, tm = run_path(eng, b, q, True)
            assert_groups_match(got, O.run_query(b, q), agg, ctx=f"{ds} {iv} {agg} rows={mode}")
            res[(mode, agg)] = got
    for agg in ("sum", "none"):
        assert_bit_equal(res[("1", agg)], res[("0", agg)], f"{ds} {iv} {agg} k_seq_rows vs k_seq_dense")


def run_rows(eng, batch, q, rows: bool, monkeypatch):
    set_option("ROWS", "1" if rows else "0")
    try:
        return run_path(eng, batch, q, True)
    finally:
        set_option("ROWS", None)


@pytest.mark.parametrize("agg,ds,iv,win,rate", [
    ("sum", "avg", 3600000, (0, 86399), False),       # K 24: register partials
    ("avg", "sum", 600000, (5000, 80000), False),     # K 126, rows cut at both ends: LDS partials
    ("dev", "avg", 60000, (0, 86399), False),         # K 1440: series buckets to HBM, then k_emit_win
    ("max", "min", 3600000, (7200, 50000), False),
    ("count", "count", 1800000, (0, 86399), False),
    ("sum", "avg", 3600000, (0, 86399), True),        # rate: LDS partials
    ("none", "avg", 3600000, (0, 86399), False),      # one tile a series
])
def test_rows_kernel_matches_walker(eng, monkeypatch, agg, ds, iv, win, rate):
    """k_rows (series of several one-chunk rows, descriptors in 64-row batches) against k_fast's
    row walker (option ROWS = 0) and k_grid, bit for bit: 40000 series of 24 hour rows (4 series a
    tile, 96 rows: the batch refill), int and float series (two row classes).  (k_hwin off: the
    1m case runs the dense split; its buckets are one datapoint in 100 s, LERP fills between.)"""
    set_option("HWIN", "0")
    eng.synth(40000, T0, 24 * 36, 100000, 2, 1000, 30000, 0x5EED)
    q = abi.new_query(T0 + win[0], T0 + win[1], agg, ds_function=abi.AGG[ds], ds_interval_ms=iv, rate=rate)
    r, tr = run_rows(eng, None, q, True, monkeypatch)
    w, tw = run_rows(eng, None, q, False, monkeypatch)
    g, tg = run_path(eng, None, q, False)
    assert tr.fast_ms > 0 and tr.redo_tiles == 0
    assert_bit_equal(r, w, f"rows vs walker {agg}:{ds} {iv} {win}")
    assert_bit_equal(r, g, f"rows vs general {agg}:{ds} {iv} {win}")


def _irregular_rows(seed=5, n=240):
    """Series of 0 to 90 hour rows at mixed periods with gaps; some with a row of 1 s points (over
    CH: that tile goes to the walker), some starting before or ending after the query window."""
    rng = np.random.default_rng(seed)
    series, gids = [], []
    for s in range(n):
        nh = 0 if s % 13 == 0 else int(rng.integers(1, 90 if s % 5 == 0 else 12))
        h0 = int(rng.integers(-4, 6))
        ts = []
        for h in range(nh):
            period = 1 if (s % 29 == 1 and h == 0) else int(rng.choice([10, 20, 30, 60, 120]))
            k = np.arange(3600 // period) * period
            k = k[rng.random(len(k)) > 0.1]
            ts.append(T0 + (h0 + h) * 3600 + k)
        ts = np.concatenate(ts) * 1000 if ts else np.zeros(0, np.int64)
        fv = np.round(rng.normal(50, 5, len(ts)), 3)
        series.append(synth.encode_rows(ts, None, fv, np.ones(len(ts), int), np.zeros(len(ts), bool)))
        gids.append(s % 3)
    order = sorted(range(n), key=lambda i: gids[i])
    return synth.from_series([series[i] for i in order], [gids[i] for i in order])


def test_rows_kernel_irregular(eng, monkeypatch):
    """k_rows on ragged series (no rows, > 64 rows, rows outside the window, a row over CH) against
    the walker, the general kernel and the oracle."""
    b = _irregular_rows()
    for agg, ds, iv in [("sum", "avg", 3600000), ("avg", "sum", 600000), ("max", "max", 86400000),
                        ("dev", "avg", 900000), ("sum", "avg", 60000)]:
        q = abi.new_query(T0 + 1800, T0 + 40 * 3600, agg, ds_function=abi.AGG[ds], ds_interval_ms=iv)
        r, tr = run_rows(eng, b, q, True, monkeypatch)
        w, tw = run_rows(eng, b, q, False, monkeypatch)
        g, tg = run_path(eng, b, q, False)
        ctx = f"irregular {agg}:{ds} {iv}"
        if 60000 < iv < 86400000:   # (1m here and 1d: other routes; both still compared below)
            assert tr.fast_ms > 0, ctx
        assert_bit_equal(r, w, ctx + " rows vs walker")
        assert_bit_equal(r, g, ctx + " rows vs general")
        assert_groups_match(r, O.run_query(b, q), agg, ctx=ctx)


def run_hwin(eng, batch, q, on: bool, monkeypatch):
    set_option("HWIN", "1" if on else "0")
    try:
        return run_path(eng, batch, q, True)
    finally:
        set_option("HWIN", None)


@pytest.mark.parametrize("agg,ds,iv,win,fill", [
    ("sum", "avg", 60000, (0, 86399), abi.FILL_NONE),        # K 1440 (config 3's day)
    ("avg", "sum", 60000, (7200, 79199), abi.FILL_NONE),     # K 1200, window inside the data
    ("max", "min", 60000, (0, 86399), abi.FILL_NONE),
    ("dev", "avg", 60000, (3600, 86399), abi.FILL_NONE),
    ("count", "count", 60000, (0, 86399), abi.FILL_NONE),
    ("sum", "squareSum", 60000, (0, 86399), abi.FILL_NONE),  # squares rarely certify: handed back
    ("sum", "avg", 60000, (-3600, 90000 - 1), abi.FILL_NONE),   # window wider than the data
])
def test_hwin_matches_dense_split(eng, monkeypatch, agg, ds, iv, win, fill):
    """k_hwin (K > 64 buckets tiling the hour, walked window by window with register partials; the
    queries whose one-pass slot LDS does not fit, K >= 859) against the dense split (option HWIN = 0: buckets stored, then k_emit_win) and the general
    kernel, bit for bit: 40000 series x a day of 10 s points (24 hour rows), int and float series."""
    eng.synth(40000, T0, 24 * 360, 10000, 2, 1000, 30000, 0x5EED)
    q = abi.new_query(T0 + win[0], T0 + win[1], agg, ds_function=abi.AGG[ds], ds_interval_ms=iv, ds_fill=fill)
    h, th = run_hwin(eng, None, q, True, monkeypatch)
    d, td = run_hwin(eng, None, q, False, monkeypatch)
    g, tg = run_path(eng, None, q, False)
    ctx = f"hwin {agg}:{ds} {iv} {win} fill {fill}"
    assert th.fast_ms > 0, ctx
    if ds != "squareSum":
        assert th.redo_tiles == 0, f"{ctx}: {th.redo_tiles} tiles handed back"
    assert_bit_equal(h, d, ctx + " hwin vs split")
    assert_bit_equal(h, g, ctx + " hwin vs general")


def test_hwin_holes_handed_back(eng, monkeypatch):
    """Buckets missing inside a series' span (100 s points in 1m buckets; a series missing an hour):
    LERP needs neighbours from other windows, so k_hwin hands those tiles to the general kernel --
    same answers as the general path and the oracle."""
    b = _irregular_rows(seed=9, n=120)
    for agg, ds, iv in [("sum", "avg", 60000), ("avg", "max", 120000)]:
        q = abi.new_query(T0, T0 + 30 * 3600 - 1, agg, ds_function=abi.AGG[ds], ds_interval_ms=iv)
        h, th = run_hwin(eng, b, q, True, monkeypatch)
        g, tg = run_path(eng, b, q, False)
        ctx = f"hwin holes {agg}:{ds} {iv}"
        assert_bit_equal(h, g, ctx)
        assert_groups_match(h, O.run_query(b, q), agg, ctx=ctx)
    eng.synth(4000, T0, 24 * 36, 100000, 0, 16, 1, 3)
    q = abi.new_query(T0, T0 + 86399, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    h, th = run_hwin(eng, None, q, True, monkeypatch)
    g, tg = run_path(eng, None, q, False)
    assert th.redo_tiles > 0
    assert_bit_equal(h, g, "hwin 100 s points")
