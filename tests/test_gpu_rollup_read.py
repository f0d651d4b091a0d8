"""GPU parity of the rollup read path: tsdbhip_load_rollup + run
(engine.cpp run_rollup: the RollupSeq restatement on the host, the value / count series on
the device, k_rollup_combine for avg and count downsampling of rollups).

  * every known answer of test/core/TestTsdbQueryRollup.java (tests/golden/rollup_queries.json)
    through the engine, and against the oracle on the same inputs;
  * the RollupSeq corner cases (sync, duplicates, zero counts, exceptions);
  * randomized multi-series rollup tables with missing sum / count cells against the oracle:
    aggregators, downsampling functions and intervals, fills, rate, NONE."""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np
import pytest

from opentsdb_amd import abi, engine
from opentsdb_amd.engine import set_option
from opentsdb_amd.engine import EngineError
from opentsdb_amd.rollup_read import make_rollup_batch
from oracle import oracle as O
from tests import golden_util as gu
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

DOC = gu.load("rollup_queries.json")
CASES = [c for c in DOC["cases"] if "write_error" not in c["expect"]]
B = 1356998400


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_known_answers_on_gpu(eng, case):
    q = gu.rollup_query(DOC, case, eng.run_batch, eng.run_rollup_batch)
    if "error" in case["expect"]:
        with pytest.raises(EngineError) as e:
            q.run()
        assert e.value.java == case["expect"]["error"]
        return
    gu.check_rollup_expect(case, q.run())
    # the same inputs through the oracle, bit for bit
    name = q.rollup_interval_name()
    if name is None:
        return
    rb, _ = q.build_rollup_batch(name)
    if rb.cells.n_series:
        assert_groups_match(eng.run_rollup_batch(rb, q.to_abi()), O.run_rollup_query(rb, q.to_abi()),
                            q.aggregator, tol=0.0, ctx=case["name"])


def _iv(interval="10m", span="6h"):
    return engine.rollup_interval(interval, span)


def _batch(rows, counts=True, fix=False, groups=None, iv=None):
    spans = []
    for s in rows:
        rr = []
        for base, vals, cnts in s:
            rr.append((base, [(struct.pack(">H", (o << 4) | f), v) for o, f, v in vals],
                       [(struct.pack(">H", (o << 4) | f), v) for o, f, v in cnts]))
        spans.append((None, rr))
    return make_rollup_batch(spans, groups if groups is not None else [0] * len(spans), iv or _iv(), counts, fix)


def _l(v):
    return (0x7, struct.pack(">q", v))


def _q(ds="10m-avg", agg="avg", start=B, end=B + 43200, rate=False):
    q = abi.new_query(start, end, agg, rate=rate)
    assert O.lib().ref_parse_downsample(ds.encode(), C.byref(q)) == 0
    return q


def both(eng, rb, q):
    return eng.run_rollup_batch(rb, q), O.run_rollup_query(rb, q)


def test_sync_count_zero(eng):
    rb = _batch([[(B, [(0, *_l(20)), (1, *_l(40)), (3, *_l(60)), (4, *_l(9))],
                   [(0, *_l(2)), (2, *_l(9)), (3, *_l(3)), (4, *_l(0))])]])
    for ds in ("10m-avg", "20m-avg", "10m-count", "30m-count", "10m-sum", "10m-max", "1h-avg-zero"):
        g, w = both(eng, rb, _q(ds))
        assert_groups_match(g, w, "avg", tol=0.0, ctx=ds)


def test_errors_match_oracle(eng):
    cases = [
        (_batch([[(B, [(2, *_l(1)), (1, *_l(2))], [])]], counts=False), _q("10m-sum", "sum")),
        (_batch([[(B, [(1, *_l(1)), (2, *_l(2))], [(2, *_l(1)), (1, *_l(2))])]]), _q()),
        (_batch([[(B, [(0, *_l(20))], [(0, *_l(2))])]]), _q("10m-dev", "avg")),
    ]
    for rb, q in cases:
        with pytest.raises(O.OracleError) as eo:
            O.run_rollup_query(rb, q)
        with pytest.raises(EngineError) as ee:
            eng.run_rollup_batch(rb, q)
        assert ee.value.code == eo.value.code
    # a bad row outside the scan range is never scanned
    rb = _batch([[(B, [(0, *_l(1))], []), (B + 86400 * 3, [(2, *_l(1)), (1, *_l(2))], [])]], counts=False)
    g, w = both(eng, rb, _q("10m-sum", "sum"))
    assert_groups_match(g, w, "sum", tol=0.0)


def test_scan_impossible_cells_raise_illegal_data(eng):
    """Cells an HBase scan of a rollup table cannot return -- one row key's cells split by another
    key's, an offset past the row span -- are refused as IllegalDataException (RollupSeq.addRow,
    src/rollup/RollupSeq.java:170-205), never as an unimplemented case."""
    split = _batch([[(B, [(0, *_l(1))], []), (B + 21600, [(0, *_l(2))], []), (B, [(3, *_l(3))], [])]], counts=False)
    past = _batch([[(B, [(0, *_l(1)), (40, *_l(2))], [])]], counts=False)   # 40 x 10m beyond a 6h row
    for rb in (split, past):
        with pytest.raises(EngineError) as ee:
            eng.run_rollup_batch(rb, _q("10m-sum", "sum"))
        assert ee.value.java == "IllegalDataException"


def test_duplicates_fixed(eng):
    rb = _batch([[(B, [(1, *_l(1)), (1, 0xB, struct.pack(">f", 42.5))], [])]], counts=False, fix=True)
    g, w = both(eng, rb, _q("10m-sum", "sum"))
    assert_groups_match(g, w, "sum", tol=0.0)
    assert g[0][2].view(np.float64).tolist() == [42.5]


def test_rollup_mode_guards(eng):
    rb = _batch([[(B, [(0, *_l(20))], [(0, *_l(2))])]])
    eng.load_rollup(rb)
    with pytest.raises(EngineError):
        eng.run(abi.new_query(B, B + 3600, "sum"))   # a rollup query needs a downsampler


@pytest.mark.parametrize("seed", [4, 5])
def test_percentile_and_ordered_over_rollup_avg(eng, seed):
    """A percentile / median group-by and TSDB_QF_ORDERED over rollup avg / count downsampling
    (Sigma sum / Sigma count buckets, Downsampler.java:165-221, under any AggregationIterator):
    the combined buckets are the span values of the selection / ordered fold -- bit for bit."""
    rng = np.random.default_rng(seed)
    rb = random_table(rng, 40, 4, 2, floats=seed == 5)
    eng.load_rollup(rb)
    end = B + 86400 + 7200
    for ds in ("10m-avg", "1h-avg", "1h-count", "30m-avg-nan", "20m-count-zero"):
        for agg, flags in (("p99", 0), ("median", 0), ("p50", 0), ("ep90r7", 0), ("sum", abi.QF_ORDERED),
                           ("avg", abi.QF_ORDERED), ("dev", abi.QF_ORDERED)):
            for rate in (False, True):
                q = _q(ds, agg, start=B + 600, end=end, rate=rate)
                q.flags = flags
                tol = 1e-9 if agg == "dev" else 0.0
                assert_groups_match(eng.run(q), O.run_rollup_query(rb, q), agg, tol=tol,
                                    ctx=f"{ds} {agg} flags={flags} rate={rate}")


def test_run_multi_over_rollup(eng):
    """tsdbhip_run_multi over a rollup table: each sub-query as tsdbhip_run answers it."""
    rng = np.random.default_rng(21)
    rb = random_table(rng, 30, 3, 2)
    eng.load_rollup(rb)
    qs = [_q("1h-avg", a, end=B + 86400) for a in ("sum", "avg", "count", "p90", "max")]
    got = eng.run_multi(qs)
    for q, g in zip(qs, got):
        w = eng.run(q)
        assert len(g) == len(w)
        for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(g, w):
            assert g1 == g2
            np.testing.assert_array_equal(t1, t2)
            np.testing.assert_array_equal(b1, b2)
            np.testing.assert_array_equal(i1, i2)


def random_table(rng, n_series, n_groups, days, p_sum=0.9, p_cnt=0.9, floats=False, counts=True,
                 interval="10m", span="6h", cnt_hi=40):
    """Rollup rows of n_series series over `days` days with cells missing at random."""
    iv = _iv(interval, span)
    step = iv.interval_s
    slots = {}   # rollup row base -> offsets, as addAggregatePoint files them
    for t in range(B, B + days * 86400, step):
        base = engine.rollup_basetime(t, iv)
        slots.setdefault(base, []).append((t - base) // step)
    rows = []
    for s in range(n_series):
        rr = []
        for base, offs in slots.items():
            n = len(offs)
            has_v = rng.random(n) < p_sum
            has_c = rng.random(n) < p_cnt
            fv = rng.normal(100, 50, n)
            iv_ = rng.integers(-1000, 100000, n)
            cv = rng.integers(0, cnt_hi, n)
            vals, cnts = [], []
            for j, o in enumerate(offs):
                if has_v[j]:
                    vals.append((o, 0xF, struct.pack(">d", float(fv[j]))) if floats else
                                (o, 0x7, struct.pack(">q", int(iv_[j]))))
                if counts and has_c[j]:
                    cnts.append((o, 0x0, struct.pack(">b", int(cv[j]))) if cv[j] < 128 else
                                (o, 0x1, struct.pack(">h", int(cv[j]))))
            if vals or cnts:
                rr.append((base, vals, cnts))
        rows.append(rr)
    groups = [int(x) for x in rng.integers(0, n_groups, n_series)]
    return _batch(rows, counts=counts, groups=groups, iv=iv)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("floats", [False, True])
def test_random_tables(eng, seed, floats):
    rng = np.random.default_rng(seed * 7 + floats)
    rb = random_table(rng, 24, 5, 3, floats=floats)
    eng.load_rollup(rb)
    end = B + 2 * 86400 + 3600
    for ds in ("10m-avg", "30m-avg", "1h-count", "10m-count-zero", "20m-avg-nan", "1h-sum", "10m-max",
               "30m-min", "1h-zimsum", "1h-avg-null", "1d-avg"):
        for agg in ("avg", "sum", "count", "max", "none", "dev", "zimsum"):
            for rate in (False, True):
                q = _q(ds, agg, start=B + 1800, end=end, rate=rate)
                g = eng.run(q)
                w = O.run_rollup_query(rb, q)
                fn = ds.split("-")[1]
                exact = fn in ("max", "min", "count") and agg in ("max", "min", "none") and not rate
                tol = 0.0 if exact else (1e-9 if agg == "dev" else 1e-12)
                assert_groups_match(g, w, agg, tol=tol, ctx=f"{ds} {agg} rate={rate}")


def test_no_counts_table(eng):
    rng = np.random.default_rng(11)
    rb = random_table(rng, 16, 3, 2, counts=False)
    eng.load_rollup(rb)
    for ds, agg in (("10m-avg", "sum"), ("1h-count", "sum"), ("30m-sum", "avg"), ("1h-max", "max"),
                    ("10m-avg", "none")):
        q = _q(ds, agg, end=B + 86400 * 2)
        assert_groups_match(eng.run(q), O.run_rollup_query(rb, q), agg, tol=1e-12, ctx=f"{ds} {agg}")


def test_hour_and_day_tables(eng):
    rng = np.random.default_rng(5)
    for interval, span, days, ds in (("1h", "1d", 6, "1h-avg"), ("1h", "1d", 6, "6h-count"), ("1d", "1n", 70, "1d-avg"),
                                     ("1d", "1n", 70, "7d-sum")):
        rb = random_table(rng, 8, 2, days, interval=interval, span=span)
        q = _q(ds, "avg", start=B, end=B + days * 86400)
        assert_groups_match(eng.run_rollup_batch(rb, q), O.run_rollup_query(rb, q), "avg", tol=1e-12,
                            ctx=f"{interval} {ds}")


def test_larger_table_properties(eng):
    """1,000 series x 4 days of 10m rollups against the oracle: avg and count downsampling."""
    rng = np.random.default_rng(99)
    rb = random_table(rng, 1000, 40, 4, p_sum=0.97, p_cnt=0.97)
    eng.load_rollup(rb)
    q = _q("1h-avg", "avg", start=B, end=B + 4 * 86400)
    got = eng.run(q)
    want = O.run_rollup_query(rb, q)
    assert_groups_match(got, want, "avg", tol=1e-12, ctx="1000 series")
    q = _q("1d-count", "sum", start=B, end=B + 4 * 86400)
    got = eng.run(q)
    want = O.run_rollup_query(rb, q)
    assert_groups_match(got, want, "sum", tol=0.0, ctx="1000 series count")


@pytest.mark.parametrize("cnt_hi", [40, 3000])
def test_fused_avg_count_stage(eng, monkeypatch, cnt_hi):
    """Rollup avg / count downsampling over full-mantissa sums: k_seq_rows_ro (a value row with its
    lock-step count row, combined in place) bit-identical to the separate passes + k_rollup_combine
    (option RO_FUSE = 0) and within the oracle's tolerance; counts up to 3000 make count rows of
    mixed 1- and 2-byte cells, which hand their series back (k_seq_dense + the list combine)."""
    rng = np.random.default_rng(17 + cnt_hi)
    rb = random_table(rng, 40, 4, 2, floats=True, cnt_hi=cnt_hi)
    eng.load_rollup(rb)
    for ds in ("10m-avg", "1h-avg", "30m-count", "20m-avg-nan", "1d-avg"):
        for agg in ("sum", "none", "p90"):
            q = _q(ds, agg, start=B + 1800, end=B + 2 * 86400)
            res = {}
            for fuse in ("1", "0"):
                set_option("RO_FUSE", fuse)
                res[fuse] = eng.run(q)
            assert len(res["1"]) == len(res["0"])
            for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(res["1"], res["0"]):
                assert g1 == g2
                np.testing.assert_array_equal(t1, t2, err_msg=f"{ds} {agg}")
                np.testing.assert_array_equal(b1, b2, err_msg=f"{ds} {agg}: fused vs separate passes")
                np.testing.assert_array_equal(i1, i2, err_msg=f"{ds} {agg}")
            assert_groups_match(res["1"], O.run_rollup_query(rb, q), agg, tol=1e-12, ctx=f"{ds} {agg}")


@pytest.mark.parametrize("p_cell", [1.0, 0.97])
@pytest.mark.parametrize("floats", [False, True])
def test_pair_runs_equal_packed_pairs(eng, p_cell, floats):
    """Hour rows read as runs (RoRun: one descriptor a series' run of equal-shape rows and a run id
    a row) give the answers of the packed 24-B pairs (option RO_RUNS = 0), bit for bit, and the
    oracle's; rows with every cell present form one run a series, rows with cells missing at random
    mostly runs of one row (the pairs are then kept)."""
    rng = np.random.default_rng(31 + int(p_cell * 100) + floats)
    rb = random_table(rng, 300, 7, 2, p_sum=p_cell, p_cnt=p_cell, floats=floats, span="1d")
    try:
        res = {}
        for runs in ("-1", "0"):
            set_option("RO_RUNS", runs)
            eng.load_rollup(rb)
            for ds, agg in (("1h-avg", "sum"), ("1h-count", "sum"), ("30m-sum", "max"), ("1h-max", "none"),
                            ("1h-avg", "p90"), ("2h-min", "avg")):
                q = _q(ds, agg, start=B + 1800, end=B + 2 * 86400 - 3600)
                res[(runs, ds, agg)] = eng.run(q)
        for (runs, ds, agg), got in res.items():
            if runs != "-1":
                continue
            ref = res[("0", ds, agg)]
            assert len(got) == len(ref)
            for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(got, ref):
                assert g1 == g2
                np.testing.assert_array_equal(t1, t2, err_msg=f"{ds} {agg}")
                np.testing.assert_array_equal(b1, b2, err_msg=f"{ds} {agg}: runs vs packed pairs")
                np.testing.assert_array_equal(i1, i2, err_msg=f"{ds} {agg}")
            q = _q(ds, agg, start=B + 1800, end=B + 2 * 86400 - 3600)
            assert_groups_match(got, O.run_rollup_query(rb, q), agg, tol=1e-12, ctx=f"runs {ds} {agg}")
    finally:
        set_option("RO_RUNS", "-1")


@pytest.mark.parametrize("floats", [False, True])
def test_emit_half_waves_equal_full_waves(eng, floats):
    """The group-by over stored buckets with K <= 32 takes two series a step (k_emit_reg2: each
    half wave one series, the lower half folding both in series order): bit-identical to one series
    a step (option EMIT_HALF = 0) for every group-by aggregator, with cells missing at random (LERP
    across holes), fill policies and percentile / median group-bys of the stored buckets."""
    rng = np.random.default_rng(57 + floats)
    rb = random_table(rng, 150, 5, 2, p_sum=0.8, p_cnt=0.9, floats=floats, span="1d")
    eng.load_rollup(rb)
    specs = [("1h-avg", a) for a in ("sum", "avg", "min", "max", "dev", "count", "zimsum", "mimmax", "first",
                                     "last", "p90", "median")]
    specs += [("1h-avg-zero", "sum"), ("1h-avg-nan", "avg"), ("2h-count", "sum"), ("30m-sum", "max")]
    try:
        for ds, agg in specs:
            q = _q(ds, agg, start=B + 1800, end=B + 2 * 86400 - 3600)
            set_option("EMIT_HALF", None)
            got = eng.run(q)
            set_option("EMIT_HALF", 0)
            ref = eng.run(q)
            assert len(got) == len(ref)
            for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(got, ref):
                assert g1 == g2
                np.testing.assert_array_equal(t1, t2, err_msg=f"{ds} {agg}")
                np.testing.assert_array_equal(b1, b2, err_msg=f"{ds} {agg}: half waves vs full waves")
                np.testing.assert_array_equal(i1, i2, err_msg=f"{ds} {agg}")
    finally:
        set_option("EMIT_HALF", None)
