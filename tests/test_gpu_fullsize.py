"""GPU parity at the real sizes of BASELINE configs 3, 4 and 5, against the CPU oracle.

The engine runs each query over the WHOLE store resident in HBM (so every kernel walks row
offsets far past 2^31 and 2^32 bytes); the oracle then runs the same query over a slice of
the store downloaded from the device (tsdbhip_batch_download_range): whole groups picked with
a stride that includes the last group (the highest offsets), or single series for the NONE
aggregator.  A group's result depends only on its own spans, so the oracle's answer for the
slice is the reference's answer for those groups of the full store.

* config 3, 1-GPU point: 10M series x 1 h @10 s (even series int [0, 30000), odd float32),
  1000 groups, 18.2 GB -- {sum,avg,min,max,count,dev}:1m-avg one by one and through
  tsdbhip_run_multi, p99:1m-avg (percentile group-by), TSDB_QF_ORDERED sum (bit-exact).
* config 4 at full size: 100k jittered counters x 1 h (ms qualifiers), 64 groups of ~1560
  spans: sum without downsampling (union LERP, long arithmetic), sum:rate{counter,2^32,1e6},
  and p99 without downsampling on one group -- bit-exact.
* config 5, one GPU's shard: 1.25M series x 1 day @10 s float32 (65 GB): none:1h-p99 and
  none:1h-ep99r7 per series on a strided series subset, ORDERED sum:1h-p99 over whole groups
  (bit-exact), and the 1h/1d rollup cells of a strided subset byte for byte.

Reference known answer these configurations scale: test/core/TestTsdbQueryDownsample.java:137-172.
"""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def concat_batches(parts):
    """One host batch of several (series appended in order, group ids kept)."""
    srp, qo, vo = [np.zeros(1, np.int64)], [np.zeros(1, np.uint64)], [np.zeros(1, np.uint64)]
    nr = 0
    qb = vb = 0
    for p in parts:
        srp.append(p.series_row_ptr[1:] + nr)
        qo.append(p.row_qual_off[1:] + np.uint64(qb))
        vo.append(p.row_val_off[1:] + np.uint64(vb))
        nr += p.n_rows
        qb += int(p.row_qual_off[-1])
        vb += int(p.row_val_off[-1])
    return abi.HostBatch(np.concatenate(srp), np.concatenate([p.row_base_time for p in parts]),
                         np.concatenate(qo), np.concatenate(vo),
                         np.concatenate([p.qual[:int(p.row_qual_off[-1])] for p in parts]),
                         np.concatenate([p.val[:int(p.row_val_off[-1])] for p in parts]),
                         np.concatenate([p.group_id for p in parts]))


def group_slice(eng, groups):
    """The resident series of `groups` (whole groups) as one host batch."""
    g = eng.resident_groups()
    assert np.all(np.diff(g) >= 0), "resident order is group-sorted"
    parts = []
    for gid in groups:
        a, b = int(np.searchsorted(g, gid, "left")), int(np.searchsorted(g, gid, "right"))
        assert b > a, gid
        parts.append(eng.download_range(a, b))
    return concat_batches(parts)


def only_groups(res, groups):
    keep = set(int(x) for x in groups)
    return [r for r in res if r[0] in keep]


def check_groups(got, want, agg, groups, tol=None, ctx=""):
    got = only_groups(got, groups)
    assert len(want) == len(groups), f"{ctx}: oracle returned {len(want)} groups"
    assert_groups_match(got, want, agg, tol=tol, ctx=ctx)


def dsq(agg, spec, end, **kw):
    from opentsdb_amd.engine import parse_downsample
    d = parse_downsample(spec)
    return abi.new_query(T0, end, agg, ds_function=d.ds_function, ds_interval_ms=d.ds_interval_ms,
                         ds_fill=d.ds_fill, **kw)


# ---- config 3: 10M series x 360 dp, 1000 groups -------------------------------------------
C3_GROUPS = [int(x) for x in np.linspace(0, 999, 12).round()]   # 0 ... 999 (last = highest offsets)


def test_config3_full_size(eng):
    eng.synth(10_000_000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
    end = T0 + 3599
    aggs = ["sum", "avg", "min", "max", "count", "dev"]
    got = {a: eng.run(dsq(a, "1m-avg", end)) for a in aggs}
    t = eng.timing()
    assert t.datapoints == 3_600_000_000
    multi = eng.run_multi([dsq(a, "1m-avg", end) for a in aggs[1:]])
    assert eng.timing().fused_queries == len(aggs) - 1   # one fused streaming pass
    w0 = eng.debug_sel_window()
    got["p99"] = eng.run(dsq("p99", "1m-avg", end))
    got["median"] = eng.run(dsq("median", "1m-avg", end))
    w1 = eng.debug_sel_window()
    assert (w1[0] - w0[0], w1[1] - w0[1]) == (1, 0), f"sampled-window select runs / misses {w0} -> {w1}"   # (p99; the median keeps the full path)
    ordered = eng.run(dsq("sum", "1m-avg", end, flags=abi.QF_ORDERED))
    host = group_slice(eng, C3_GROUPS)
    assert host.n_series == 10_000 * len(C3_GROUPS)
    for a in aggs + ["p99", "median"]:
        want = O.run_query(host, dsq(a, "1m-avg", end), threads=16)
        assert all(len(w[1]) == 60 for w in want)
        check_groups(got[a], want, a, C3_GROUPS, tol=0.0 if a in ("p99", "median") else None, ctx=f"config3 {a}")
        if a in aggs[1:]:
            check_groups(multi[aggs.index(a) - 1], want, a, C3_GROUPS, ctx=f"config3 run_multi {a}")
        if a == "sum":
            check_groups(ordered, want, a, C3_GROUPS, tol=0.0, ctx="config3 ordered sum (bit-exact)")


# ---- config 3's day on one GPU of eight: 1.25M series x 8640 dp, 1000 groups ------------------
def test_config3_day_shard_full_size(eng):
    """The per-GPU workload of strong-scaled config 3 (bench.py config3_strong at 8 GPUs): 1.25M
    series x 1 day @10 s kept as hour rows (54.6 GB), int/float alternating, 1000 groups.
    {sum,avg,min,max,count,dev}:1m-avg take k_hwin (K = 1440 slots, window by window), the fused
    run_multi takes its MULTI variant and must equal the separate queries bit for bit;
    sum:10m-avg and sum:1h-avg take k_rows.  A strided slice of whole groups against the oracle."""
    eng.synth(1_250_000, T0, 8640, 10000, 2, 1000, 30000, 0x5EED)
    end = T0 + 86400 - 1
    aggs = ["sum", "avg", "min", "max", "count", "dev"]
    got = {}
    for a in aggs:
        got[a] = eng.run(dsq(a, "1m-avg", end))
        t = eng.timing()
        assert t.datapoints == 1_250_000 * 8640 and t.redo_tiles == 0 and t.fast_ms > 0, (a, t.redo_tiles)
    multi = eng.run_multi([dsq(a, "1m-avg", end) for a in aggs])
    assert eng.timing().fused_queries == len(aggs)   # one k_hwin MULTI pass
    for a, m in zip(aggs, multi):
        check_groups(m, got[a], a, sorted(set(r[0] for r in got[a])), tol=0.0, ctx=f"day run_multi {a} vs own pass")
    for spec in ("10m-avg", "1h-avg"):
        got["sum:" + spec] = eng.run(dsq("sum", spec, end))
        assert eng.timing().redo_tiles == 0
    host = group_slice(eng, C3_GROUPS)
    assert host.n_series == 1250 * len(C3_GROUPS)
    for a in aggs:
        want = O.run_query(host, dsq(a, "1m-avg", end), threads=16)
        assert all(len(w[1]) == 1440 for w in want)
        check_groups(got[a], want, a, C3_GROUPS, tol=0.0 if a in ("min", "max", "count") else None,
                     ctx=f"config3 day {a}")
    for spec, k in (("10m-avg", 144), ("1h-avg", 24)):
        want = O.run_query(host, dsq("sum", spec, end), threads=16)
        assert all(len(w[1]) == k for w in want)
        check_groups(got["sum:" + spec], want, "sum", C3_GROUPS, ctx=f"config3 day sum:{spec}")


# ---- config 4: 100k jittered counters x 1 h, 64 groups --------------------------------------
def test_config4_full_size(eng):
    b = synth.generate_counters(100_000, T0, 360, n_groups=64, seed=0x5EED)
    eng.load(b)
    queries = {
        "sum": abi.new_query(T0, T0 + 3599, "sum"),
        "rate": abi.new_query(T0, T0 + 3599, "sum", rate=True, counter=True, counter_max=1 << 32,
                              reset_value=1_000_000),
    }
    got = {k: eng.run(q) for k, q in queries.items()}
    # jitter moves some first / last points into the hour rows either side of the window
    assert 0.99 * 100_000 * 360 < eng.timing().datapoints <= 100_000 * 360
    groups = [0, 21, 42, 63]
    host = group_slice(eng, groups)
    assert host.n_series == int(np.isin(b.group_id, groups).sum())
    del b
    for k, q in queries.items():
        want = O.run_query(host, q, threads=len(groups))
        if k == "sum":   # union of ~1560 jittered spans: ~5.6e5 points per group
            assert all(len(w[1]) > 100_000 for w in want)
        check_groups(got[k], want, "sum", groups, tol=0.0, ctx=f"config4 {k}")
    # percentile group-by per union point (k_raw_vals / k_raw_sel) on the last group
    qp = abi.new_query(T0, T0 + 3599, "p99")
    gp = eng.run(qp)
    one = group_slice(eng, [63])
    check_groups(gp, O.run_query(one, qp), "p99", [63], tol=0.0, ctx="config4 p99")


# ---- config 5: one GPU's shard, 1.25M series x 8640 dp float32 -----------------------------
def test_config5_shard_full_size(eng):
    n = 1_250_000
    eng.synth(n, T0, 8640, 10000, 0, 64, 1, 0x5EED)
    end = T0 + 86399
    assert eng.n_series() == n
    stride = 997
    picks = list(range(0, n, stride)) + [n - 1]
    single = concat_batches([eng.download_range(s, s + 1) for s in picks])
    for fn in ["p99", "ep99r7"]:
        got = eng.run(dsq("none", f"1h-{fn}", end))
        assert eng.timing().datapoints == n * 8640
        assert len(got) == n
        sub = [got[s] for s in picks]
        # the oracle numbers the slice's spans 0..; the engine numbers the store's
        sub = [(j, ts, bits, isi) for j, (_, ts, bits, isi) in enumerate(sub)]
        want = O.run_query(single, dsq("none", f"1h-{fn}", end), threads=16)
        assert all(len(w[1]) == 24 for w in want)
        assert_groups_match(sub, want, "none", tol=0.0, ctx=f"config5 none:1h-{fn}")
        del got, sub
    groups = [0, 63]
    host = group_slice(eng, groups)
    qo = dsq("sum", "1h-p99", end, flags=abi.QF_ORDERED)
    check_groups(eng.run(qo), O.run_query(host, qo, threads=2), "sum", groups, tol=0.0,
                 ctx="config5 ordered sum:1h-p99 (bit-exact)")
    del host
    # rollup generation over the whole shard; the cells of a strided subset byte for byte
    from opentsdb_amd import engine
    from oracle import rollup as R
    cells = eng.rollup(engine.rollup_interval("1h", "1d"), T0, T0 + 86400)
    assert len(cells) == n * 24 * 4
    rpicks = list(range(0, n, 25_013)) + [n - 1]
    sub = concat_batches([eng.download_range(s, s + 1) for s in rpicks])
    exp = R.generate(sub, R.Interval("1h", "1d"), T0, T0 + 86400)
    pos = {s: j for j, s in enumerate(rpicks)}
    sel = np.flatnonzero(np.isin(cells.series, np.array(rpicks, np.int32)))
    got = []
    for i in sel:
        s, base, q, v = cells.cell(int(i))
        got.append((pos[s], base, q, v))
    assert len(got) == len(exp) == len(rpicks) * 24 * 4
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g == e, (i, g, e)
