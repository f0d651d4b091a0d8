"""Rollup reads over several GPUs (SURVEY.md 8e x 8f row f2).

A rollup scan (tsdbhip_load_rollup) shards like a raw one:
  * the multi-device context splits it by SpanGroups (every query local, results concatenated:
    bit for bit against one GPU) or by series (partial states / span contributions gathered to
    devices[0] -- whose merge context holds an empty batch of the same rollup table, so the
    plans agree: rollup scan bounds, count group-by planned as sum);
  * one process per GPU loads dist.shard_rollup_batch(rb, rank, world) and runs the partials
    (tsdbhip_run_partials / tsdbhip_finalize) or percentile (tsdbhip_sel_*) exchange.
Every answer is checked against the one-GPU run and the oracle's RollupSeq restatement
(oracle.run_rollup_query).  N devices are emulated by repeating device 0."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, dist
from opentsdb_amd import engine as E
from oracle import oracle as O
from tests.test_gpu_dist import run_sharded_sel
from tests.test_gpu_multidev import bit_same
from tests.test_gpu_parity import assert_groups_match
from tests.test_gpu_rollup_read import B, _q, random_table

pytestmark = pytest.mark.gpu

END = B + 2 * 86400 + 3600
# (downsample, group-by aggregator, kind): avg / count downsampling combine the count cells
QUERIES = [("10m-avg", "avg", "partials"), ("1h-count", "sum", "partials"), ("30m-sum", "count", "partials"),
           ("1h-max", "max", "partials"), ("20m-avg-nan", "sum", "partials"), ("1h-zimsum", "min", "partials"),
           ("1h-max", "p99", "sel"), ("30m-min", "median", "sel"), ("10m-avg", "none", "none")]
IDS = [f"{a}:{d}" for d, a, _ in QUERIES]


@pytest.fixture(scope="module")
def table():
    rng = np.random.default_rng(2024)
    return random_table(rng, 40, 6, 3, floats=True)


@pytest.fixture(scope="module")
def single(table):
    e = E.Engine(0)
    e.load_rollup(table)
    want = {f"{a}:{d}": e.run(_q(d, a, start=B + 1800, end=END)) for d, a, _ in QUERIES}
    yield e, want
    e.close()


@pytest.mark.parametrize("world", [2, 3])
def test_md_rollup_group_shards_bit_identical(table, single, world):
    _, want = single
    e = E.Engine(devices=[0] * world)
    try:
        e.shard_mode(E.SHARD_GROUPS)
        e.load_rollup(table)
        nd, _, mode, per = e.md_info()
        assert (nd, mode) == (world, E.SHARD_GROUPS) and int(per.sum()) > 0
        for (d, a, _), name in zip(QUERIES, IDS):
            bit_same(e.run(_q(d, a, start=B + 1800, end=END)), want[name], f"rollup groups x{world} {name}")
    finally:
        e.close()


@pytest.mark.parametrize("world", [2, 4])
def test_md_rollup_series_shards(table, single, world):
    """Groups straddle devices: partials within the oracle's tolerance (and against one GPU),
    order statistics and NONE bit for bit."""
    _, want = single
    e = E.Engine(devices=[0] * world)
    try:
        e.shard_mode(E.SHARD_SERIES)
        e.load_rollup(table)
        assert e.md_info()[2] == E.SHARD_SERIES
        for (d, a, kind), name in zip(QUERIES, IDS):
            q = _q(d, a, start=B + 1800, end=END)
            got = e.run(q)
            if kind == "partials":
                agg = "sum" if a == "count" else a
                assert_groups_match(got, O.run_rollup_query(table, q), agg, tol=1e-12, ctx=f"rollup series x{world} {name}")
                assert_groups_match(got, want[name], agg, tol=1e-12, ctx=f"rollup series x{world} {name} vs one GPU")
            else:
                bit_same(got, want[name], f"rollup series x{world} {name}")
        assert e.timing().exchange_ms > 0
    finally:
        e.close()


def test_md_load_after_rollup_resets_merge_context(table):
    """A raw load after a rollup load: the merge context plans raw queries again."""
    from opentsdb_amd import synth
    b = synth.generate(60, B, 360, 10000, value_kind=2, n_groups=5, int_mod=3000, seed=7)
    one = E.Engine(0)
    e = E.Engine(devices=[0, 0])
    try:
        e.shard_mode(E.SHARD_SERIES)
        e.load_rollup(table)
        e.load(b)
        one.load(b)
        q = abi.new_query(B, B + 3599, "count", ds_function=abi.AGG["sum"], ds_interval_ms=60000)
        bit_same(e.run(q), one.run(q), "raw after rollup")
    finally:
        e.close()
        one.close()


@pytest.fixture(scope="module")
def engines():
    es = [E.Engine(0) for _ in range(4)]
    yield es
    for e in es:
        e.close()


def run_rank_partials(engines, rb, q, world):
    G = dist.n_groups_of(rb.cells)
    bufs = []
    for r in range(world):
        eng = engines[r]
        eng.load_rollup(dist.shard_rollup_batch(rb, r, world))
        lay = eng.partials_layout(q, G)
        buf = np.zeros(int(lay.bytes), np.uint8)
        eng.run_partials(q, G, buf.ctypes.data)
        bufs.append(buf)
    gathered = np.concatenate(bufs)   # (kept alive across the call: .ctypes.data is a bare address)
    return engines[0].finalize(q, G, gathered.ctypes.data, world)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_rank_shards_partials(engines, table, world):
    """One context per rank, each with its rollup shard: the partials exchange."""
    for d, a, kind in QUERIES:
        if kind != "partials":
            continue
        q = _q(d, a, start=B + 1800, end=END)
        agg = "sum" if a == "count" else a
        assert_groups_match(run_rank_partials(engines, table, q, world), O.run_rollup_query(table, q), agg,
                            tol=1e-12, ctx=f"rollup ranks x{world} {a}:{d}")


@pytest.mark.parametrize("world", [2, 3])
def test_rank_shards_percentile_group(engines, table, world):
    """The percentile group-by exchange over rollup shards (the count series stay local)."""
    for d, a, kind in QUERIES:
        if kind != "sel":
            continue
        q = _q(d, a, start=B + 1800, end=END)
        loaders = []

        class Shim:   # run_sharded_sel calls e.load(shard): route it to the rollup loader
            def __init__(self, eng, r):
                self.eng, self.r = eng, r

            def load(self, _):
                self.eng.load_rollup(dist.shard_rollup_batch(table, self.r, world))

            def __getattr__(self, k):
                return getattr(self.eng, k)

        loaders = [Shim(engines[r], r) for r in range(world)]
        got = run_sharded_sel(loaders, table.cells, q, world)
        assert_groups_match(got, O.run_rollup_query(table, q), a, tol=0.0, ctx=f"rollup sel ranks x{world} {a}:{d}")


def test_group_shards_by_rank(engines, table):
    """dist.shard_rollup_batch(by_group=True): whole groups per rank, results concatenated."""
    q = _q("10m-avg", "avg", start=B + 1800, end=END)
    parts = []
    for r in range(3):
        engines[r].load_rollup(dist.shard_rollup_batch(table, r, 3, by_group=True))
        parts.append(engines[r].run(q))
    assert_groups_match(dist.merge_group_results(parts), O.run_rollup_query(table, q), "avg", tol=1e-12,
                        ctx="rollup group shards")
