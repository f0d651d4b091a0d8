"""Multi-GPU exchange on the device: shards reduced by separate libtsdbhip contexts,
partial states merged in rank order by tsdbhip_finalize, checked against the oracle over
the whole (unsharded) batch.

Ranks are emulated by several contexts on cuda:0 (the round-end 8-GPU run uses one
process per GPU with RCCL; tests/test_dist_cpu.py covers the gloo exchange itself), plus
one real 2-process gloo run through opentsdb_amd/dist.run_distributed."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from opentsdb_amd import abi, dist, synth
from oracle import oracle as O
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

T0 = 1356998400


@pytest.fixture(scope="module")
def engines():
    from opentsdb_amd.engine import Engine
    es = [Engine(0) for _ in range(8)]
    yield es
    for e in es:
        e.close()


@pytest.fixture(scope="module")
def batch():
    return synth.generate(150, T0, 360, 10000, value_kind=2, n_groups=7, int_mod=30000, seed=0x5EED)


def run_sharded(engines, b, q, world):
    G = dist.n_groups_of(b)
    bufs = []
    for r in range(world):
        e = engines[r]
        e.load(dist.shard_batch(b, r, world))
        lay = e.partials_layout(q, G)
        buf = np.zeros(int(lay.bytes), np.uint8)
        e.run_partials(q, G, buf.ctypes.data)
        bufs.append(buf)
    gathered = np.concatenate(bufs)
    return engines[0].finalize(q, G, gathered.ctypes.data, world)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("agg", ["sum", "avg", "min", "max", "count", "dev", "first", "last", "diff", "zimsum",
                                 "mimmax", "pfsum"])
def test_sharded_equals_oracle(engines, batch, world, agg):
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    assert_groups_match(run_sharded(engines, batch, q, world), O.run_query(batch, q), agg, ctx=f"{agg} x{world}")


@pytest.mark.parametrize("world", [1, 3])
@pytest.mark.parametrize("ds_ms", [60000, 600000])
def test_run_partials_multi_equals_separate(engines, batch, world, ds_ms):
    """tsdbhip_run_partials_multi: the shard's partial states of six queries from one fused pass,
    byte for byte those of six tsdbhip_run_partials calls; a mix the fused pass does not take
    (first, a rate) runs query by query with the same bytes."""
    G = dist.n_groups_of(batch)
    mixes = [["sum", "avg", "min", "max", "count", "dev"], ["sum", "first", "dev"]]
    for aggs in mixes:
        qs = [abi.new_query(T0, T0 + 3599, a, ds_function=abi.AGG["avg"], ds_interval_ms=ds_ms) for a in aggs]
        for r in range(world):
            e = engines[r]
            e.load(dist.shard_batch(batch, r, world))
            nb = int(e.partials_layout(qs[0], G).bytes)
            sep = np.zeros(nb * len(qs), np.uint8)
            for i, q in enumerate(qs):
                e.run_partials(q, G, sep.ctypes.data + i * nb)
            fused = np.full(nb * len(qs), 0xAB, np.uint8)
            e.run_partials_multi(qs, G, fused.ctypes.data)
            if aggs == mixes[0]:
                assert e.timing().fused_queries == len(qs)
            np.testing.assert_array_equal(fused, sep, err_msg=f"{aggs} rank {r}/{world}")


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_fill_rate_all(engines, batch, world):
    cases = [
        ("sum", dict(ds_function=abi.AGG["sum"], ds_interval_ms=60000, ds_fill=abi.FILL_NAN)),
        ("avg", dict(ds_function=abi.AGG["max"], ds_interval_ms=300000, ds_fill=abi.FILL_ZERO)),
        ("sum", dict(ds_function=abi.AGG["avg"], ds_interval_ms=60000, rate=True)),
        ("sum", dict(ds_function=abi.AGG["sum"], ds_all=True)),
    ]
    for agg, kw in cases:
        q = abi.new_query(T0, T0 + 3599, agg, **kw)
        assert_groups_match(run_sharded(engines, batch, q, world), O.run_query(batch, q), agg, ctx=f"{kw} x{world}")


def test_group_on_one_rank_only(engines):
    """More ranks than groups: most ranks hold no span of most groups."""
    b = synth.generate(12, T0, 360, 10000, value_kind=0, n_groups=2, seed=3)
    for agg in ["min", "max", "sum", "dev"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        assert_groups_match(run_sharded(engines, b, q, 4), O.run_query(b, q), agg, ctx=agg)


def _worker(rank, world, port, out):
    import torch.distributed as td
    from opentsdb_amd.engine import Engine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(0)
    try:
        b = synth.generate(150, T0, 360, 10000, value_kind=2, n_groups=7, int_mod=30000, seed=0x5EED)
        eng.load(dist.shard_batch(b, rank, world))
        q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        groups = dist.run_distributed(eng, q, td, dist.n_groups_of(b))
        _save(os.path.join(out, f"r{rank}.npz"), groups)
        qs = [abi.new_query(T0, T0 + 3599, a, ds_function=abi.AGG["avg"], ds_interval_ms=60000) for a in MULTI]
        for a, gs in zip(MULTI, dist.run_distributed_multi(eng, qs, td, dist.n_groups_of(b))):
            _save(os.path.join(out, f"r{rank}_{a}.npz"), gs)
    finally:
        eng.close()
        td.destroy_process_group()


MULTI = ["avg", "min", "max", "count", "dev"]


def _save(path, groups):
    np.savez(path, gid=np.array([g[0] for g in groups]), n=np.array([len(g[1]) for g in groups]),
             ts=np.concatenate([g[1] for g in groups]), bits=np.concatenate([g[2] for g in groups]),
             isi=np.concatenate([g[3] for g in groups]))


def _load(path):
    z = np.load(path)
    cut = np.concatenate([[0], np.cumsum(z["n"])])
    return [(int(z["gid"][i]), z["ts"][cut[i]:cut[i + 1]], z["bits"][cut[i]:cut[i + 1]], z["isi"][cut[i]:cut[i + 1]])
            for i in range(len(z["gid"]))]


def test_two_process_gloo(tmp_path, batch):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    want = O.run_query(batch, q)
    for r in range(2):
        assert_groups_match(_load(tmp_path / f"r{r}.npz"), want, "sum", ctx=f"gloo rank {r}")
        # run_distributed_multi: one fused pass + one all-gather for the five queries
        for a in MULTI:
            qa = abi.new_query(T0, T0 + 3599, a, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
            assert_groups_match(_load(tmp_path / f"r{r}_{a}.npz"), O.run_query(batch, qa), a, ctx=f"gloo multi {a} rank {r}")


# ---- percentile / median group-by: values to the owning rank ----------
def run_sharded_sel(engines, b, q, world):
    """run_distributed_sel with the collectives done in-process (one context per rank)."""
    import torch
    G = dist.n_groups_of(b)
    vals, counts, unis, acts = [], [], [], []
    K = 0
    for r in range(world):
        e = engines[r]
        e.load(dist.shard_batch(b, r, world))
        c, K = e.sel_layout(q, G)
        v = np.zeros(max(1, int(c.sum()) * K))
        u = np.zeros(max(1, G * K), np.uint8)
        a = np.zeros(max(1, G), np.int32)
        e.sel_run_values(q, G, v.ctypes.data, u.ctypes.data, a.ctypes.data)
        vals.append(torch.from_numpy(v[:int(c.sum()) * K]))
        counts.append(c)
        unis.append(u)
        acts.append(a)
    uni = np.maximum.reduce(unis)
    act = np.maximum.reduce(acts)
    counts_all = np.stack(counts)
    own = dist.sel_owner(counts_all)
    sends = [dist.sel_pack(vals[r], counts[r], K, own, r, world) for r in range(world)]
    rows_v, rows_f = [], []
    for me in range(world):
        pieces = []
        for r in range(world):
            send, splits = sends[r]
            off = int(sum(splits[:me]))
            pieces.append(send[off:off + splits[me]])
        ov, seg = dist.sel_unpack(torch.cat(pieces), counts_all, K, me, vals[me])
        ov = np.ascontiguousarray(ov.numpy())
        out_v = np.zeros(max(1, G * K))
        out_f = np.zeros(max(1, G * K), np.uint8)
        engines[me].sel_select(q, G, ov.ctypes.data, seg, uni.ctypes.data, out_v.ctypes.data, out_f.ctypes.data)
        rows_v.append(out_v)
        rows_f.append(out_f)
    val = np.ascontiguousarray(dist.sel_combine(torch.from_numpy(np.stack(rows_v)).reshape(-1), G, K, own).numpy())
    flag = np.ascontiguousarray(dist.sel_combine(torch.from_numpy(np.stack(rows_f)).reshape(-1), G, K, own).numpy())
    return engines[0].assemble(q, G, val.ctypes.data, flag.ctypes.data, act.ctypes.data)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("agg,ds", [("p99", "avg"), ("p50", "max"), ("median", "sum"), ("p90", "p99"),
                                    ("ep95r7", "avg")])
def test_sharded_percentile_group_equals_oracle(engines, batch, world, agg, ds):
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG[ds], ds_interval_ms=60000)
    assert_groups_match(run_sharded_sel(engines, batch, q, world), O.run_query(batch, q), agg, tol=0.0,
                        ctx=f"{agg}:{ds} x{world}")


def test_sharded_percentile_group_rate_fill(engines, batch):
    for kw in [dict(ds_function=abi.AGG["avg"], ds_interval_ms=60000, rate=True),
               dict(ds_function=abi.AGG["sum"], ds_interval_ms=300000, ds_fill=abi.FILL_NAN)]:
        q = abi.new_query(T0, T0 + 3599, "p75", **kw)
        assert_groups_match(run_sharded_sel(engines, batch, q, 3), O.run_query(batch, q), "p75", tol=0.0, ctx=str(kw))


def _sel_worker(rank, world, port, out):
    import torch.distributed as td
    from opentsdb_amd.engine import Engine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(0)
    try:
        b = synth.generate(150, T0, 360, 10000, value_kind=2, n_groups=7, int_mod=30000, seed=0x5EED)
        eng.load(dist.shard_batch(b, rank, world))
        q = abi.new_query(T0, T0 + 3599, "p99", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        groups = dist.run_distributed_sel(eng, q, td, dist.n_groups_of(b))
        np.savez(os.path.join(out, f"p{rank}.npz"), gid=np.array([g[0] for g in groups]),
                 n=np.array([len(g[1]) for g in groups]), ts=np.concatenate([g[1] for g in groups]),
                 bits=np.concatenate([g[2] for g in groups]), isi=np.concatenate([g[3] for g in groups]))
    finally:
        eng.close()
        td.destroy_process_group()


def test_two_process_gloo_percentile(tmp_path, batch):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_sel_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    q = abi.new_query(T0, T0 + 3599, "p99", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    want = O.run_query(batch, q)
    for r in range(2):
        z = np.load(tmp_path / f"p{r}.npz")
        cut = np.concatenate([[0], np.cumsum(z["n"])])
        got = [(int(z["gid"][i]), z["ts"][cut[i]:cut[i + 1]], z["bits"][cut[i]:cut[i + 1]], z["isi"][cut[i]:cut[i + 1]])
               for i in range(len(z["gid"]))]
        assert_groups_match(got, want, "p99", tol=0.0, ctx=f"gloo rank {r}")


# ---- raw (no-downsampling) queries: whole groups per rank ---------------------------
@pytest.fixture(scope="module")
def raw_batch():
    from tests.test_gpu_raw import random_batch
    return random_batch(21, n_series=60, n_groups=5)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("agg", ["sum", "avg", "min", "max", "dev", "zimsum", "mimmax", "first", "diff", "pfsum",
                                 "p99", "ep90r3", "median"])
def test_group_sharded_raw_equals_oracle(engines, raw_batch, world, agg):
    q = abi.new_query(T0, T0 + 7199, agg)
    parts = []
    for r in range(world):
        parts.append(engines[r].run_batch(dist.shard_batch_by_group(raw_batch, r, world), q))
    assert_groups_match(dist.merge_group_results(parts), O.run_query(raw_batch, q), agg, tol=0.0,
                        ctx=f"{agg} x{world}")


def test_group_sharded_raw_counters_rate(engines):
    b = synth.generate_counters(80, T0, 120, n_groups=6, seed=9)
    for kw in [dict(rate=True, counter=True, counter_max=1 << 32, reset_value=1000000), dict()]:
        q = abi.new_query(T0, T0 + 3599, "sum", **kw)
        parts = [engines[r].run_batch(dist.shard_batch_by_group(b, r, 3), q) for r in range(3)]
        assert_groups_match(dist.merge_group_results(parts), O.run_query(b, q), "sum", tol=0.0, ctx=str(kw))


def _raw_worker(rank, world, port, out):
    import torch.distributed as td
    from opentsdb_amd.engine import Engine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    eng = Engine(0)
    try:
        b = synth.generate_counters(80, T0, 120, n_groups=6, seed=9)
        eng.load(dist.shard_batch_by_group(b, rank, world))
        q = abi.new_query(T0, T0 + 3599, "sum")
        groups = dist.run_distributed_raw(eng, q, td)
        np.savez(os.path.join(out, f"w{rank}.npz"), gid=np.array([g[0] for g in groups]),
                 n=np.array([len(g[1]) for g in groups]), ts=np.concatenate([g[1] for g in groups]),
                 bits=np.concatenate([g[2] for g in groups]), isi=np.concatenate([g[3] for g in groups]))
    finally:
        eng.close()
        td.destroy_process_group()


def test_two_process_gloo_raw(tmp_path):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_raw_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    b = synth.generate_counters(80, T0, 120, n_groups=6, seed=9)
    want = O.run_query(b, abi.new_query(T0, T0 + 3599, "sum"))
    for r in range(2):
        z = np.load(tmp_path / f"w{r}.npz")
        cut = np.concatenate([[0], np.cumsum(z["n"])])
        got = [(int(z["gid"][i]), z["ts"][cut[i]:cut[i + 1]], z["bits"][cut[i]:cut[i + 1]], z["isi"][cut[i]:cut[i + 1]])
               for i in range(len(z["gid"]))]
        assert_groups_match(got, want, "sum", tol=0.0, ctx=f"gloo raw rank {r}")


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("agg", ["sum", "avg", "dev", "squareSum"])
def test_sharded_ordered_bit_exact(engines, batch, world, agg):
    """TSDB_QF_ORDERED over ranks: span values to the owner, folded in rank (= span) order."""
    q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000, flags=abi.QF_ORDERED)
    assert_groups_match(run_sharded_sel(engines, batch, q, world), O.run_query(batch, q), agg, tol=0.0,
                        ctx=f"ordered {agg} x{world}")


# ---- NONE aggregator: span-sharded, results concatenated in rank order -----------------
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_span_sharded_none_equals_oracle(engines, batch, raw_batch, world):
    for b, q in [(batch, abi.new_query(T0, T0 + 3599, "none", ds_function=abi.AGG["avg"], ds_interval_ms=60000)),
                 (raw_batch, abi.new_query(T0, T0 + 7199, "none"))]:
        parts = [engines[r].run_batch(dist.shard_batch_spans(b, r, world), q) for r in range(world)]
        assert_groups_match(dist.merge_none_results(parts), O.run_query(b, q), "none", tol=0.0, ctx=f"none x{world}")


# ---- the library's sharding: tsdbhip_load_shard / tsdbhip_synth_shard -------------------
def run_lib_sharded(engines, b, q, world):
    G = dist.n_groups_of(b)
    bufs = []
    for r in range(world):
        e = engines[r]
        dist.load_rank_shard(e, b, r, world, "series")
        lay = e.partials_layout(q, G)
        buf = np.zeros(int(lay.bytes), np.uint8)
        e.run_partials(q, G, buf.ctypes.data)
        bufs.append(buf)
    gathered = np.concatenate(bufs)   # (kept alive while finalize reads it)
    return engines[0].finalize(q, G, gathered.ctypes.data, world)


@pytest.mark.parametrize("world", [2, 8])
def test_library_shards_equal_python_shards(engines, batch, world):
    """tsdbhip_load_shard over the host batch == loading dist.shard_batch's copy, bit for bit
    (run_partials + finalize), and both equal the oracle."""
    for agg in ["sum", "max", "dev"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        lib = run_lib_sharded(engines, batch, q, world)
        py = run_sharded(engines, batch, q, world)
        for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(lib, py):
            assert g1 == g2
            np.testing.assert_array_equal(b1, b2)
        assert_groups_match(lib, O.run_query(batch, q), agg, ctx=f"lib shards {agg} x{world}")


def test_library_group_and_span_shards(engines, raw_batch):
    q = abi.new_query(T0, T0 + 7199, "sum")
    parts = []
    for r in range(4):
        dist.load_rank_shard(engines[r], raw_batch, r, 4, "groups")
        parts.append(engines[r].run(q))
    assert_groups_match(dist.merge_group_results(parts), O.run_query(raw_batch, q), "sum", tol=0.0, ctx="groups")
    qn = abi.new_query(T0, T0 + 7199, "none")
    parts = []
    for r in range(3):
        dist.load_rank_shard(engines[r], raw_batch, r, 3, "spans")
        parts.append(engines[r].run(qn))
    assert_groups_match(dist.merge_none_results(parts), O.run_query(raw_batch, qn), "none", tol=0.0, ctx="spans")


@pytest.mark.parametrize("world", [2, 3, 8])
def test_synth_shards_concatenate_to_the_store(engines, world):
    """tsdbhip_synth_shard: rank r generates batch positions [b_r, b_r+1) of the one global
    store; the shards' bytes are the store's, and the sharded query equals the oracle."""
    args = (203, T0, 360, 10000, 2, 7, 30000, 0x5EED)
    engines[0].synth(*args)
    whole = engines[0].download()
    bounds = dist.synth_bounds(args[0], world)
    G = args[5]
    q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    bufs = []
    quals, gids = [], []
    for r in range(world):
        e = engines[r]
        e.synth_shard(bounds[r], bounds[r + 1], *args)
        sh = e.download()
        quals.append(sh.qual)
        gids.append(sh.group_id)
        lay = e.partials_layout(q, G)
        buf = np.zeros(int(lay.bytes), np.uint8)
        e.run_partials(q, G, buf.ctypes.data)
        bufs.append(buf)
    np.testing.assert_array_equal(np.concatenate(quals), whole.qual)
    np.testing.assert_array_equal(np.concatenate(gids), whole.group_id)
    gathered = np.concatenate(bufs)
    got = engines[0].finalize(q, G, gathered.ctypes.data, world)
    assert_groups_match(got, O.run_query(whole, q), "sum", ctx=f"synth shards x{world}")
