"""Multi-GPU driver (opentsdb_amd/dist.py) on CPU: sharding and the gloo exchange step.

The per-rank partial states come from the GPU (tsdbhip_run_partials); here a stand-in
engine writes rank-tagged bytes so the test checks what the driver owns: byte-balanced
contiguous shards in SpanGroup order, and an all-gather that hands tsdbhip_finalize the
rank buffers in rank order (the GPU tests check the merge itself)."""
from __future__ import annotations

import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from opentsdb_amd import abi, dist, synth

T0 = 1356998400


def test_shard_bounds_balanced():
    w = np.arange(1, 101)
    for world in (1, 2, 3, 4, 8):
        b = dist.shard_bounds(w, world)
        assert b[0] == 0 and b[-1] == 100 and all(x <= y for x, y in zip(b, b[1:]))
        sums = [w[b[r]:b[r + 1]].sum() for r in range(world)]
        assert max(sums) - min(sums) <= 2 * w.max()


def test_shard_bounds_more_ranks_than_series():
    b = dist.shard_bounds([5, 5], 4)
    assert b[0] == 0 and b[-1] == 2 and len(b) == 5


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_shards_concatenate_to_group_order(world):
    b = synth.generate(37, T0, 400, 10000, value_kind=2, n_groups=4, int_mod=30000, seed=11)
    # scramble group ids so the group-sorted order differs from batch order
    gid = b.group_id.copy()
    gid[::3] = (gid[::3] + 1) % 4
    gid[5] = -1
    b = abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, b.val, gid)
    order = dist.group_sorted_order(b)
    shards = [dist.shard_batch(b, r, world) for r in range(world)]
    assert sum(s.n_series for s in shards) == len(order)
    np.testing.assert_array_equal(np.concatenate([s.group_id for s in shards]), gid[order])
    qual = np.concatenate([s.qual[:int(s.row_qual_off[-1])] for s in shards])
    want = np.concatenate([b.qual[int(b.row_qual_off[r]):int(b.row_qual_off[r + 1])]
                           for s in order for r in range(b.series_row_ptr[s], b.series_row_ptr[s + 1])])
    np.testing.assert_array_equal(qual, want)
    gs = np.concatenate([s.group_id for s in shards])
    assert np.all(np.diff(gs) >= 0)


class TaggedEngine:
    """Stand-in for Engine: partial buffers of rank-tagged bytes; finalize returns them."""

    def __init__(self, rank, nbytes):
        self.rank, self.nbytes = rank, nbytes

    def partials_layout(self, q, G):
        lay = abi.PartialsLayout()
        lay.n_groups, lay.n_slots, lay.bytes = G, 1, self.nbytes
        return lay

    def run_partials(self, q, G, ptr):
        data = (np.arange(self.nbytes) * 7 + self.rank * 31).astype(np.uint8)
        C.memmove(ptr, data.ctypes.data, self.nbytes)

    def finalize(self, q, G, ptr, n_ranks):
        return np.ctypeslib.as_array((C.c_uint8 * (self.nbytes * n_ranks)).from_address(ptr)).copy()


def _worker(rank, world, port, nbytes, out):
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q = abi.new_query(T0, T0 + 3599, "sum")
        got = dist.run_distributed(TaggedEngine(rank, nbytes), q, td, 4)
        np.save(os.path.join(out, f"r{rank}.npy"), got)
    finally:
        td.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_exchange_rank_order(tmp_path, world):
    nbytes = 1000
    mp.spawn(_worker, args=(world, _free_port(), nbytes, str(tmp_path)), nprocs=world, join=True)
    want = np.concatenate([(np.arange(nbytes) * 7 + r * 31).astype(np.uint8) for r in range(world)])
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"r{r}.npy"), want)


# ---- percentile / median group-by exchange (values to the owning rank) --------------
def _emulate_sel_exchange(per_rank_vals, per_rank_counts, K):
    """all-to-all of sel_pack outputs, in-process: recv[me] = concat over r of r's piece for me."""
    import torch
    world = len(per_rank_vals)
    counts_all = np.stack(per_rank_counts)
    own = dist.sel_owner(counts_all)
    sends = [dist.sel_pack(per_rank_vals[r], per_rank_counts[r], K, own, r, world) for r in range(world)]
    outs = []
    for me in range(world):
        pieces = []
        for r in range(world):
            send, splits = sends[r]
            off = int(sum(splits[:me]))
            pieces.append(send[off:off + splits[me]])
        recv = torch.cat(pieces)
        assert recv.numel() == sum(dist.sel_recv_splits(counts_all, K, own, me))
        outs.append(dist.sel_unpack(recv, counts_all, K, me, per_rank_vals[me]))
    return outs, own


def _rank_values(counts, K, world):
    import torch
    vals = []
    for r in range(world):
        v = []
        for g in range(len(counts[r])):
            for i in range(counts[r][g]):
                for k in range(K):
                    v.append(r * 1e6 + g * 1e4 + k * 1e2 + i)
        vals.append(torch.tensor(v, dtype=torch.float64))
    return vals


def _check_owned(outs, own, counts, K, world):
    G = len(own)
    for me, (ov, seg) in enumerate(outs):
        pos = 0
        for g in range(G):
            if own[g] != me:
                assert seg[g] == 0
                continue
            n = sum(int(counts[r][g]) for r in range(world))
            assert seg[g] == n
            want = [r * 1e6 + g * 1e4 + k * 1e2 + i for r in range(world) for i in range(counts[r][g])
                    for k in range(K)]
            np.testing.assert_array_equal(ov[pos:pos + n * K].numpy(), want)
            pos += n * K
        assert pos == ov.numel()


def test_sel_owner_is_first_rank_with_spans():
    ca = np.array([[0, 2, 0, 1], [3, 1, 0, 0], [1, 0, 0, 4]])
    np.testing.assert_array_equal(dist.sel_owner(ca), [1, 0, 0, 0])


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sel_pack_unpack_routes_every_value(world):
    rng = np.random.default_rng(world)
    G, K = 7, 5
    counts = [rng.integers(0, 4, G) for _ in range(world)]
    vals = _rank_values(counts, K, world)
    outs, own = _emulate_sel_exchange(vals, counts, K)
    _check_owned(outs, own, counts, K, world)


@pytest.mark.parametrize("world", [2, 4])
def test_sel_whole_groups_move_nothing(world):
    """Contiguous series shards with whole groups per rank: no value leaves its rank and each
    owner selects over its own contribution buffer in place."""
    G, K = 8, 3
    counts = [np.array([3 if g * world // G == r else 0 for g in range(G)]) for r in range(world)]
    vals = _rank_values(counts, K, world)
    outs, own = _emulate_sel_exchange(vals, counts, K)
    _check_owned(outs, own, counts, K, world)
    for me, (ov, _) in enumerate(outs):
        assert ov.data_ptr() == vals[me].data_ptr()   # no copy


def test_sel_combine_takes_owner_rows():
    import torch
    world, G, K = 3, 5, 2
    rows = torch.zeros(world, G * K, dtype=torch.float64)
    for r in range(world):
        rows[r] = r + 10 * torch.arange(G * K)
    own = np.array([2, 0, 1, 1, 0])
    got = dist.sel_combine(rows.reshape(-1), G, K, own).reshape(G, K)
    for g in range(G):
        np.testing.assert_array_equal(got[g].numpy(), own[g] + 10 * np.arange(g * K, g * K + K))


def _sel_gloo_worker(rank, world, port, out):  # noqa: C901
    """The collective sequence of run_distributed_sel over gloo, with the engine calls
    replaced by host arithmetic (no GPU here): every rank contributes known values, and
    the owner's gathered segments must hold every rank's values of its groups."""
    import torch
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G, K = 6, 3
        counts = np.array([(rank + g) % 3 for g in range(G)], np.int64)
        vals = torch.tensor([rank * 1e6 + g * 1e4 + k * 1e2 + i for g in range(G) for i in range(counts[g])
                             for k in range(K)], dtype=torch.float64)
        c_all = torch.empty(world * G, dtype=torch.int64)
        td.all_gather_into_tensor(c_all, torch.as_tensor(counts))
        counts_all = c_all.numpy().reshape(world, G)
        own = dist.sel_owner(counts_all)
        send, in_splits = dist.sel_pack(vals, counts, K, own, rank, world)
        out_splits = dist.sel_recv_splits(counts_all, K, own, rank)
        recv = torch.empty(sum(out_splits), dtype=torch.float64)
        td.all_to_all_single(recv, send.contiguous(), out_splits, in_splits)
        ov, seg = dist.sel_unpack(recv, counts_all, K, rank, vals)
        np.savez(os.path.join(out, f"s{rank}.npz"), ov=ov.numpy(), seg=seg, counts_all=counts_all)
    finally:
        td.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sel_exchange_gloo(tmp_path, world):
    mp.spawn(_sel_gloo_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    G, K = 6, 3
    for me in range(world):
        z = np.load(tmp_path / f"s{me}.npz")
        ca = z["counts_all"]
        own = dist.sel_owner(ca)
        want = []
        for g in range(G):
            if own[g] != me:
                continue
            want += [r * 1e6 + g * 1e4 + k * 1e2 + i for r in range(world) for i in range(ca[r, g]) for k in range(K)]
        np.testing.assert_array_equal(z["ov"], want)


# ---- raw queries: group-sharded (whole SpanGroups per rank) ---------------------------
@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_shard_by_group_keeps_groups_whole(world):
    b = synth.generate_counters(60, 1356998400, 40, n_groups=7, seed=5)
    seen = []
    owner = {}
    for r in range(world):
        s = dist.shard_batch_by_group(b, r, world)
        for g in np.unique(s.group_id):
            assert owner.setdefault(int(g), r) == r, "group split across ranks"
        seen.append(s.n_series)
        # series of a group keep their batch (SpanGroup) order
        for g in np.unique(s.group_id):
            idx = np.nonzero(s.group_id == g)[0]
            assert np.all(np.diff(idx) == 1)
    assert sum(seen) == b.n_series
    assert sorted(owner) == list(range(7))


@pytest.mark.parametrize("world", [1, 2, 3])
def test_shard_spans_covers_batch_in_order(world):
    b = synth.generate(17, 1356998400, 30, 10000, value_kind=0, n_groups=4, seed=1)
    got = []
    for r in range(world):
        s = dist.shard_batch_spans(b, r, world)
        got.append(s.n_series)
    assert sum(got) == b.n_series
    parts = [[(0, np.zeros(1), np.zeros(1), np.zeros(1))] * n for n in got]
    assert [g[0] for g in dist.merge_none_results(parts)] == list(range(b.n_series))


# ---- result gathers as tensors (raw / NONE queries) ------------------------------------
def _rank_groups(rank):
    rng = np.random.default_rng(100 + rank)
    out = []
    for i in range(int(rng.integers(0, 5))):
        n = int(rng.integers(0, 40))
        out.append((rank * 10 + i, rng.integers(0, 1 << 40, n).astype(np.int64),
                    rng.integers(0, 1 << 63, n, dtype=np.uint64) | np.uint64(1 << 63), rng.integers(0, 2, n).astype(np.uint8)))
    return out


def _gather_worker(rank, world, port, out):
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        parts = dist.gather_groups(_rank_groups(rank), td)
        flat = [(r, g, ts, bits, isi) for r, p in enumerate(parts) for (g, ts, bits, isi) in p]
        np.savez(os.path.join(out, f"g{rank}.npz"), rg=np.array([(f[0], f[1]) for f in flat]).reshape(-1, 2),
                 n=np.array([len(f[2]) for f in flat]),
                 ts=np.concatenate([f[2] for f in flat]) if flat else np.zeros(0, np.int64),
                 bits=np.concatenate([f[3] for f in flat]) if flat else np.zeros(0, np.uint64),
                 isi=np.concatenate([f[4] for f in flat]) if flat else np.zeros(0, np.uint8))
    finally:
        td.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gather_groups_gloo(tmp_path, world):
    """Uneven per-rank results (0..4 groups of 0..39 points, all 64 value bits used) arrive
    on every rank, in rank order, bit for bit."""
    mp.spawn(_gather_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = [(r, g) for r in range(world) for (g, _, _, _) in _rank_groups(r)]
    wts = [x for r in range(world) for (_, ts, _, _) in _rank_groups(r) for x in ts]
    wbits = [x for r in range(world) for (_, _, b, _) in _rank_groups(r) for x in b]
    for me in range(world):
        z = np.load(tmp_path / f"g{me}.npz")
        assert [tuple(x) for x in z["rg"]] == want
        np.testing.assert_array_equal(z["ts"], np.array(wts, np.int64))
        np.testing.assert_array_equal(z["bits"], np.array(wbits, np.uint64))


# ---- sharding inside the library (host logic of libtsdbhip, no GPU) ---------------------
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_library_shard_bounds_match_python(world):
    from opentsdb_amd import engine
    b = synth.generate(57, T0, 400, 10000, value_kind=2, n_groups=6, int_mod=30000, seed=7)
    gid = b.group_id.copy()
    gid[::4] = (gid[::4] + 2) % 6
    gid[7] = -1
    b = abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, b.val, gid)
    order = dist.group_sorted_order(b)
    sb = dist.series_bytes(b)
    assert list(engine.shard_bounds(b, world, engine.SHARD_SERIES)) == dist.shard_bounds(sb[order], world)
    assert list(engine.shard_bounds(b, world, engine.SHARD_GROUPS)) == dist.group_shard_bounds(b, world)
    assert list(engine.shard_bounds(b, world, engine.SHARD_SPANS)) == dist.shard_bounds(sb, world)


def test_shard_ten_million_series_in_seconds():
    """A 10M-series batch (config 3's series count, one 4-point row each) is sharded 8 ways
    on the host in seconds: library bounds, and the vectorised Python selection of a shard."""
    import time
    from opentsdb_amd import engine
    n = 10_000_000
    srp = np.arange(n + 1, dtype=np.int64)
    qo = np.arange(n + 1, dtype=np.uint64) * 8
    vo = np.arange(n + 1, dtype=np.uint64) * 17
    b = abi.HostBatch(srp, np.full(n, T0, np.uint32), qo, vo, np.zeros(8 * n, np.uint8), np.zeros(17 * n, np.uint8),
                      (np.arange(n) % 1000).astype(np.int32))
    t = time.perf_counter()
    bounds = engine.shard_bounds(b, 8, engine.SHARD_SERIES)
    t_bounds = time.perf_counter() - t
    assert bounds[0] == 0 and bounds[-1] == n and np.all(np.diff(bounds) > 0)
    assert t_bounds < 10, t_bounds
    t = time.perf_counter()
    order = dist.group_sorted_order(b)
    s = dist.select_series(b, order[bounds[3]:bounds[4]])
    t_sel = time.perf_counter() - t
    assert s.n_series == bounds[4] - bounds[3] and len(s.qual) == 8 * s.n_series
    assert t_sel < 20, t_sel


def _rollup_batch(seed=3):
    """A rollup scan result: value cells from synth, count cells of random length per row."""
    b = synth.generate(37, 1356998400, 120, 60000, value_kind=2, n_groups=5, int_mod=100, seed=seed)
    gid = b.group_id.copy()
    gid[::7] = -1
    rng = np.random.default_rng(seed)
    clen = rng.integers(0, 5, b.n_rows) * 2
    cq_off = np.concatenate([[0], np.cumsum(clen)]).astype(np.uint64)
    cv_off = np.concatenate([[0], np.cumsum(clen // 2)]).astype(np.uint64)
    cq = rng.integers(0, 256, int(cq_off[-1]), dtype=np.uint8)
    cv = rng.integers(0, 256, int(cv_off[-1]), dtype=np.uint8)
    cells = abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, b.val, gid)
    return abi.HostRollupBatch(cells, (cq_off, cv_off, cq, cv), abi.RollupInterval())


def _series_cells(rb):
    c = rb.cells
    srp = c.series_row_ptr
    out = []
    for s in range(c.n_series):
        rows = range(srp[s], srp[s + 1])
        cut = lambda o, buf: [bytes(buf[int(o[r]):int(o[r + 1])]) for r in rows]  # noqa: E731
        out.append((int(c.group_id[s]), [int(c.row_base_time[r]) for r in rows], cut(c.row_qual_off, c.qual),
                    cut(c.row_val_off, c.val), cut(rb.counts[0], rb.counts[2]), cut(rb.counts[1], rb.counts[3])))
    return out


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("by_group", [False, True])
def test_shard_rollup_batch_covers_groups(world, by_group):
    """dist.shard_rollup_batch: the ranks' shards hold every grouped series once, value and count
    cells of each row intact; series shards follow the SpanGroup order, group shards keep groups
    whole."""
    rb = _rollup_batch()
    full = _series_cells(rb)
    want = sorted([x for x in full if x[0] >= 0], key=lambda x: x[0])
    got, owner = [], {}
    for r in range(world):
        sh = dist.shard_rollup_batch(rb, r, world, by_group=by_group)
        assert sh.counts is not None and sh.interval is rb.interval
        part = _series_cells(sh)
        for x in part:
            owner.setdefault(x[0], set()).add(r)
        got.extend(part)
    if by_group:
        assert all(len(v) == 1 for v in owner.values())
        got = sorted(got, key=lambda x: x[0])
    assert got == want
