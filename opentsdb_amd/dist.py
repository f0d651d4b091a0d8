"""Multi-GPU driver: series sharded over ranks, one exchange step.

One process per GPU (``torch.distributed.run``), each with its own libtsdbhip context.
Series are split into contiguous shards of the group-sorted span order (a SpanGroup may
straddle ranks); every rank reduces its shard to per-(group, slot) partial states
(``tsdbhip_run_partials``), the ranks all-gather those buffers -- RCCL over xGMI with the
``nccl`` backend, or gloo on host memory -- and ``tsdbhip_finalize`` merges them in rank
order, which continues the reference's SpanGroup series order across GPUs
(``TsdbQuery.GroupByAndAggregateCB`` src/core/TsdbQuery.java:927-1048 feeds every span of a
group to one ``AggregationIterator``; here the spans of one group are spread over ranks).

There is no data-path collective: the only communication is the all-gather of
G x K x 24 bytes of partial state per rank.
"""
from __future__ import annotations

import numpy as np

from . import abi


def shard_bounds(series_bytes, world: int):
    """Contiguous, byte-balanced split of series (in batch order) over `world` ranks.

    Returns world+1 series indices; rank r owns series [b[r], b[r+1]).  Boundaries sit at
    the first series whose cumulative byte count reaches r/world of the total, so every
    shard streams about the same HBM bytes (the kernel is bandwidth-bound)."""
    w = np.asarray(series_bytes, dtype=np.float64)
    n = len(w)
    if world < 1:
        raise ValueError("world must be >= 1")
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    b = [0]
    for r in range(1, world):
        b.append(int(np.searchsorted(cum, total * r / world, side="left")) if total > 0 else n * r // world)
        b[-1] = max(b[-1], b[-2])
    b.append(n)
    return b


def group_sorted_order(batch: abi.HostBatch):
    """Series in SpanGroup order: stable by group id, dropped series (-1) removed."""
    g = batch.group_id
    keep = np.nonzero(g >= 0)[0]
    return keep[np.argsort(g[keep], kind="stable")]


def _ranges(starts, ends):
    """Concatenation of arange(starts[i], ends[i]) (vectorised)."""
    starts = np.asarray(starts, np.int64)
    lens = np.asarray(ends, np.int64) - starts
    if lens.sum() == 0:
        return np.zeros(0, np.int64)
    keep = lens > 0
    starts, lens = starts[keep], lens[keep]
    first = np.repeat(np.cumsum(lens) - lens, lens)
    return np.repeat(starts, lens) + (np.arange(int(lens.sum()), dtype=np.int64) - first)


def select_series(batch: abi.HostBatch, series) -> abi.HostBatch:
    """A batch holding only `series` (indices, in the given order); group ids unchanged.
    Vectorised (no per-row Python); the library's tsdbhip_load_shard does the same without a
    host copy."""
    srp = batch.series_row_ptr
    qo, vo = batch.row_qual_off.astype(np.int64), batch.row_val_off.astype(np.int64)
    series = np.asarray(series, np.int64)
    rows = _ranges(srp[series], srp[series + 1])
    new_srp = np.zeros(len(series) + 1, np.int64)
    if len(series):
        new_srp[1:] = np.cumsum(srp[series + 1] - srp[series])
    ql = qo[rows + 1] - qo[rows]
    vl = vo[rows + 1] - vo[rows]
    nqo = np.concatenate([[0], np.cumsum(ql)]).astype(np.uint64)
    nvo = np.concatenate([[0], np.cumsum(vl)]).astype(np.uint64)
    q = batch.qual[_ranges(qo[rows], qo[rows + 1])]
    v = batch.val[_ranges(vo[rows], vo[rows + 1])]
    return abi.HostBatch(new_srp, batch.row_base_time[rows], nqo, nvo, q, v, batch.group_id[series])


def shard_batch(batch: abi.HostBatch, rank: int, world: int) -> abi.HostBatch:
    """The rank's shard of a host batch (group ids stay global)."""
    order = group_sorted_order(batch)
    srp = batch.series_row_ptr
    qo, vo = batch.row_qual_off.astype(np.int64), batch.row_val_off.astype(np.int64)
    sbytes = [(qo[srp[s + 1]] - qo[srp[s]]) + (vo[srp[s + 1]] - vo[srp[s]]) for s in order]
    b = shard_bounds(sbytes, world)
    return select_series(batch, order[b[rank]:b[rank + 1]])


def shard_rollup_batch(rb: abi.HostRollupBatch, rank: int, world: int, by_group: bool = False) -> abi.HostRollupBatch:
    """The rank's shard of a rollup scan (value cells and, with RollupSeq.need_count, the count
    cells of the same rows): series split like shard_batch / shard_batch_by_group.  Load it with
    eng.load_rollup; run_distributed / run_distributed_sel then work over rollup shards as over
    raw ones (the library plans a count group-by as sum on every rank)."""
    cells = rb.cells
    srp = cells.series_row_ptr
    w = series_bytes(cells)
    if rb.counts is not None:
        cqo, cvo = rb.counts[0].astype(np.int64), rb.counts[1].astype(np.int64)
        w = w + np.array([(cqo[srp[s + 1]] - cqo[srp[s]]) + (cvo[srp[s + 1]] - cvo[srp[s]])
                          for s in range(cells.n_series)], np.float64)
    if by_group:
        gw = np.bincount(cells.group_id[cells.group_id >= 0], weights=w[cells.group_id >= 0],
                         minlength=n_groups_of(cells))
        b = shard_bounds(gw, world)
        series = np.nonzero((cells.group_id >= b[rank]) & (cells.group_id < b[rank + 1]))[0]
    else:
        order = group_sorted_order(cells)
        b = shard_bounds(w[order], world)
        series = order[b[rank]:b[rank + 1]]
    sub = select_series(cells, series)
    counts = None
    if rb.counts is not None:
        cqo, cvo = rb.counts[0].astype(np.int64), rb.counts[1].astype(np.int64)
        series = np.asarray(series, np.int64)
        rows = _ranges(srp[series], srp[series + 1])
        nq = np.concatenate([[0], np.cumsum(cqo[rows + 1] - cqo[rows])]).astype(np.uint64)
        nv = np.concatenate([[0], np.cumsum(cvo[rows + 1] - cvo[rows])]).astype(np.uint64)
        counts = (nq, nv, rb.counts[2][_ranges(cqo[rows], cqo[rows + 1])], rb.counts[3][_ranges(cvo[rows], cvo[rows + 1])])
    return abi.HostRollupBatch(sub, counts, rb.interval, rb.fix_duplicates)


def n_groups_of(batch: abi.HostBatch) -> int:
    return int(batch.group_id.max()) + 1 if batch.n_series else 0


def run_distributed(eng, q: abi.Query, dist, n_groups_global: int, device=None):
    """One query over the sharded store: local partials -> all-gather -> rank-ordered merge.

    `dist` is an initialised ``torch.distributed``.  With the nccl (RCCL) backend the
    buffers live in HBM on `device`; with gloo they are host tensors.  Returns the groups
    (every rank gets the full result)."""
    import torch

    world = dist.get_world_size()
    lay = eng.partials_layout(q, n_groups_global)
    on_gpu = dist.get_backend() == "nccl"
    dev = device if on_gpu else "cpu"
    mine = torch.empty(int(lay.bytes), dtype=torch.uint8, device=dev)
    eng.run_partials(q, n_groups_global, mine.data_ptr())   # synchronous on the engine stream
    gathered = torch.empty(world * int(lay.bytes), dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, mine)
    if on_gpu:
        torch.cuda.current_stream(dev).synchronize()
    return eng.finalize(q, n_groups_global, gathered.data_ptr(), world)


def run_distributed_multi(eng, qs, dist, n_groups_global: int, device=None):
    """Several decomposable queries sharing the time range and downsampling (a TSQuery's
    sub-queries over one metric, TsdbQuery.java:916-1049 once each): ONE fused pass over the
    shard for all of them (tsdbhip_run_partials_multi), ONE all-gather of the concatenated
    partial states, then the rank-ordered merge per query.  Returns one group list per query."""
    import torch

    world = dist.get_world_size()
    sizes = [int(eng.partials_layout(q, n_groups_global).bytes) for q in qs]
    if len(set(sizes)) != 1:
        raise ValueError("run_distributed_multi: the queries must share the time range and downsampling")
    total = sum(sizes)
    on_gpu = dist.get_backend() == "nccl"
    dev = device if on_gpu else "cpu"
    mine = torch.empty(total, dtype=torch.uint8, device=dev)
    eng.run_partials_multi(qs, n_groups_global, mine.data_ptr())
    gathered = torch.empty(world * total, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, mine)
    per_q = gathered.view(world, len(qs), sizes[0]).transpose(0, 1).contiguous()   # [query][rank][bytes]
    if on_gpu:
        torch.cuda.current_stream(dev).synchronize()
    return [eng.finalize(q, n_groups_global, per_q[i].data_ptr(), world) for i, q in enumerate(qs)]


# ---- percentile / median as the group-by aggregator: values to the owning rank --------
#
# PercentileAgg / Median.runDouble need every span's value of a (group, slot) at once
# (src/core/Aggregators.java:397-431, 657-708): there is no partial state to all-gather.
# Group g is owned by the FIRST rank holding one of its spans (as the one-process multi-device
# context does, multi.cpp): with contiguous series shards a group lives on one rank or straddles
# a boundary, so only the straddling groups' values move.  Every rank sends its spans'
# contributions of g to the owner (one all-to-all over RCCL), the owner sorts and selects, and
# the owners' dense rows are all-gathered (G x K x 9 B) so every rank can build the full result.

def sel_owner(counts_all):
    """Owning rank per group from every rank's span counts ([world, G]): the first rank with a
    span of the group (rank 0 for a group without spans)."""
    counts_all = np.asarray(counts_all, np.int64)
    if counts_all.ndim != 2 or counts_all.shape[1] == 0:
        return np.zeros(counts_all.shape[-1] if counts_all.ndim else 0, np.int64)
    has = counts_all > 0
    return np.where(has.any(axis=0), has.argmax(axis=0), 0).astype(np.int64)


def sel_pack(vals, counts, K: int, own, me: int, world: int):
    """This rank's [span][slot] contributions (spans group by group) of the groups OTHER ranks
    own (`own` = sel_owner(counts_all)), ordered by owning rank; the groups `me` owns stay put.

    Returns (send, in_splits): `send` holds, for owner 0, 1, ... (never `me`), the blocks of
    the groups it owns in increasing group order; in_splits[o] is the element count for o."""
    import torch
    counts = np.asarray(counts, np.int64)
    off = np.concatenate([[0], np.cumsum(counts * K)])
    own = np.asarray(own, np.int64)
    pieces, splits = [], []
    for o in range(world):
        gs = np.nonzero((own == o) & (counts > 0))[0] if o != me else np.zeros(0, np.int64)
        splits.append(int(counts[gs].sum() * K))
        pieces += [vals[int(off[g]):int(off[g + 1])] for g in gs]
    send = torch.cat(pieces) if pieces else vals[:0]
    return send, splits


def sel_recv_splits(counts_all, K: int, own, me: int):
    """Element counts the owner `me` receives from each rank (0 from itself)."""
    counts_all = np.asarray(counts_all, np.int64)
    mine = np.asarray(own) == me
    return [0 if r == me else int(counts_all[r, mine].sum() * K) for r in range(counts_all.shape[0])]


def sel_unpack(recv, counts_all, K: int, me: int, local_vals):
    """The owner's side.  `recv` holds, per source rank r != me (in rank order), r's blocks of
    the groups `me` owns ([n_rg][K] each, increasing g); `local_vals` is this rank's own
    contribution buffer (sel_run_values).  Returns (vals, seg_counts): per owned group every
    rank's spans one after the other in rank order ([g][j][k] -- rank order is SpanGroup
    order), and the per-group span counts (0 for groups owned elsewhere).  When nothing arrives
    and every local group is owned here (whole groups per rank), `local_vals` is returned as is."""
    import torch
    counts_all = np.asarray(counts_all, np.int64)
    world, G = counts_all.shape
    own = sel_owner(counts_all)
    mine = np.nonzero(own == me)[0]
    local = counts_all[me]
    if recv.numel() == 0 and not np.any((local > 0) & (own != me)):
        seg = np.where(own == me, local, 0).astype(np.int64)
        return local_vals[:int(local.sum()) * K], seg
    loff = np.concatenate([[0], np.cumsum(local * K)])
    blocks = {int(g): [None] * world for g in mine}
    pos = 0
    for r in range(world):
        for g in mine:
            n = int(counts_all[r, g])
            if not n:
                continue
            if r == me:
                blocks[int(g)][r] = local_vals[int(loff[g]):int(loff[g + 1])]
            else:
                blocks[int(g)][r] = recv[pos:pos + n * K]
                pos += n * K
    seg = np.zeros(G, np.int64)
    out = []
    for g in mine:
        parts = [b for b in blocks[int(g)] if b is not None]
        if parts:
            b = torch.cat(parts)
            seg[g] = b.numel() // K
            out.append(b)
    vals = torch.cat(out) if out else recv[:0]
    return vals, seg


def sel_combine(rows_all, G: int, K: int, own):
    """Row g of the dense [G][K] outputs from its owner (rows_all: [world, G * K])."""
    import torch
    own = np.asarray(own, np.int64)
    world = rows_all.numel() // max(1, G * K)
    r = rows_all.reshape(world, G, K)
    idx = torch.as_tensor(own, device=r.device)
    return r[idx, torch.arange(G, device=r.device)].reshape(-1)


def run_distributed_sel(eng, q: abi.Query, dist, n_groups_global: int, device=None):
    """A percentile / median group-by query -- or a TSDB_QF_ORDERED one, whose owner folds
    the spans in rank (= SpanGroup) order -- over the sharded store:
    local contributions -> the straddling groups' values to their owners (all-to-all) ->
    sort + select on the owners -> all-gather of the owners' rows -> result on every rank."""
    import torch

    world, me = dist.get_world_size(), dist.get_rank()
    on_gpu = dist.get_backend() == "nccl"
    dev = device if on_gpu else "cpu"
    G = n_groups_global
    counts, K = eng.sel_layout(q, G)
    vals = torch.empty(max(1, int(counts.sum()) * K), dtype=torch.float64, device=dev)
    uni = torch.empty(max(1, G * K), dtype=torch.uint8, device=dev)
    act = torch.empty(max(1, G), dtype=torch.int32, device=dev)
    eng.sel_run_values(q, G, vals.data_ptr(), uni.data_ptr(), act.data_ptr())
    c_mine = torch.as_tensor(counts, dtype=torch.int64, device=dev)
    c_all = torch.empty(world * G, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(c_all, c_mine)
    counts_all = c_all.cpu().numpy().reshape(world, G)
    own = sel_owner(counts_all)
    send, in_splits = sel_pack(vals, counts, K, own, me, world)
    out_splits = sel_recv_splits(counts_all, K, own, me)
    recv = torch.empty(sum(out_splits), dtype=torch.float64, device=dev)
    dist.all_to_all_single(recv, send.contiguous(), out_splits, in_splits)
    dist.all_reduce(uni, op=dist.ReduceOp.MAX)
    dist.all_reduce(act, op=dist.ReduceOp.MAX)
    ovals, seg = sel_unpack(recv, counts_all, K, me, vals)
    ovals = ovals.contiguous()
    ov = torch.empty(max(1, G * K), dtype=torch.float64, device=dev)
    of = torch.empty(max(1, G * K), dtype=torch.uint8, device=dev)
    if on_gpu:
        torch.cuda.current_stream(dev).synchronize()
    eng.sel_select(q, G, ovals.data_ptr(), seg, uni.data_ptr(), ov.data_ptr(), of.data_ptr())
    ov_all = torch.empty(world * ov.numel(), dtype=torch.float64, device=dev)
    of_all = torch.empty(world * of.numel(), dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(ov_all, ov)
    dist.all_gather_into_tensor(of_all, of)
    val = sel_combine(ov_all, G, K, own).contiguous() if G * K else ov
    flag = sel_combine(of_all, G, K, own).contiguous() if G * K else of
    if on_gpu:
        torch.cuda.current_stream(dev).synchronize()
    return eng.assemble(q, G, val.data_ptr(), flag.data_ptr(), act.data_ptr())


# ---- raw (no-downsampling) queries: whole SpanGroups per rank -------------------------
#
# Without a downsampler the group-by runs over the union of the group's raw timestamps
# (AggregationIterator, src/core/AggregationIterator.java:500-797): O(U k) interpolations per
# group, compute-bound, with Java's span-order operand sequence for float sums.  Splitting a
# group over ranks would need the union itself exchanged and a rank-order merge of every
# aggregator state per union point; instead the raw path shards by GROUP -- each rank holds
# whole SpanGroups (contiguous, byte-balanced ranges of group ids), evaluates them exactly as
# one GPU does (bit-exact), and only the finished points are gathered.  No data-path
# collective.

def series_bytes(batch: abi.HostBatch):
    srp = batch.series_row_ptr
    qo, vo = batch.row_qual_off.astype(np.int64), batch.row_val_off.astype(np.int64)
    return (qo[srp[1:]] - qo[srp[:-1]]) + (vo[srp[1:]] - vo[srp[:-1]])


def group_shard_bounds(batch: abi.HostBatch, world: int):
    """world+1 group ids: rank r owns groups [b[r], b[r+1]), byte-balanced."""
    G = n_groups_of(batch)
    g = batch.group_id
    keep = g >= 0
    gbytes = np.bincount(g[keep], weights=series_bytes(batch)[keep].astype(np.float64), minlength=G)
    return shard_bounds(gbytes, world)


def shard_batch_by_group(batch: abi.HostBatch, rank: int, world: int) -> abi.HostBatch:
    """The rank's whole groups (group ids stay global, SpanGroup order kept)."""
    b = group_shard_bounds(batch, world)
    order = group_sorted_order(batch)
    g = batch.group_id[order]
    keep = order[(g >= b[rank]) & (g < b[rank + 1])]
    return select_series(batch, keep)


def merge_group_results(parts):
    """Concatenate per-rank result groups (disjoint group ids) in group id order."""
    groups = [g for p in parts for g in p]
    groups.sort(key=lambda x: x[0])
    return groups


def gather_groups(local, dist, device=None):
    """Every rank's result groups [(group_id, ts, bits, is_int)] on every rank, as tensor
    all-gathers (RCCL on `device` with the nccl backend, host tensors with gloo): the sizes
    first, then one padded int64 buffer [gid | n | ts | bits] and one uint8 buffer [is_int]
    per rank.  Returns the per-rank group lists in rank order."""
    import torch
    world = dist.get_world_size()
    dev = device if dist.get_backend() == "nccl" else "cpu"
    ng = len(local)
    npts = int(sum(len(g[1]) for g in local))
    sizes = torch.tensor([ng, npts], dtype=torch.int64, device=dev)
    sizes_all = torch.empty(2 * world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes_all, sizes)
    sz = sizes_all.cpu().numpy().reshape(world, 2)
    L = int(max(1, (2 * sz[:, 0] + 2 * sz[:, 1]).max()))
    P = int(max(1, sz[:, 1].max()))
    buf = np.zeros(L, np.int64)
    isi = np.zeros(P, np.uint8)
    if ng:
        buf[:ng] = [g[0] for g in local]
        buf[ng:2 * ng] = [len(g[1]) for g in local]
    if npts:
        buf[2 * ng:2 * ng + npts] = np.concatenate([np.asarray(g[1], np.int64) for g in local])
        buf[2 * ng + npts:2 * ng + 2 * npts] = np.concatenate([np.asarray(g[2], np.uint64) for g in local]).view(np.int64)
        isi[:npts] = np.concatenate([np.asarray(g[3], np.uint8) for g in local])
    t_all = torch.empty(world * L, dtype=torch.int64, device=dev)
    i_all = torch.empty(world * P, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(t_all, torch.from_numpy(buf).to(dev))
    dist.all_gather_into_tensor(i_all, torch.from_numpy(isi).to(dev))
    t_all = t_all.cpu().numpy().reshape(world, L)
    i_all = i_all.cpu().numpy().reshape(world, P)
    parts = []
    for r in range(world):
        g_n, p_n = int(sz[r, 0]), int(sz[r, 1])
        row = t_all[r]
        gid, cnt = row[:g_n], row[g_n:2 * g_n]
        ts, bits = row[2 * g_n:2 * g_n + p_n], row[2 * g_n + p_n:2 * g_n + 2 * p_n].view(np.uint64)
        cut = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
        parts.append([(int(gid[i]), ts[cut[i]:cut[i + 1]], bits[cut[i]:cut[i + 1]], i_all[r][cut[i]:cut[i + 1]])
                      for i in range(g_n)])
    return parts


def run_distributed_raw(eng, q: abi.Query, dist, device=None):
    """A raw (no-downsampling) query over a group-sharded store (shard_batch_by_group):
    local evaluation, then the points of every rank gathered to every rank."""
    if q.aggregator == abi.AGG["none"]:
        raise NotImplementedError("NONE aggregator: one group per span, ids are per rank")
    return merge_group_results(gather_groups(eng.run(q), dist, device))


# ---- NONE aggregator: one SpanGroup per span ---------------------------------------------
#
# TsdbQuery with the NONE aggregator emits every span as its own group, in span order
# (src/core/TsdbQuery.java:941-962).  Ranks take contiguous ranges of spans in batch order;
# each rank's result lists its spans in order, so concatenating the ranks' results in rank
# order and renumbering the groups reproduces the single-GPU result.  No data exchange.

def shard_batch_spans(batch: abi.HostBatch, rank: int, world: int) -> abi.HostBatch:
    """Contiguous, byte-balanced range of spans in batch order (NONE aggregator: every span,
    group-by tags ignored, TsdbQuery.java:940-961)."""
    keep = np.arange(batch.n_series)
    srp = batch.series_row_ptr
    qo, vo = batch.row_qual_off.astype(np.int64), batch.row_val_off.astype(np.int64)
    sbytes = [(qo[srp[s + 1]] - qo[srp[s]]) + (vo[srp[s + 1]] - vo[srp[s]]) for s in keep]
    b = shard_bounds(sbytes, world)
    return select_series(batch, keep[b[rank]:b[rank + 1]])


def merge_none_results(parts):
    """Rank-ordered concatenation of per-rank NONE results, group ids renumbered."""
    out = []
    for p in parts:
        for g in p:
            out.append((len(out), g[1], g[2], g[3]))
    return out


def run_distributed_none(eng, q: abi.Query, dist, device=None):
    """A NONE-aggregator query over a span-sharded store (shard_batch_spans)."""
    return merge_none_results(gather_groups(eng.run(q), dist, device))


# ---- the library's own sharding (no host copy) -------------------------------------------
MODE_OF = {"series": 0, "groups": 1, "spans": 2}   # tsdbhip.h TSDB_SHARD_*


def load_rank_shard(eng, batch: abi.HostBatch, rank: int, world: int, mode: str = "series"):
    """tsdbhip_shard_bounds + tsdbhip_load_shard: this rank's shard of a host batch, selected
    and copied by the library (series / groups / spans as shard_batch /
    shard_batch_by_group / shard_batch_spans)."""
    from . import engine
    m = MODE_OF[mode]
    b = engine.shard_bounds(batch, world, m)
    eng.load_shard(batch, m, int(b[rank]), int(b[rank + 1]))
    return b


def synth_bounds(n_series: int, world: int):
    """Byte-balanced shard boundaries of a uniform synthetic store (every series the same
    size): world + 1 batch positions."""
    return [n_series * r // world for r in range(world + 1)]
