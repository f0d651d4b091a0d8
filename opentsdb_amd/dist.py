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


def select_series(batch: abi.HostBatch, series) -> abi.HostBatch:
    """A batch holding only `series` (indices, in the given order); group ids unchanged."""
    srp = batch.series_row_ptr
    qo, vo = batch.row_qual_off.astype(np.int64), batch.row_val_off.astype(np.int64)
    series = np.asarray(series, np.int64)
    rows = [np.arange(srp[s], srp[s + 1]) for s in series]
    rows = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    new_srp = np.zeros(len(series) + 1, np.int64)
    if len(series):
        new_srp[1:] = np.cumsum(srp[series + 1] - srp[series])
    ql = qo[rows + 1] - qo[rows]
    vl = vo[rows + 1] - vo[rows]
    nqo = np.concatenate([[0], np.cumsum(ql)]).astype(np.uint64)
    nvo = np.concatenate([[0], np.cumsum(vl)]).astype(np.uint64)
    q = np.concatenate([batch.qual[qo[r]:qo[r + 1]] for r in rows]) if len(rows) else np.zeros(0, np.uint8)
    v = np.concatenate([batch.val[vo[r]:vo[r + 1]] for r in rows]) if len(rows) else np.zeros(0, np.uint8)
    return abi.HostBatch(new_srp, batch.row_base_time[rows], nqo, nvo, q, v, batch.group_id[series])


def shard_batch(batch: abi.HostBatch, rank: int, world: int) -> abi.HostBatch:
    """The rank's shard of a host batch (group ids stay global)."""
    order = group_sorted_order(batch)
    srp = batch.series_row_ptr
    qo, vo = batch.row_qual_off.astype(np.int64), batch.row_val_off.astype(np.int64)
    sbytes = [(qo[srp[s + 1]] - qo[srp[s]]) + (vo[srp[s + 1]] - vo[srp[s]]) for s in order]
    b = shard_bounds(sbytes, world)
    return select_series(batch, order[b[rank]:b[rank + 1]])


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
