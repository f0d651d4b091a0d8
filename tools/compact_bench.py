"""Query-time compaction at scale: S series x N one-datapoint cells
per hour row (1 s data, 8-byte values, columns in shuffled order, distinct write
timestamps), compacted on the GPU by tsdbhip_load_cells.  Prints the wall time of the call,
the device compaction time (k_compact pipeline, host layout excluded), k_index, and the
algorithmic bytes rate: per cell 2 B qualifier + 8 B value + 16 B column offsets + 8 B
timestamp read, 10 B written."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from opentsdb_amd import abi  # noqa: E402
from opentsdb_amd.engine import Engine  # noqa: E402

B = 1356998400


def build(S, N, seed=1, scan_order=False):
    """scan_order: each row's columns in qualifier order, as an HBase scan returns them (time
    order for second qualifiers); else shuffled (the general merge)."""
    rng = np.random.default_rng(seed)
    nrow = S
    if scan_order:
        perm = np.tile(np.arange(N, dtype=np.uint32), (nrow, 1))
    else:
        perm = np.argsort(rng.random((nrow, N)), axis=1).astype(np.uint32)
    quals = ((perm << 4) | 7).astype(">u2")
    vals = rng.integers(-10**6, 10**6, size=(nrow, N)).astype(">i8")
    ncol = nrow * N
    return abi.HostCellBatch(np.arange(S + 1, dtype=np.int64), np.full(S, B, np.uint32),
                             np.arange(nrow + 1, dtype=np.int64) * N, np.arange(ncol + 1, dtype=np.uint64) * 2,
                             np.arange(ncol + 1, dtype=np.uint64) * 8, quals.view(np.uint8).reshape(-1),
                             vals.view(np.uint8).reshape(-1), (np.arange(S) * 64 // S).astype(np.int32),
                             rng.permutation(ncol).astype(np.int64), False)


def pinned(cb):
    """The same scan assembled in page-locked host memory (tsdbhip_host_alloc)."""
    from opentsdb_amd.engine import pinned_copy
    return abi.HostCellBatch(*(pinned_copy(x) for x in (cb.series_row_ptr, cb.row_base_time, cb.row_col_ptr,
                                                         cb.col_qual_off, cb.col_val_off, cb.qual, cb.val,
                                                         cb.group_id, cb.col_timestamp)), False)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    S = int(args[0]) if len(args) > 0 else 20000
    N = int(args[1]) if len(args) > 1 else 3600
    steps = int(args[2]) if len(args) > 2 else 3
    t = time.perf_counter()
    order = "--scan-order" in sys.argv
    cb = build(S, N, scan_order=order)
    gen_s = time.perf_counter() - t
    if "--pinned-first" in sys.argv:   # (diagnostic: page-locked buffers before the context exists)
        cb = pinned(cb)
    from opentsdb_amd.engine import set_option
    for a in sys.argv:   # --opt=NAME=VALUE: a developer option (A/B runs)
        if a.startswith("--opt="):
            k, v = a[6:].split("=")
            set_option(k, v)
    eng = Engine(0)
    if "--pinned" in sys.argv:
        cb = pinned(cb)
    eng.load_cells(cb)
    walls, cms, ims = [], [], []
    for _ in range(steps):
        t = time.perf_counter()
        eng.load_cells(cb)
        walls.append((time.perf_counter() - t) * 1000)
        tm = eng.timing()
        cms.append(tm.compact_ms)
        ims.append(tm.index_ms)
    cells = S * N
    cm = sum(cms) / steps
    q = abi.new_query(B, B + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    eng.run(q)
    t = time.perf_counter()
    eng.run(q)
    run_ms = (time.perf_counter() - t) * 1000
    print(json.dumps({"workload": f"{S} series x {N} one-datapoint cells "
                                  f"({'qualifier (scan) order' if order else 'shuffled'}), 8-byte ints",
                      "host_memory": "pinned" if any(a.startswith("--pinned") for a in sys.argv) else "pageable",
                      "cells": cells, "load_cells_wall_ms": sum(walls) / steps, "compact_ms": cm,
                      "index_ms": sum(ims) / steps, "cells_per_s_device": cells / (cm / 1000),
                      "algorithmic_GBps": cells * 44 / (cm / 1000) / 1e9, "query_ms_after": run_ms,
                      "gen_s": gen_s}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
