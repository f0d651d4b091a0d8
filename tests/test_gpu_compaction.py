"""GPU parity of query-time compaction: tsdbhip_load_cells compacts
the scanner's rows on the device (k_compact.hip) as CompactionQueue.Compaction.compact
returns them to a query (src/core/CompactionQueue.java:330-566).

  * every TestCompactionQueue known answer of the query path (tests/golden/compaction.json):
    the resident row's bytes after load_cells, or the exception a covering query raises;
  * randomized rows -- individual cells in any order, earlier compactions, append columns
    with repeats, 2-byte float / length fixups, annotations, duplicates with equal and
    different values, mixed s / ms -- against the oracle's compaction row by row, and the
    queries over them against the oracle's queries over its own compaction;
  * a 3,000-series store of one-cell-per-datapoint rows in shuffled column order;
  * tsd.storage.use_otsdb_timestamp (dtcsMergeDataPoints, CompactionQueue.java:508-547): every
    known-answer row and randomized rows with repeated offsets against the oracle."""
from __future__ import annotations

import importlib.util
import os
import struct

import numpy as np
import pytest

from opentsdb_amd import abi
from opentsdb_amd.engine import get_option, set_option
from opentsdb_amd.engine import EngineError
from opentsdb_amd.store import make_batch
from oracle import oracle as O
from tests import golden_util as gu
from tests.test_gpu_parity import assert_groups_match

pytestmark = pytest.mark.gpu

DOC = gu.load("compaction.json")
_spec = importlib.util.spec_from_file_location("make_compaction_golden",
                                               os.path.join(gu.GOLDEN, "make_compaction_golden.py"))
MK = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MK)
B = 1356998400


@pytest.fixture(scope="module")
def eng():
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


def rows_of(batch):
    out = []
    for r in range(batch.n_rows):
        q = batch.qual[int(batch.row_qual_off[r]):int(batch.row_qual_off[r + 1])].tobytes()
        v = batch.val[int(batch.row_val_off[r]):int(batch.row_val_off[r + 1])].tobytes()
        out.append((int(batch.row_base_time[r]), q, v))
    return out


@pytest.mark.parametrize("case", DOC["cases"], ids=[c["name"] for c in DOC["cases"]])
def test_known_answers_on_gpu(eng, case):
    cols, expect = MK.expand_columns(case)
    ts = case.get("timestamps") or list(range(len(cols)))
    cb = abi.HostCellBatch.from_rows([[(B, [(q, v, t) for t, (q, v) in zip(ts, cols)])]], [0],
                                     case["fix_duplicates"], case.get("use_otsdb_timestamp", False))
    eng.load_cells(cb)
    got = rows_of(eng.download())
    q = abi.new_query(B, B + 3599, "sum")
    if expect == "IllegalDataException":
        assert got == []
        with pytest.raises(EngineError) as e:
            eng.run(q)
        assert e.value.java == "IllegalDataException"
        # a query whose scan does not cover the row never compacts it
        eng.run(abi.new_query(B + 7200, B + 9000, "sum"))
        return
    if expect is None:
        assert got == []
        return
    assert got == [(B, expect[0], expect[1])]


def _cell(off_ms, ms, value, kind):
    """One datapoint as a cell: (qualifier, value bytes)."""
    if kind == "long":
        v = struct.pack(">q", value)
        fl = 7
    elif kind == "int":
        v = struct.pack(">i", value)
        fl = 3
    elif kind == "float":
        v = struct.pack(">f", value)
        fl = 0xB
    else:
        v = struct.pack(">d", value)
        fl = 0xF
    if ms:
        q = struct.pack(">I", 0xF0000000 | (off_ms << 6) | fl)
    else:
        q = struct.pack(">H", ((off_ms // 1000) << 4) | fl)
    return q, v


def random_row(rng, n, dup_p=0.05, diff_p=0.3):
    """Columns of one row: datapoints as single cells, compacted groups and appends."""
    offs = sorted(set(int(x) for x in rng.choice(3600, size=n, replace=False) * 1000 +
                      np.where(rng.random(n) < 0.3, rng.integers(1, 999, n), 0)))
    pts = []
    for o in offs:
        kind = ["long", "int", "float", "double"][int(rng.integers(0, 4))]
        val = float(rng.normal(0, 100)) if kind in ("float", "double") else int(rng.integers(-1000, 1000))
        pts.append((o, o % 1000 != 0 or rng.random() < 0.2, val, kind))
    cells = [_cell(*p) for p in pts]
    cols = []
    i = 0
    while i < len(cells):
        r = rng.random()
        if r < 0.15 and i + 2 < len(cells):            # an earlier compaction of a few datapoints
            k = int(rng.integers(2, 5))
            grp = cells[i:i + k]
            ms = any(len(q) == 4 for q, _ in grp) and any(len(q) == 2 for q, _ in grp)
            cols.append((b"".join(q for q, _ in grp), b"".join(v for _, v in grp) + bytes([1 if ms else 0])))
            i += k
        elif r < 0.25 and i + 1 < len(cells):          # an append column (pairs in any order)
            k = int(rng.integers(1, 4))
            grp = cells[i:i + k]
            order = rng.permutation(len(grp))
            cols.append((bytes([5, 0, 0]), b"".join(grp[j][0] + grp[j][1] for j in order)))
            i += k
        else:
            q, v = cells[i]
            if len(q) == 2 and q[1] & 0xF == 0xB and rng.random() < 0.3:   # float stored on 8 bytes
                v = b"\0\0\0\0" + v
            elif len(q) == 2 and q[1] & 0xF == 0x3 and rng.random() < 0.3:  # int flagged 4, stored on 8
                v = struct.pack(">q", struct.unpack(">i", v)[0])
            cols.append((q, v))
            i += 1
        if rng.random() < dup_p and cells:             # a duplicate of some datapoint
            q, v = cells[int(rng.integers(0, len(cells)))]
            if rng.random() < diff_p:
                v = bytes(b ^ 0x5A for b in v)
            cols.append((q, v))
        if rng.random() < 0.03:
            cols.append((bytes([1, 0, 0]), b'{"note":1}'))   # an annotation
    order = rng.permutation(len(cols))
    ts = rng.permutation(len(cols) * 3)[:len(cols)]
    return [(cols[j][0], cols[j][1], int(ts[k])) for k, j in enumerate(order)]


@pytest.mark.parametrize("seed,fix", [(1, True), (2, True), (3, False), (4, True)])
def test_random_rows_match_oracle(eng, seed, fix):
    rng = np.random.default_rng(seed)
    series, groups = [], []
    for s in range(40):
        rows = []
        for h in range(int(rng.integers(1, 4))):
            rows.append((B + 3600 * (h * 2 + int(rng.integers(0, 2))), random_row(rng, int(rng.integers(1, 60)),
                                                                               dup_p=0.08 if fix else 0.01)))
        series.append(rows)
        groups.append(int(rng.integers(0, 4)))
    order = np.argsort(groups, kind="stable")
    series = [series[i] for i in order]
    groups = [groups[i] for i in order]
    cb = abi.HostCellBatch.from_rows(series, groups, fix)
    eng.load_cells(cb)
    got = rows_of(eng.download())
    want, errs = [], []
    spans = []
    for s, rows in enumerate(series):
        rr = []
        for base, cols in sorted(rows, key=lambda x: x[0]):
            try:
                c = O.compact_row([(q, v) for q, v, _ in cols], fix, [t for _, _, t in cols])
            except O.OracleError as e:
                errs.append((base, e.code))
                continue
            if c is not None:
                rr.append((base, c[0], c[1]))
        want += rr
        spans.append((s, rr))
    assert got == want
    # the queries over the compacted rows, against the oracle over its own compaction
    ref = make_batch(spans, groups)
    for agg, ds in (("sum", "1m-avg"), ("max", "10m-max"), ("none", None), ("zimsum", None)):
        for start, end in ((B, B + 3 * 3600 * 2), (B + 7200, B + 3 * 3600 * 2)):
            q = abi.new_query(start, end, agg)
            if ds:
                d = O.parse_downsample(ds)
                q.ds_function, q.ds_interval_ms = d.ds_function, d.ds_interval_ms
            covered = [c for b, c in errs if start // 3600 * 3600 <= b]
            try:
                w = O.run_query(ref, q)
            except O.OracleError:
                w = None
            if covered:
                with pytest.raises(EngineError):
                    eng.run(q)
                continue
            g = eng.run(q)
            if w is not None:
                assert_groups_match(g, w, agg, ctx=f"{agg} {ds} {start}")


@pytest.mark.parametrize("use_max", [True, False])
@pytest.mark.parametrize("case", DOC["cases"], ids=[c["name"] for c in DOC["cases"]])
def test_known_answer_rows_dtcs_on_gpu(eng, case, use_max):
    """Every known-answer row under tsd.storage.use_otsdb_timestamp (dtcsMergeDataPoints,
    CompactionQueue.java:508-547) with use_max_value true / false: the GPU's cell equals the
    oracle's (no duplicate exception under this merge)."""
    cols, _ = MK.expand_columns(case)
    ts = case.get("timestamps") or list(range(len(cols)))
    cb = abi.HostCellBatch.from_rows([[(B, [(q, v, t) for t, (q, v) in zip(ts, cols)])]], [0],
                                     case["fix_duplicates"], True, use_max)
    eng.load_cells(cb)
    got = rows_of(eng.download())
    try:
        want = O.compact_row(cols, case["fix_duplicates"], ts, use_otsdb_timestamp=True, use_max_value=use_max)
    except O.OracleError as e:
        assert got == []
        with pytest.raises(EngineError) as ge:
            eng.run(abi.new_query(B, B + 3599, "sum"))
        assert ge.value.code == e.code
        return
    assert got == ([] if want is None else [(B, want[0], want[1])])


def random_row_dtcs(rng, n):
    """random_row with many repeated offsets: equal and different values of every width, NaN
    floats, second / millisecond duplicates of one offset, and now and then a value
    getCellValueAsDouble cannot read (a 3-byte integer)."""
    cols = random_row(rng, n, dup_p=0.35, diff_p=0.6)
    out = []
    for q, v, t in cols:
        r = rng.random()
        if len(q) == 2 and not (q[1] & 8) and r < 0.05:       # the same second as a ms qualifier
            off = (int.from_bytes(q, "big") >> 4) * 1000
            q2, v2 = _cell(off, True, int(rng.integers(-50, 50)), "int")
            out.append((q2, v2, int(rng.integers(0, 10**6))))
        elif len(q) == 2 and (q[1] & 0xB) == 0xB and r < 0.1:  # a NaN float duplicate
            out.append((q, struct.pack(">f", float("nan")), int(rng.integers(0, 10**6))))
        elif r < 0.004:                                       # an unreadable 3-byte integer
            out.append((bytes([q[0], (q[1] & 0xF0) | 2]) if len(q) == 2 else q, b"\x00\x01\x02", t))
            continue
        out.append((q, v, t))
    return out


@pytest.mark.parametrize("seed,use_max", [(61, True), (62, False), (63, True), (64, False)])
def test_random_rows_dtcs_match_oracle(eng, seed, use_max):
    """Randomized scans with repeated offsets under dtcsMergeDataPoints against the oracle, row by
    row; rows the oracle rejects raise the same exception from a covering query."""
    rng = np.random.default_rng(seed)
    series, groups = [], []
    for s in range(40):
        series.append([(B + 3600 * h, random_row_dtcs(rng, int(rng.integers(1, 60)))) for h in range(2)])
        groups.append(s // 10)
    cb = abi.HostCellBatch.from_rows(series, groups, False, True, use_max)
    eng.load_cells(cb)
    got = rows_of(eng.download())
    want, errs = [], []
    for rows in series:
        for base, cols in rows:
            try:
                c = O.compact_row([(q, v) for q, v, _ in cols], False, [t for _, _, t in cols],
                                  use_otsdb_timestamp=True, use_max_value=use_max)
            except O.OracleError as e:
                errs.append((base, e.code))
                continue
            if c is not None:
                want.append((base, c[0], c[1]))
    assert got == want
    if errs:
        with pytest.raises(EngineError):
            eng.run(abi.new_query(B, B + 7199, "sum"))


@pytest.mark.parametrize("seed", [5, 6])
def test_pinned_scan_buffers(eng, seed):
    """The scan assembled in page-locked host memory (tsdbhip_host_alloc, engine.pinned_copy --
    the path whose use-after-free crashed in round 3): the compacted rows equal those of the
    same scan from pageable memory, repeated loads included, and queries agree with the oracle."""
    import gc

    from opentsdb_amd.engine import pinned_copy
    rng = np.random.default_rng(seed)
    series, groups = [], []
    for s in range(30):
        series.append([(B + 3600 * h, random_row(rng, int(rng.integers(1, 50)), dup_p=0.05)) for h in range(2)])
        groups.append(s % 3)
    cb = abi.HostCellBatch.from_rows(series, groups, True)
    eng.load_cells(cb)
    want = rows_of(eng.download())
    ref = eng.download()
    for _ in range(3):
        pc = abi.HostCellBatch(*(None if x is None else pinned_copy(x) for x in (cb.series_row_ptr, cb.row_base_time, cb.row_col_ptr,
                                                           cb.col_qual_off, cb.col_val_off, cb.qual, cb.val,
                                                           cb.group_id, cb.col_timestamp)), True)
        eng.load_cells(pc)
        del pc
        gc.collect()   # the pinned blocks may go now: the engine holds its own device copy
        assert rows_of(eng.download()) == want
    q = abi.new_query(B, B + 7199, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    try:
        got = eng.run(q)
    except EngineError:   # a compaction error of some row, raised by the covering query
        return
    assert_groups_match(got, O.run_query(ref, q), "sum", ctx="pinned")


def test_shuffled_single_cells_at_scale(eng):
    """3,000 series x 2 rows of 3,600 one-datapoint cells in shuffled order: the compacted rows
    are the sorted cells plus a meta byte, and the queries equal those over tsdbhip_load."""
    rng = np.random.default_rng(7)
    S, R, N = 3000, 2, 3600
    nrow = S * R
    offs = np.tile(np.arange(N, dtype=np.uint32), nrow).reshape(nrow, N)
    perm = np.argsort(rng.random((nrow, N)), axis=1)
    shuf = np.take_along_axis(offs, perm, axis=1)
    quals = ((shuf << 4) | 7).astype(">u2")
    vals = rng.integers(-10**6, 10**6, size=(nrow, N)).astype(">i8")
    sorted_vals = np.empty_like(vals)
    np.put_along_axis(sorted_vals, shuf.astype(np.int64), vals, axis=1)
    qual = quals.view(np.uint8).reshape(-1)
    val = vals.view(np.uint8).reshape(-1)
    ncol = nrow * N
    cb = abi.HostCellBatch(np.arange(S + 1, dtype=np.int64) * R,
                           (B + 3600 * np.tile(np.arange(R), S)).astype(np.uint32),
                           np.arange(nrow + 1, dtype=np.int64) * N,
                           np.arange(ncol + 1, dtype=np.uint64) * 2, np.arange(ncol + 1, dtype=np.uint64) * 8,
                           qual, val, np.repeat(np.arange(30), S // 30).astype(np.int32),
                           rng.permutation(ncol).astype(np.int64), False)
    eng.load_cells(cb)
    got = eng.download()
    exp_q = ((np.arange(N, dtype=np.uint32) << 4) | 7).astype(">u2").view(np.uint8)
    assert np.array_equal(np.diff(got.row_qual_off.astype(np.int64)), np.full(nrow, 2 * N))
    assert np.array_equal(np.diff(got.row_val_off.astype(np.int64)), np.full(nrow, 8 * N + 1))
    gq = got.qual[:nrow * 2 * N].reshape(nrow, 2 * N)
    assert (gq == exp_q[None, :]).all()
    gv = got.val[:nrow * (8 * N + 1)].reshape(nrow, 8 * N + 1)
    assert (gv[:, -1] == 0).all()
    assert np.array_equal(gv[:, :-1], sorted_vals.view(np.uint8).reshape(nrow, 8 * N))
    q = abi.new_query(B, B + 7199, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    a = eng.run(q)
    eng.load(got)
    b = eng.run(q)
    assert_groups_match(a, b, "sum", tol=0.0)


@pytest.mark.parametrize("seed", [11, 12])
def test_salt_bucket_rows_merge(eng, seed):
    """Two or three scanned rows of one series with the same base time (one per salt bucket):
    each is compacted, then Span.addRow merges the later ones into the first (RowSeq.addRow,
    src/core/Span.java:202-219).  The resident rows equal tsdbhip_load's host merge of the
    oracle's compactions, and the queries equal the oracle's over those rows."""
    rng = np.random.default_rng(seed)
    series, groups, spans = [], [], []
    for s in range(30):
        rows, rr = [], []
        for h in range(int(rng.integers(1, 3))):
            base = B + 3600 * h
            for _ in range(int(rng.integers(1, 4))):   # salt buckets holding this hour
                cols = random_row(rng, int(rng.integers(1, 40)), dup_p=0.0)
                rows.append((base, cols))
                c = O.compact_row([(q, v) for q, v, _ in cols], True, [t for _, _, t in cols])
                if c is not None:
                    rr.append((base, c[0], c[1]))
        series.append(rows)
        spans.append((s, rr))
        groups.append(s % 3)
    order = np.argsort(groups, kind="stable")
    series = [series[i] for i in order]
    spans = [(k, spans[i][1]) for k, i in enumerate(order)]
    groups = [groups[i] for i in order]
    cb = abi.HostCellBatch.from_rows(series, groups, True)
    eng.load_cells(cb)
    got = rows_of(eng.download())
    ref = make_batch(spans, groups)
    eng.load(ref)   # the host merge of tsdbhip_load (RowSeq.addRow restated, pinned by TestRowSeq)
    assert got == rows_of(eng.download())
    eng.load_cells(cb)
    for agg, ds in (("sum", "1m-avg"), ("max", "10m-max"), ("none", None), ("zimsum", None)):
        q = abi.new_query(B, B + 2 * 3600, agg)
        if ds:
            d = O.parse_downsample(ds)
            q.ds_function, q.ds_interval_ms = d.ds_function, d.ds_interval_ms
        assert_groups_match(eng.run(q), O.run_query(ref, q), agg, ctx=f"salt {agg} {ds}")


def _random_scan(seed, n_series=40, salt=False):
    rng = np.random.default_rng(seed)
    series, groups = [], []
    for s in range(n_series):
        rows = []
        for h in range(int(rng.integers(1, 4))):
            for _ in range(int(rng.integers(1, 3)) if salt else 1):
                rows.append((B + 3600 * (h * 2 + int(rng.integers(0, 2))),
                             random_row(rng, int(rng.integers(1, 60)), dup_p=0.0 if salt else 0.05)))
        series.append(rows)
        groups.append(int(rng.integers(-1, 4)))
    order = np.argsort(groups, kind="stable")
    return [series[i] for i in order], [groups[i] for i in order]


@pytest.mark.parametrize("seed,salt", [(21, False), (22, True), (23, False)])
@pytest.mark.parametrize("chunk", [1, 97, 2000])
def test_chunked_compaction_equals_one_pass(eng, seed, salt, chunk):
    """A scan over the 2^31-datapoint chunk limit is compacted in chunks of whole rows (two passes:
    sizes, then entries + writes at the host's layout).  option CMP_CHUNK  lowers the limit so
    small scans take that path: the resident batch, the lazily raised errors and the query results
    equal the one-pass compaction's."""
    series, groups = _random_scan(seed, salt=salt)
    cb = abi.HostCellBatch.from_rows(series, groups, True)
    eng.load_cells(cb)
    want = eng.download()
    qs = []
    for agg, ds in (("sum", "1m-avg"), ("max", "10m-max"), ("none", None)):
        q = abi.new_query(B, B + 6 * 3600, agg)
        if ds:
            d = O.parse_downsample(ds)
            q.ds_function, q.ds_interval_ms = d.ds_function, d.ds_interval_ms
        try:
            qs.append((q, agg, eng.run(q)))
        except EngineError as e:
            qs.append((q, agg, e.code))
    set_option("CMP_CHUNK", chunk)
    try:
        eng.load_cells(cb)
    finally:
        set_option("CMP_CHUNK", None)
    got = eng.download()
    assert rows_of(got) == rows_of(want)
    assert np.array_equal(got.group_id, want.group_id)
    for q, agg, w in qs:
        if isinstance(w, int):
            with pytest.raises(EngineError) as ei:
                eng.run(q)
            assert ei.value.code == w
        else:
            assert_groups_match(eng.run(q), w, agg, tol=0.0, ctx=f"chunk {chunk} {agg}")


def _load_with_opts(eng, cb, **opts):
    for k, v in opts.items():
        set_option(k, v)
    try:
        eng.load_cells(cb)
    finally:
        for k in opts:
            set_option(k, None)
    return eng.download()


def _queries_and_answers(eng):
    out = []
    for agg, ds in (("sum", "1m-avg"), ("max", "10m-max"), ("none", None), ("zimsum", None)):
        q = abi.new_query(B, B + 6 * 3600, agg)
        if ds:
            d = O.parse_downsample(ds)
            q.ds_function, q.ds_interval_ms = d.ds_function, d.ds_interval_ms
        try:
            out.append((q, agg, eng.run(q)))
        except EngineError as e:
            out.append((q, agg, e.code))
    return out


@pytest.mark.parametrize("seed,salt,fix", [(41, False, True), (42, True, True), (43, False, False), (44, False, True)])
def test_row_lds_path_equals_global_sort(eng, seed, salt, fix):
    """The per-row LDS compaction -- one pass (k_cmp_rowone: explode, sort, dedup and the cell
    written into the region the host laid out from k_cmp_cols' bounds), and the sizing + write
    passes (k_cmp_row / k_cmp_rowwrite, option CMP_ONEPASS = 0, and in chunks) -- against the
    global-sort pipeline (option CMP_ROWS = 0): the same resident rows, the same lazily raised
    errors, the same query answers."""
    series, groups = _random_scan(seed, salt=salt)
    cb = abi.HostCellBatch.from_rows(series, groups, fix)
    want = _load_with_opts(eng, cb, CMP_ROWS=0)
    answers = _queries_and_answers(eng)
    for env in ({}, {"CMP_ONEPASS": 0}, {"CMP_CHUNK": 150}):
        got = _load_with_opts(eng, cb, **env)
        assert rows_of(got) == rows_of(want), env
        assert np.array_equal(got.group_id, want.group_id)
        for q, agg, w in answers:
            if isinstance(w, int):
                with pytest.raises(EngineError) as ei:
                    eng.run(q)
                assert ei.value.code == w
            else:
                assert_groups_match(eng.run(q), w, agg, tol=0.0, ctx=f"rows path {env} {agg}")


def test_row_over_lds_capacity_takes_global_sort(eng):
    """A row of more than 4096 datapoints (ms cells of one hour) cannot be sorted in one block: the
    chunk falls back to the global sort; both agree with the oracle's compaction."""
    rng = np.random.default_rng(77)
    offs = np.sort(rng.choice(3_600_000, size=5000, replace=False))
    cols = [_cell(int(o), True, int(rng.integers(-500, 500)), "int") for o in offs]
    order = rng.permutation(len(cols))
    row = [(cols[j][0], cols[j][1], int(k)) for k, j in enumerate(order)]
    small = [(B + 3600, random_row(rng, 40))]
    cb = abi.HostCellBatch.from_rows([[(B, row)], small], [0, 1], True)
    got = _load_with_opts(eng, cb)
    want = O.compact_row([(q, v) for q, v, _ in row], True, [t for _, _, t in row])
    assert rows_of(got)[0] == (B, want[0], want[1])


@pytest.mark.parametrize("chunk", [None, 5])
def test_decreasing_column_offsets_rejected(eng, chunk):
    """Column offsets are checked on the device chunk by chunk: a decreasing offset inside a row
    is an IllegalArgumentException before any compaction kernel reads the bytes."""
    series, groups = _random_scan(31, n_series=6)
    cb = abi.HostCellBatch.from_rows(series, groups, True)
    qo = cb.col_qual_off.copy()
    k = len(qo) // 2
    qo[k] = qo[k + 1] + 2   # column k ends before it starts
    bad = abi.HostCellBatch(cb.series_row_ptr, cb.row_base_time, cb.row_col_ptr, qo, cb.col_val_off, cb.qual,
                            cb.val, cb.group_id, cb.col_timestamp, True)
    if chunk:
        set_option("CMP_CHUNK", chunk)
    try:
        with pytest.raises(EngineError) as ei:
            eng.load_cells(bad)
        assert ei.value.code == abi.TSDB_E_ILLEGAL_ARGUMENT
    finally:
        set_option("CMP_CHUNK", None)


def _single_second_rows(rng, n_rows, dup_row=None, fix_rows=()):
    """Rows of one-datapoint second cells in shuffled order (the one-pass kernel's fast path):
    mixed value kinds; in fix_rows some floats stored as 8 bytes with a 4-byte flag (the
    checkForFixup cases); in dup_row two cells on one second (the general path's dedup)."""
    rows = []
    for r in range(n_rows):
        n = int(rng.integers(1200, 3600))
        secs = np.sort(rng.choice(3600, size=n, replace=False))
        cells = []
        for k, s_ in enumerate(secs):
            kind = ["long", "int", "float", "double"][int(rng.integers(0, 4))]
            val = float(rng.normal(0, 100)) if kind in ("float", "double") else int(rng.integers(-1000, 1000))
            q, v = _cell(int(s_) * 1000, False, val, kind)
            if r in fix_rows and kind == "float" and k % 3 == 0:
                v = b"\x00\x00\x00\x00" + v          # 8 value bytes under a 4-byte float flag
                q = struct.pack(">H", (int(s_) << 4) | 0xB)
            if r in fix_rows and kind == "long" and k % 5 == 0:
                q = struct.pack(">H", (int(s_) << 4) | 0x3)   # flags say 4 bytes, 8 stored: fixed to 8
            cells.append((q, v))
        if r == dup_row:
            cells.append(cells[len(cells) // 2])     # a second cell on one second (same bytes)
        order = rng.permutation(len(cells))
        rows.append((B + 3600 * r, [(cells[j][0], cells[j][1], int(t)) for t, j in enumerate(order)]))
    return rows


@pytest.mark.parametrize("fix", [True, False])
def test_single_cell_fast_path(eng, fix):
    """k_cmp_rowone's fast path (each column at its second) against the global-sort pipeline and
    the oracle's compaction, with fixups and a row whose duplicate second sends it to the general
    path."""
    rng = np.random.default_rng(31)
    rows = _single_second_rows(rng, 6, dup_row=2, fix_rows=(1, 4))
    cb = abi.HostCellBatch.from_rows([rows], [0], fix)
    want = _load_with_opts(eng, cb, CMP_ROWS=0)
    got = _load_with_opts(eng, cb)
    two = _load_with_opts(eng, cb, CMP_ONEPASS=0)
    assert rows_of(got) == rows_of(want)
    assert rows_of(two) == rows_of(want)
    for (base, cells), (gb, gq, gv) in zip(rows, rows_of(got)):
        exp = O.compact_row([(q, v) for q, v, _ in cells], fix, [t for _, _, t in cells])
        assert (gb, gq, gv) == (base, exp[0], exp[1])
