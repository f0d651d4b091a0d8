"""Rollup generation and query-time compaction on the one-process multi-device context
(tsdbhip_init_devices): every device rolls up / compacts its own series; the result must be what
one GPU returns for the same input -- rollup cells byte for byte in the one-GPU order (function,
batch series, time), compacted stores answering every query as the one-GPU store does.
References: src/rollup/RollupUtils.java:52-171 (the cells), src/core/CompactionQueue.java:267-626
(the compaction).  Devices are emulated by repeating GPU 0 (peer copies), as in
tests/test_gpu_multidev.py."""
from __future__ import annotations

import numpy as np
import pytest

from opentsdb_amd import abi, synth
from opentsdb_amd import engine as E
from oracle import rollup as R
from tests.test_gpu_compaction import _random_scan, B
from tests.test_gpu_multidev import bit_same

pytestmark = pytest.mark.gpu

T0 = 1356998400
FUNCS = (("sum", 0), ("count", 1), ("max", 2), ("min", 3))


def cells_of(eng, interval, span, start, end, funcs=FUNCS):
    c = eng.rollup(E.rollup_interval(interval, span), start, end, funcs)
    return [c.cell(i) for i in range(len(c))]


@pytest.fixture(scope="module")
def batch():
    """120 series, 1 day @10 s, int/float alternating, 7 groups interleaved in batch order (group
    sorting moves series away from batch order), every 11th series without a group."""
    b = synth.generate(120, T0, 8640, 10000, value_kind=2, n_groups=7, int_mod=30000, seed=0x5EED)
    gid = b.group_id.copy()
    gid[::11] = -1
    return abi.HostBatch(b.series_row_ptr, b.row_base_time, b.row_qual_off, b.row_val_off, b.qual, b.val, gid)


@pytest.mark.parametrize("mode", [E.SHARD_SERIES, E.SHARD_GROUPS])
@pytest.mark.parametrize("world", [2, 3])
def test_md_rollup_cells_equal_one_gpu(batch, mode, world):
    one = E.Engine(0)
    md = E.Engine(devices=[0] * world)
    try:
        one.load(batch)
        md.shard_mode(mode)
        md.load(batch)
        assert (md.md_info()[3] > 0).sum() >= 2
        for iv, span, st, en, funcs in (("1h", "1d", T0, T0 + 86400, FUNCS), ("1d", "1n", T0, T0 + 86400, FUNCS),
                                        ("10m", "1d", T0 + 3600, T0 + 7 * 3600, (("min", 7), ("sum", 42)))):
            want = cells_of(one, iv, span, st, en, funcs)
            got = cells_of(md, iv, span, st, en, funcs)
            assert want and got == want, (iv, span, mode, world)
        # the one-GPU cells are the oracle's (tests/test_gpu_rollup.py); once more here
        exp = R.generate(batch, R.Interval("1h", "1d"), T0, T0 + 86400, FUNCS)
        assert cells_of(md, "1h", "1d", T0, T0 + 86400) == exp
    finally:
        md.close()
        one.close()


@pytest.mark.parametrize("mode", [E.SHARD_SERIES, E.SHARD_GROUPS])
def test_md_rollup_synth_store(mode):
    """The device-synthesized store (each device generates its shard): cells in device order."""
    args = (3000, T0, 8640, 10000, 2, 64, 30000, 0x5EED)
    one = E.Engine(0)
    md = E.Engine(devices=[0, 0, 0, 0])
    try:
        one.synth(*args)
        md.shard_mode(mode)
        md.synth(*args)
        for iv, span in (("1h", "1d"), ("1d", "1n")):
            n1, b1 = one.rollup_run(E.rollup_interval(iv, span), T0, T0 + 86400)
            n2, b2 = md.rollup_run(E.rollup_interval(iv, span), T0, T0 + 86400)
            assert (n1, b1) == (n2, b2)
            c1 = one.rollup_download(n1, b1)
            c2 = md.rollup_download(n2, b2)
            for f in ("series", "base_time", "qualifier", "val_off", "value"):
                np.testing.assert_array_equal(getattr(c1, f), getattr(c2, f), err_msg=f"{iv}/{span} {f}")
    finally:
        md.close()
        one.close()


def test_md_rollup_download_before_run_refused(batch):
    md = E.Engine(devices=[0, 0])
    try:
        md.load(batch)
        with pytest.raises(E.EngineError) as ei:
            md.rollup_download(1, 1)
        assert ei.value.code == abi.TSDB_E_ILLEGAL_STATE
    finally:
        md.close()


QUERIES = [("sum", "1m-avg"), ("max", "10m-max"), ("min", "1m-min"), ("count", "1m-sum"), ("p99", "10m-avg"),
           ("none", None), ("zimsum", None)]


def _queries():
    from oracle import oracle as O
    out = []
    for agg, ds in QUERIES:
        q = abi.new_query(B, B + 6 * 3600, agg)
        if ds:
            d = O.parse_downsample(ds)
            q.ds_function, q.ds_interval_ms = d.ds_function, d.ds_interval_ms
        out.append((agg, q))
    return out


def _answers(eng):
    res = []
    for agg, q in _queries():
        try:
            res.append(eng.run(q))
        except E.EngineError as e:
            res.append(e.code)
    return res


@pytest.mark.parametrize("seed,salt,fix", [(51, False, True), (52, True, True), (53, False, False)])
@pytest.mark.parametrize("mode", [E.SHARD_SERIES, E.SHARD_GROUPS])
def test_md_load_cells_equals_one_gpu(seed, salt, fix, mode):
    """tsdbhip_load_cells on the multi-device context: each device compacts its series' rows (salt
    buckets merged per series, duplicates, fix_duplicates); every query -- decomposable, order
    statistic, NONE, raw -- and every lazily raised compaction exception as on one GPU."""
    series, groups = _random_scan(seed, n_series=60, salt=salt)
    cb = abi.HostCellBatch.from_rows(series, groups, fix)
    one = E.Engine(0)
    md = E.Engine(devices=[0, 0, 0])
    try:
        one.load_cells(cb)
        md.shard_mode(mode)
        md.load_cells(cb)
        assert (md.md_info()[3] > 0).sum() >= 2
        for (agg, _), w, g in zip(_queries(), _answers(one), _answers(md)):
            if isinstance(w, int):
                assert g == w, (agg, g, w)
            elif agg in ("sum", "zimsum") and mode == E.SHARD_SERIES:
                from tests.test_gpu_parity import assert_groups_match
                assert_groups_match(g, w, agg, ctx=f"cells {agg}")
            else:
                bit_same(g, w, f"cells {agg}")
    finally:
        md.close()
        one.close()
