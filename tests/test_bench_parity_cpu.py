"""bench.py's self-check of the N-GPU answer (no GPU needed): the group geometry of the synthetic
store, the comparison bar, the rank merge of the stats over gloo, and the multi-device
supervisor's outcomes (a parity failure is final, an RCCL failure is surfaced at top level)."""
from __future__ import annotations

import json
import os
import socket
import sys
import types

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from opentsdb_amd import synth  # noqa: E402


@pytest.mark.parametrize("n,G", [(103, 7), (64, 64), (1000, 61), (5, 8)])
def test_group_span_matches_series_order(n, G):
    _, grp = synth.series_order(n, G)
    for g in range(G):
        p0, p1 = bench.group_span(n, G, g)
        assert np.all(grp[p0:p1] == g) and (p1 - p0) == np.count_nonzero(grp == g)
    for p in range(n):
        assert bench.group_at(n, G, p) == grp[p]


def test_checked_groups_take_the_shard_edges():
    n, G = 48000, 61
    bounds = [0, 24000, 48000]
    gs = bench.checked_groups(n, G, bounds)
    assert bench.group_at(n, G, 23999) in gs and bench.group_at(n, G, 24000) in gs
    assert 0 in gs and G - 1 in gs and len(gs) <= 10
    # whole groups per shard: the groups on both sides of the edge
    gs = bench.checked_groups(8_000_000, 64, [0, 4_000_000, 8_000_000])
    assert {31, 32} <= set(gs)


def grp(ts, vals, ints=None):
    ts = np.asarray(ts, np.int64)
    bits = np.asarray(vals, np.float64).view(np.uint64)
    return ts, bits, np.zeros(len(ts), np.uint8) if ints is None else np.asarray(ints, np.uint8)


def test_compare_groups_bar():
    want = {0: grp([1, 2], [1.0, 2.0]), 3: grp([1], [float("nan")])}
    assert not bench.compare_groups(want, want, "sum")["mismatch"]
    near = {0: grp([1, 2], [1.0, 2.0 * (1 + 1e-13)]), 3: grp([1], [float("nan")])}
    st = bench.compare_groups(near, want, "sum")
    assert not st["mismatch"] and 0 < st["max_rel_err"] < 1e-12 and st["bit_exact_points"] == 2
    assert bench.compare_groups(near, want, "max")["mismatch"]               # order statistic: exact
    assert bench.compare_groups(near, want, "sum", exact=True)["mismatch"]   # ordered fold: exact
    far = {0: grp([1, 2], [1.0, 2.1]), 3: grp([1], [float("nan")])}
    assert bench.compare_groups(far, want, "avg")["mismatch"]
    assert bench.compare_groups({0: want[0]}, want, "sum")["mismatch"] == ["group 3 missing"]
    shifted = {0: grp([1, 3], [1.0, 2.0]), 3: want[3]}
    assert "timestamps" in bench.compare_groups(shifted, want, "sum")["mismatch"][0]
    ints = {0: grp([1], [0.0], [1])}
    other = {0: (ints[0][0], ints[0][1] + np.uint64(1), ints[0][2])}
    assert "integer" in bench.compare_groups(other, ints, "dev")["mismatch"][0]


def test_parity_block_and_all_ok():
    st = {"sum": {"groups": 2, "points": 4, "bit_exact_points": 4, "max_rel_err": 0.0, "tol": 1e-12, "mismatch": []},
          "p99": {"skipped": "refused"}}
    blk = bench.parity_block(st, [0, 5], "x")
    assert blk["ok"] and blk["checked"] == ["sum"] and blk["queries"]["p99"] == {"skipped": "refused"}
    st["sum"]["mismatch"] = ["group 0: max relative error 1 > 1e-12"]
    bad = bench.parity_block(st, [0, 5], "x")
    assert not bad["ok"] and "sum" in bad["mismatch"]
    assert bench.parity_all_ok(blk, {"config3": {"parity": blk}})
    assert not bench.parity_all_ok(blk, {"config3": {"parity": bad}})
    assert not bench.parity_all_ok(dict(blk, straddle=bad), None)
    assert not bench.parity_block({"p99": {"skipped": "r"}}, [], "x")["ok"]   # nothing checked


def _args(**kw):
    d = dict(transport="auto", md_timeout=10.0)
    d.update(kw)
    return types.SimpleNamespace(**d)


LINE = json.dumps({"metric": "m", "value": 1.0, "parity": {"ok": True}})


def test_supervisor_clean_run(capsys):
    calls = []
    rc = bench.md_supervise(_args(), child=lambda extra: calls.append(extra) or (0, LINE, ""))
    assert rc == 0 and calls == [[]]
    assert json.loads(capsys.readouterr().out)["value"] == 1.0


def test_supervisor_rccl_failure_reruns_over_copies(capsys):
    calls = []

    def child(extra):
        calls.append(extra)
        return (None, None, "ncclCommInitAll: unhandled system error") if not extra else (0, LINE, "")
    rc = bench.md_supervise(_args(), child=child)
    assert rc == 0 and calls == [[], ["--transport", "copy"]]
    d = json.loads(capsys.readouterr().out)
    assert d["rccl_failed"] is True and "ncclCommInitAll" in d["rccl_error"] and "time-out" in d["rccl_error"]


def test_supervisor_parity_failure_is_final(capsys):
    calls = []
    bad = json.dumps({"value": 1.0, "parity": {"ok": False}})
    rc = bench.md_supervise(_args(), child=lambda extra: calls.append(extra) or (1, bad, "mismatch"))
    assert rc == 1 and calls == [[]]   # a wrong answer is not retried over another transport
    assert json.loads(capsys.readouterr().out)["parity"]["ok"] is False


def test_supervisor_refusals_and_double_failure(capsys):
    assert bench.md_supervise(_args(), child=lambda extra: (2, None, "only 1 GPU")) == 2
    assert bench.md_supervise(_args(transport="rccl"), child=lambda extra: (1, None, "x")) == 1
    rc = bench.md_supervise(_args(), child=lambda extra: (134, None, "abort"))
    assert rc == 134 and not capsys.readouterr().out.strip()


def _merge_worker(rank, world, port, out):
    import torch.distributed as td
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = {"sum": {"groups": 1, "points": 10 + rank, "bit_exact_points": 10, "max_rel_err": 1e-15 * (rank + 1),
                      "tol": 1e-12, "mismatch": ["group 9: x"] if rank == 1 else []},
              "p99": {"groups": 1, "points": 5, "bit_exact_points": 5, "max_rel_err": 0.0, "tol": 0.0, "mismatch": []}}
        m = bench.merge_rank_stats(td, "cpu", st)
        with open(os.path.join(out, f"m{rank}.json"), "w") as f:
            json.dump(m, f)
    finally:
        td.destroy_process_group()


def test_merge_rank_stats_gloo(tmp_path):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_merge_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        m = json.load(open(tmp_path / f"m{r}.json"))
        assert m["sum"]["points"] == 21 and m["sum"]["groups"] == 2 and m["sum"]["max_rel_err"] == 2e-15
        assert len(m["sum"]["mismatch"]) == 1   # rank 1's message, or "1 on other ranks" on rank 0
        assert m["p99"]["points"] == 10 and not m["p99"]["mismatch"]
