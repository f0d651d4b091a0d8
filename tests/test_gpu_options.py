"""Release hygiene on the device: the library reads no environment variable, so a process whose
environment sets every switch earlier rounds read (TSDBHIP_FAST, TSDBHIP_HIST_DBG ... 54 names) to
garbage or to a kernel-changing value returns exactly the bits of a clean process, over queries
that reach every kernel family (streaming, general, percentile, ordered, raw, histogram-free)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# every switch name the library read from the environment up to round 5
OLD_SWITCHES = [
    "FAST", "PCT_KEYS", "TRACE", "RO_PACK", "TILE_MIN", "TILE_DP", "SHORT6", "SHORT", "SEQ_WAVE", "SEQ_ROWS", "SEQ",
    "SEL_WIN", "SEL_WIDE", "SEL_WAVE", "SEL_T", "SEL_STAGE", "SEL_SLOTS", "SEL_REG", "SEL_OCC", "SEL_HL", "SEL_FUSED",
    "SEL_COLS", "SELOPS", "RO_FUSE", "ROW_ALIGN", "ROWS", "RAW_TOP", "RAW_SEL_TOP", "RAW_SEL_REG", "RAW_LERPW", "PULL",
    "PCT_VONLY", "PCT_V6", "PCTROWS", "PCTDV", "PCTD", "ONEB", "MULTI_FUSE", "INDEX_GENERIC", "HWIN_SPLIT", "HWIN",
    "HIST_WS", "HIST_WLDS", "HIST_WINDOW", "HIST_SU", "HIST_PIPE", "HIST_LAYOUT", "HIST_DBG", "EMIT_REG",
    "DENSE_SPLIT", "DBG", "CMP_ROWS", "CMP_ONEPASS", "CMP_CHUNK"]

CHILD = r'''
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
from opentsdb_amd import abi, synth
from opentsdb_amd.engine import Engine
T0 = 1356998400
eng = Engine(0)
out = {}
def digest(groups):
    h = hashlib.sha256()
    for g, ts, bits, isi in groups:
        h.update(str(int(g)).encode()); h.update(ts.tobytes()); h.update(bits.tobytes()); h.update(isi.tobytes())
    return h.hexdigest()
eng.synth(3000, T0, 3600, 1000, 2, 16, 30000, 0x5EED)          # long rows: k_fast
for agg, ds, iv in [("sum", "avg", 60000), ("dev", "avg", 60000), ("p99", "avg", 60000), ("max", "p95", 300000)]:
    out[f"long-{agg}-{ds}"] = digest(eng.run(abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG[ds], ds_interval_ms=iv)))
out["long-ordered"] = digest(eng.run(abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000,
                                                   flags=abi.QF_ORDERED)))
eng.synth(20000, T0, 360, 10000, 2, 50, 30000, 0x5EED)         # one-row series: k_short, the selects
for agg in ("sum", "avg", "p99", "median"):
    out[f"short-{agg}"] = digest(eng.run(abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)))
out["short-multi"] = [digest(r) for r in eng.run_multi([abi.new_query(T0, T0 + 3599, a, ds_function=abi.AGG["avg"],
                                                                      ds_interval_ms=60000) for a in ("min", "count", "dev")])]
eng.synth(600, T0, 8640, 10000, 2, 7, 30000, 0x5EED)           # a day: k_hwin / k_rows
for iv in (60000, 3600000):
    out[f"day-{iv}"] = digest(eng.run(abi.new_query(T0, T0 + 86399, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=iv)))
eng.load(synth.generate_counters(300, T0, 360, n_groups=5, seed=9))   # raw union path
out["raw-sum"] = digest(eng.run(abi.new_query(T0, T0 + 3599, "sum")))
out["raw-p90-rate"] = digest(eng.run(abi.new_query(T0, T0 + 3599, "p90", rate=True, counter=True)))
eng.close()
print(json.dumps(out))
'''


def run_child(env):
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-3000:]
    return json.loads(r.stdout.decode().strip().splitlines()[-1])


@pytest.mark.parametrize("value", ["zzz", "0", "2", "1"])
def test_environment_cannot_change_results(value):
    clean = {k: v for k, v in os.environ.items() if not k.startswith("TSDBHIP_")}
    want = run_child(clean)
    dirty = dict(clean, **{"TSDBHIP_" + n: value for n in OLD_SWITCHES})
    got = run_child(dirty)
    assert got == want


def test_developer_options_keep_the_answers():
    """The options the tests use to force alternatives are bit-identical (or oracle-equal)
    routes to the same answer: flipping all of them at once on the order-free integer queries
    leaves the bits unchanged."""
    from opentsdb_amd import abi
    from opentsdb_amd import engine as E
    T0 = 1356998400
    eng = E.Engine(0)
    try:
        eng.synth(4000, T0, 360, 10000, 1, 20, 2000, 0x5EED)
        qs = [abi.new_query(T0, T0 + 3599, a, ds_function=abi.AGG[d], ds_interval_ms=60000)
              for a, d in (("min", "max"), ("max", "min"), ("count", "sum"), ("p99", "avg"), ("median", "sum"))]
        want = [eng.run(q) for q in qs]
        with E.options(FAST=0, SEL_WAVE=0, SEL_WIN=0, SEL_COLS=0, SEL_FUSED=0, MULTI_FUSE=0):
            got = [eng.run(q) for q in qs]
        for w, g in zip(want, got):
            assert len(w) == len(g)
            for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(w, g):
                assert g1 == g2 and np.array_equal(t1, t2) and np.array_equal(b1, b2) and np.array_equal(i1, i2)
    finally:
        eng.close()
