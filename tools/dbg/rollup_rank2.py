import sys
import numpy as np
sys.path.insert(0, ".")
from opentsdb_amd import dist
from opentsdb_amd import engine as E
from oracle import oracle as O
from tests.test_gpu_rollup_read import B, _q, random_table

rng = np.random.default_rng(2024)
table = random_table(rng, 40, 6, 3, floats=True)
END = B + 2 * 86400 + 3600
q = _q("10m-avg", "avg", start=B + 1800, end=END)
want = O.run_rollup_query(table, q)
G = dist.n_groups_of(table.cells)

def cmp(tag, got):
    bad = []
    for (g1, t1, b1, i1), (g2, t2, b2, i2) in zip(got, want):
        a, b = b1.view(np.float64), b2.view(np.float64)
        d = np.nonzero(~((a == b) | (np.abs(a - b) <= 1e-12 * np.maximum(1, np.abs(b))) | (np.isnan(a) & np.isnan(b))))[0]
        if len(d):
            bad.append((g1, d[:6].tolist(), a[d[:4]].tolist(), b[d[:4]].tolist()))
    print(tag, "OK" if not bad else bad, flush=True)

def rank(e, rb):
    e.load_rollup(rb)
    lay = e.partials_layout(q, G)
    buf = np.zeros(int(lay.bytes), np.uint8)
    e.run_partials(q, G, buf.ctypes.data)
    return e.finalize(q, G, buf.ctypes.data, 1)

e0 = E.Engine(0)
cmp("fresh rank", rank(e0, dist.shard_rollup_batch(table, 0, 1)))
cmp("fresh rank again", rank(e0, dist.shard_rollup_batch(table, 0, 1)))
e0.load_rollup(table)
cmp("fresh run", e0.run(q))
cmp("rank after run", rank(e0, dist.shard_rollup_batch(table, 0, 1)))
md = E.Engine(devices=[0, 0])
md.shard_mode(E.SHARD_SERIES)
md.load_rollup(table)
cmp("md series", md.run(q))
md.close()
cmp("rank after md", rank(e0, dist.shard_rollup_batch(table, 0, 1)))
es = [E.Engine(0) for _ in range(4)]
cmp("new engine rank", rank(es[0], dist.shard_rollup_batch(table, 0, 1)))
