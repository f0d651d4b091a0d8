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
e = E.Engine(0)
def vals(res, n=6):
    return [(g, ts[:n].tolist(), b[:n].view(np.float64).tolist()) for g, ts, b, _ in res[:2]]
print("oracle", vals(want))
e.load_rollup(table)
print("single", vals(e.run(q)))
for name, rb in (("shard1", dist.shard_rollup_batch(table, 0, 1)), ("orig", table)):
    e.load_rollup(rb)
    lay = e.partials_layout(q, G)
    buf = np.zeros(int(lay.bytes), np.uint8)
    e.run_partials(q, G, buf.ctypes.data)
    print(name, "partials", vals(e.finalize(q, G, buf.ctypes.data, 1)))
    print(name, "run", vals(e.run(q)))
e2 = E.Engine(0)
e2.load_rollup(dist.shard_rollup_batch(table, 0, 1))
lay = e2.partials_layout(q, G)
buf = np.zeros(int(lay.bytes), np.uint8)
e2.run_partials(q, G, buf.ctypes.data)
print("fresh shard1 partials", vals(e2.finalize(q, G, buf.ctypes.data, 1)))
