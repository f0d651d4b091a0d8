"""Config 3's day shard, sum:1m-avg only, with the TRACE option's phase marks (host wall time of the
call's phases on stderr) and the Python-side result conversion timed separately."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0 = 1356998400
from opentsdb_amd import abi  # noqa: E402
from opentsdb_amd.engine import Engine  # noqa: E402
from opentsdb_amd.engine import set_option  # noqa: E402

set_option("TRACE", 1)   # the library's phase marks on stderr

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
eng = Engine(0)
eng.synth(n, T0, 8640, 10000, 2, 1000, 30000, 0x5EED)
eng.sync()
q = abi.new_query(T0, T0 + 86399, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
for i in range(4):
    t = time.perf_counter()
    r = eng.run(q)
    dt = (time.perf_counter() - t) * 1000
    print(f"step {i}: {dt:.3f} ms, groups {len(r)}", file=sys.stderr, flush=True)
