"""Config 3 (10M x 360, 1000 groups) sum:1m-avg with the TRACE option's phase marks: where the host
time of a step goes beyond the streaming kernels."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0 = 1356998400
from opentsdb_amd import abi  # noqa: E402
from opentsdb_amd.engine import Engine  # noqa: E402
from opentsdb_amd.engine import set_option  # noqa: E402

set_option("TRACE", 1)   # the library's phase marks on stderr

eng = Engine(0)
eng.synth(10_000_000, T0, 360, 10000, 2, 1000, 30000, 0x5EED)
eng.sync()
q = abi.new_query(T0, T0 + 3599, "sum", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
for i in range(5):
    t = time.perf_counter()
    r = eng.run(q)
    dt = (time.perf_counter() - t) * 1000
    tm = eng.timing()
    print(f"step {i}: {dt:.3f} ms (C call {eng.last_call_ms:.3f}), fast {tm.fast_ms:.3f} dd {tm.decode_downsample_ms:.3f} red {tm.group_reduce_ms:.3f}", file=sys.stderr, flush=True)
