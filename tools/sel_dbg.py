"""Debug: the percentile group-by on a small mixed batch under the select-kernel variants
(TSDBHIP_SEL_* environment), values of group 0 side by side."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0 = 1356998400

if len(sys.argv) > 1 and sys.argv[1] == "child":
    import numpy as np
    from opentsdb_amd import abi, synth
    from opentsdb_amd.engine import Engine
    b = synth.generate(70, T0, 720, 5000, value_kind=2, n_groups=3, int_mod=30000, seed=11)
    e = Engine(0)
    out = {}
    for agg in ["p999", "p99", "median", "p50"]:
        q = abi.new_query(T0, T0 + 3599, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        r = e.run_batch(b, q)
        gid, ts, bits, isi = r[0]
        print(agg, [hex(int(x)) for x in bits[:8]], flush=True)
    sys.exit(0)

for env in [{"TSDBHIP_SEL_HL": "0"}, {}, {"TSDBHIP_SEL_BUF": "0"}, {"TSDBHIP_SEL_T": "1024"}]:
    print("==", env, flush=True)
    subprocess.run([sys.executable, __file__, "child"], env={**os.environ, **env}, check=True, timeout=120)
