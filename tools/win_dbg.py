"""Debug: p99:1m-avg group-by on a device-synthesised tied integer batch under engine variants,
group 0 slots 0-5, against the oracle on the downloaded batch."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0 = 1356998400
ARGS = (20_000, T0, 360, 10000, 1, 2, 3, 0x51)
if len(sys.argv) > 1:
    from opentsdb_amd import abi
    from opentsdb_amd.engine import Engine
    e = Engine(0)
    e.synth(*ARGS)
    q = abi.new_query(T0, T0 + 3599, "p99", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    r = e.run(q)
    print(sys.argv[1], [hex(int(x)) for x in r[0][2][:6]], flush=True)
    if sys.argv[1] == "oracle":
        from oracle import oracle as O
        b = e.download()
        w = O.run_query(b, q, threads=8)
        print("oracle", [hex(int(x)) for x in w[0][2][:6]], flush=True)
        # the bucket values of slot 3 in group 0: distinct values near the top
        import numpy as np
        qn = abi.new_query(T0, T0 + 3599, "none", ds_function=abi.AGG["avg"], ds_interval_ms=60000)
        rn = e.run(qn)
        vals = []
        for gid, ts, bits, isi in rn[:10000]:
            if len(bits) > 3:
                v = bits[3].view(np.float64) if not isi[3] else float(np.int64(bits[3]))
                vals.append((float(v), int(isi[3])))
        from collections import Counter
        print("gpu none slot 3 top values", sorted(Counter(vals).items())[-6:], flush=True)
        wn = O.run_query(b, qn, threads=8)
        vals = []
        for gid, ts, bits, isi in wn[:10000]:
            if len(bits) > 3:
                v = bits[3].view(np.float64) if not isi[3] else float(np.int64(bits[3]))
                vals.append((float(v), int(isi[3])))
        print("oracle none slot 3 top values", sorted(Counter(vals).items())[-6:], flush=True)
    sys.exit(0)
for name, env in [("full", {"TSDBHIP_SEL_WIN": "0"}), ("nofused", {"TSDBHIP_SEL_WIN": "0", "TSDBHIP_SEL_FUSED": "0"}),
                  ("oracle", {"TSDBHIP_SEL_WIN": "0"})]:
    subprocess.run([sys.executable, __file__, name], env={**os.environ, **env}, check=True, timeout=300)
