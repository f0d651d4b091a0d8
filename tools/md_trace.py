"""Host phases of the multi-device query path (developer option TRACE=1 prints them on stderr):
config 3's shape at --series over GPU 0 repeated --devices times.
   python tools/md_trace.py [--series 2000000] [--devices 2] [--steps 3]"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opentsdb_amd import abi  # noqa: E402
from opentsdb_amd.engine import SHARD_GROUPS, SHARD_SERIES, Engine, set_option  # noqa: E402

T0 = 1356998400


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=2_000_000)
    ap.add_argument("--devices", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--hours", type=int, default=1)
    ap.add_argument("--shard", default="series", choices=("series", "groups"))
    a = ap.parse_args()
    eng = Engine(devices=[0] * a.devices, transport=0)
    eng.shard_mode(SHARD_SERIES if a.shard == "series" else SHARD_GROUPS)
    eng.synth(a.series, T0, a.hours * 360, 10000, 2, 1000, 30000, 0x5EED)
    eng.sync()

    def q(agg):
        return abi.new_query(T0, T0 + a.hours * 3600 - 1, agg, ds_function=abi.AGG["avg"], ds_interval_ms=60000)
    ql = [q(x) for x in ("avg", "min", "max", "count", "dev")]
    for name, fn in (("sum", lambda: eng.run(q("sum"))), ("multi5", lambda: eng.run_multi(ql))):
        fn()
        for _ in range(a.steps):
            set_option("TRACE", 1)
            t = time.perf_counter()
            r = fn()
            ms = (time.perf_counter() - t) * 1000
            set_option("TRACE", 0)
            tm = eng.timing()
            print(f"{name}: {ms:.3f} ms  assemble_ms {tm.assemble_ms:.3f}", file=sys.stderr, flush=True)
            del r
    eng.close()


if __name__ == "__main__":
    main()
