"""Config 4 (raw union path) step breakdown (argv: series, steps, queries = sum,rate[,p99]): wall time of the C call, of the Python result
wrapping, and the device time the library reports.  the TRACE option adds the library's own
phase marks on stderr."""
import ctypes as C
import json
import sys
import time

sys.path.insert(0, ".")
from opentsdb_amd import abi, synth  # noqa: E402
from opentsdb_amd.engine import Engine, lib, _check  # noqa: E402
from opentsdb_amd.engine import set_option  # noqa: E402

set_option("TRACE", 1)   # the library's phase marks on stderr

T0 = 1356998400


def main():
    series = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    b = synth.generate_counters(series, T0, 360, n_groups=64, seed=0x5EED)
    eng = Engine(0)
    eng.load(b)
    qs = {"sum": abi.new_query(T0, T0 + 3599, "sum"),
          "rate": abi.new_query(T0, T0 + 3599, "sum", rate=True, counter=True, counter_max=1 << 32,
                                reset_value=1000000),
          "p99": abi.new_query(T0, T0 + 3599, "p99")}
    only = sys.argv[3].split(",") if len(sys.argv) > 3 else ["sum", "rate"]
    qs = {k: v for k, v in qs.items() if k in only}
    for name, q in qs.items():
        eng.run(q)
        call, wrap, dev = [], [], []
        for _ in range(steps):
            res = C.POINTER(abi.Result)()
            t = time.perf_counter()
            _check(lib().tsdbhip_run(eng.ctx, C.byref(q), C.byref(res)))
            t1 = time.perf_counter()
            from opentsdb_amd.engine import _ResultOwner
            abi.result_to_groups(res.contents, owner=_ResultOwner(res))
            t2 = time.perf_counter()
            call.append((t1 - t) * 1000)
            wrap.append((t2 - t1) * 1000)
            dev.append(eng.timing().decode_downsample_ms)
        print(json.dumps({"query": name, "c_call_ms": sum(call) / steps, "wrap_ms": sum(wrap) / steps,
                          "device_ms": sum(dev) / steps, "points": int(eng.timing().datapoints)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
