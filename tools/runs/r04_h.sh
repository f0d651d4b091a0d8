#!/bin/bash
# sequential row kernel: parity (fast + rollup suites), rollup read bench under a kernel trace
set -o pipefail
tag=${1:-r04h}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_rollup_read.py tests/test_gpu_rollup.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_ro -o run -- \
  python3 tools/rollup_read_bench.py --check > $out/rollup.jsonl 2> $out/rollup.err || { tail $out/rollup.err; exit 1; }
cat $out/rollup.jsonl
find $out/prof_ro -name '*kernel_stats.csv' -exec cp {} $out/rollup_kernel_stats.csv \;
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open("gpurun_out/r04h/rollup_kernel_stats.csv")))[:10]:
    print(f"  {r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
