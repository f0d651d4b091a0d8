#!/bin/bash
# k_hwin (K > 64 buckets tiling the hour): fast / parity suites, config-3 day shard with k_hwin on and off
set -o pipefail
out=gpurun_out/r04x; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_calendar.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
TSDBHIP_HWIN=0 timeout -k 10 300 python3 tools/c3day_bench.py > $out/c3day_hwin0.jsonl 2> $out/c3day_hwin0.err || { tail $out/c3day_hwin0.err; exit 1; }
cat $out/c3day_hwin0.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/c3day_bench.py > $out/c3day.jsonl 2> $out/c3day.err || { tail $out/c3day.err; exit 1; }
cat $out/c3day.jsonl
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/c3day_kernel_stats.csv \;
python3 - "$out" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/c3day_kernel_stats.csv")))[:10]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
