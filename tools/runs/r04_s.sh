#!/bin/bash
# compaction one-pass (word-wide cell assembly, 32-bit row sums) + A/B of the one-bucket fold code
# on configs 2 / 3 (libtsdbhip vs a build without it)
set -o pipefail
out=gpurun_out/r04s; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_compaction.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cmp -o run -- \
  python3 tools/compact_bench.py 20000 3600 3 > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
cat $out/compact.jsonl
find $out/prof_cmp -name '*kernel_stats.csv' -exec cp {} $out/compact_kernel_stats.csv \;
TSDBHIP_CMP_ONEPASS=0 timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 > $out/compact_twopass.jsonl 2> $out/compact_twopass.err || exit 1
cat $out/compact_twopass.jsonl
python3 - "$out" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/compact_kernel_stats.csv")))[:6]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
for c in 2 3; do
  timeout -k 10 300 python3 tools/ab_lib.py --libs opentsdb_amd/lib/exp_nooneb.so,opentsdb_amd/lib/libtsdbhip.so,opentsdb_amd/lib/exp_nooneb.so,opentsdb_amd/lib/libtsdbhip.so --config $c --fns sum --steps 20 > $out/ab_c$c.jsonl 2> $out/ab_c$c.err || { tail $out/ab_c$c.err; exit 1; }
  cat $out/ab_c$c.jsonl
done
