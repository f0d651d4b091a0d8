#!/bin/bash
# one-pass row compaction (k_cmp_rowone): compaction GPU tests, then compact_bench (shuffled under
# rocprofv3, scan order, and the two-pass path for comparison); config 5 p99 / median (no per-lane sort
# before the mid-rank search)
set -o pipefail
out=gpurun_out/r04r; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_compaction.py tests/test_gpu_pct.py tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cmp -o run -- \
  python3 tools/compact_bench.py 20000 3600 3 > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
cat $out/compact.jsonl
find $out/prof_cmp -name '*kernel_stats.csv' -exec cp {} $out/compact_kernel_stats.csv \;
timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 --scan-order > $out/compact_scan.jsonl 2> $out/compact_scan.err || exit 1
cat $out/compact_scan.jsonl
TSDBHIP_CMP_ONEPASS=0 timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 > $out/compact_twopass.jsonl 2> $out/compact_twopass.err || exit 1
cat $out/compact_twopass.jsonl
python3 - "$out" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/compact_kernel_stats.csv")))[:10]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
timeout -k 10 400 python -u tools/bench_configs.py --config 5 --fns p99,median --no-extra > $out/c5.jsonl 2> $out/c5.err || { tail $out/c5.err; exit 1; }
python3 -c "
import json
for l in open('$out/c5.jsonl'):
    d=json.loads(l); print(d.get('query'), round(d.get('ms_per_step',0),2), round(d.get('hbm_frac_of_8tbs',0),3))"
timeout -k 10 300 python3 tools/c3day_bench.py > $out/c3day.jsonl 2> $out/c3day.err || { tail $out/c3day.err; exit 1; }
cat $out/c3day.jsonl
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('extra',{}).get('config3',{}).get('sum',{}))"
