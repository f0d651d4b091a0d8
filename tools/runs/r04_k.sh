#!/bin/bash
# after k_emit_reg / grouped prefix / key-kernel fixes: parity of the touched paths, config 5, rollup
set -o pipefail
tag=${1:-r04k}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pct.py tests/test_gpu_fast.py tests/test_gpu_rollup_read.py tests/test_gpu_rollup.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_compaction.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
for m in 11 00; do
  TSDBHIP_PCT_VONLY=${m:0:1} TSDBHIP_PCT_V6=${m:1:1} timeout -k 10 400 python -u tools/bench_configs.py --config 5 --fns p99,median,p50 --no-extra > $out/c5_v$m.jsonl 2> $out/c5_v$m.err || { tail $out/c5_v$m.err; exit 1; }
  python3 -c "
import json
for l in open('$out/c5_v$m.jsonl'):
    d=json.loads(l); print('vonly,v6=$m', d.get('query'), round(d.get('ms_per_step',0),2), round(d.get('hbm_frac_of_8tbs',0),3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_ro -o run -- \
  python3 tools/rollup_read_bench.py --check > $out/rollup.jsonl 2> $out/rollup.err || { tail $out/rollup.err; exit 1; }
python3 -c "
import json
for l in open('$out/rollup.jsonl'):
    d=json.loads(l); print(d['query'], round(d['ms_per_step'],3), d.get('check'))"
find $out/prof_ro -name '*kernel_stats.csv' -exec cp {} $out/rollup_kernel_stats.csv \;
python3 - "$out" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/rollup_kernel_stats.csv")))[:8]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cmp -o run -- \
  python3 tools/compact_bench.py 20000 3600 3 > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
cat $out/compact.jsonl
find $out/prof_cmp -name '*kernel_stats.csv' -exec cp {} $out/compact_kernel_stats.csv \;
timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 --scan-order > $out/compact_scan.jsonl 2> $out/compact_scan.err || exit 1
cat $out/compact_scan.jsonl
python3 - "$out" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/compact_kernel_stats.csv")))[:8]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
