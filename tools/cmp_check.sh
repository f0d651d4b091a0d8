#!/bin/bash
# compaction tests + compact_bench A/B + kernel trace: tools/cmp_check.sh <tag>
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_compaction.py tests/test_gpu_md_rollup.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $out/pytest.log | head -20; exit $rc; }
for a in "" "--scan-order" "--opt=CMP_SEC=0" "--scan-order --opt=CMP_SEC=0"; do
  timeout -k 10 200 python -u tools/compact_bench.py 20000 3600 3 --pinned $a >> $out/compact.jsonl 2>> $out/cb.err || { tail $out/cb.err; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/compact_bench.py 20000 3600 3 --pinned > $out/prof.jsonl 2> $out/prof.err || { tail $out/prof.err; exit 1; }
python3 -c "
import json, csv
for l in open('$out/compact.jsonl'): d=json.loads(l); print(d['workload'][:60], round(d['compact_ms'],3), round(d['algorithmic_GBps'],1))
for r in csv.DictReader(open('$out/prof/run_kernel_stats.csv')):
    if 'k_cmp' in r['Name']: print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
