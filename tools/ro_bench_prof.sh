#!/bin/bash
# rollup read bench + its kernel trace: tools/ro_bench_prof.sh <tag> [rollup_read_bench args]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/rollup_read_bench.py --check "$@" > $out/rollup.jsonl 2> $out/rr.err || { tail $out/rr.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/rollup_read_bench.py "$@" > $out/prof.jsonl 2> $out/prof.err || { tail $out/prof.err; exit 1; }
python3 -c "
import json, csv
for l in open('$out/rollup.jsonl'): d=json.loads(l); print(d['query'], round(d['ms_per_step'],3), d.get('check',''))
for r in csv.DictReader(open('$out/prof/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('k_ro_', 'k_emit', 'k_reduce')): print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
