#!/bin/bash
# rollup read bench: default build, then the packed-pairs A/B (RO_RUNS=0), then the kernel trace
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/rollup_read_bench.py --opt RO_RUNS=0 > $out/rollup_pairs.jsonl 2> $out/rp.err || { tail $out/rp.err; exit 1; }
bash tools/ro_bench_prof.sh $1 && python3 -c "
import json
for l in open('$out/rollup_pairs.jsonl'): d=json.loads(l); print('pairs', d['query'], round(d['ms_per_step'],3))
"
