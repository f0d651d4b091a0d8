#!/bin/bash
# round 4, GPU pass C: kernel traces of the compaction bench and config 4
set -o pipefail
tag=${1:-r04c}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cmp -o run -- \
  python3 tools/compact_bench.py 20000 3600 3 > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
cat $out/compact.jsonl
find $out/prof_cmp -name '*kernel_stats.csv' -exec cp {} $out/compact_kernel_stats.csv \;
cut -d, -f1-4 $out/compact_kernel_stats.csv | head -14
timeout -k 10 400 python -u tools/bench_configs.py --config 4 > $out/c4.jsonl 2> $out/c4.err || { tail $out/c4.err; exit 1; }
python3 -c "
import json
for l in open('$out/c4.jsonl'):
    d = json.loads(l); print(d['query'][:30], d.get('steps_ms'), d.get('device_steps_ms'), round(d['k_raw_eval_ms'],2))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c4 -o run -- \
  python3 tools/bench_configs.py --config 4 --steps 3 > $out/c4prof.jsonl 2> $out/c4prof.err || { tail $out/c4prof.err; exit 1; }
find $out/prof_c4 -name '*kernel_stats.csv' -exec cp {} $out/c4_kernel_stats.csv \;
cut -d, -f1-4 $out/c4_kernel_stats.csv | head -14
