#!/bin/bash
# config-2 default / ordered / percentile lines and the bench line; outputs under gpurun_out/<tag>/
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python -u tools/bench_configs.py --config 2 --ordered --only sum,dev > $out/c2o.jsonl || exit 1
timeout -k 10 300 python -u tools/bench_configs.py --config 2 --only dev,sum,p99,median > $out/c2.jsonl || exit 1
timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline > $out/bench.json || exit 1
cat $out/c2o.jsonl $out/c2.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['query'], round(d['ms_per_step'], 2), round(d['kernel_ms'], 2))"
cut -c1-200 $out/bench.json
