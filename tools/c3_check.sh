#!/bin/bash
# config-3 default / ordered / percentile lines; outputs under gpurun_out/<tag>/
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python -u tools/bench_configs.py --config 3 --ordered --only sum,dev > $out/c3o.jsonl || exit 1
timeout -k 10 300 python -u tools/bench_configs.py --config 3 --only sum,p99,median > $out/c3.jsonl || exit 1
cat $out/c3o.jsonl $out/c3.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['query'], round(d['ms_per_step'], 2), round(d['kernel_ms'], 2))"
