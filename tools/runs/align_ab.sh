#!/bin/bash
# Row-alignment A/B (TSDBHIP_ROW_ALIGN 16 vs 128) on config 3's day shard (k_hwin / k_rows) and its
# 1 h point (k_short), plus the run_multi trace.   bash tools/runs/align_ab.sh TAG
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for a in 16 128; do
  TSDBHIP_ROW_ALIGN=$a timeout -k 10 300 python3 -u tools/c3day_bench.py --multi > $out/day_a$a.jsonl 2> $out/day_a$a.err \
    || { tail $out/day_a$a.err; exit 1; }
  TSDBHIP_ROW_ALIGN=$a timeout -k 10 300 python3 -u tools/c3day_bench.py --series 10000000 --hours 1 --only 1m \
    > $out/h1_a$a.jsonl 2> $out/h1_a$a.err || { tail $out/h1_a$a.err; exit 1; }
  echo "align $a"; cat $out/day_a$a.jsonl $out/h1_a$a.jsonl
done
TSDBHIP_TRACE=1 timeout -k 10 300 python3 -u tools/c3day_bench.py --multi --only 1m --steps 2 > $out/trace.jsonl 2> $out/trace.txt \
  || { tail $out/trace.txt; exit 1; }
grep -A8 "run_multi_fused" $out/trace.txt | tail -12
