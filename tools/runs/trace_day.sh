#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of config 3's day shard: sum:1m-avg alone, then the
# fused run_multi.   bash tools/runs/trace_day.sh TAG
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_sum -o run -- \
  python3 tools/c3day_bench.py --only 1m --steps 3 > $out/sum.jsonl 2> $out/sum.err || { tail $out/sum.err; exit 1; }
find $out/prof_sum -name '*kernel_stats.csv' -exec cp {} $out/sum_kernel_stats.csv \;
find $out/prof_sum -name '*kernel_trace.csv' -exec cp {} $out/sum_kernel_trace.csv \;
rm -rf $out/prof_sum
head -12 $out/sum_kernel_stats.csv | cut -c1-200
