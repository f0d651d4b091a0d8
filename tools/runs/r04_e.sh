#!/bin/bash
# compaction parity + bench (kernel trace), then the rollup read bench with phase marks and a kernel trace
set -o pipefail
tag=${1:-r04e}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_compaction.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cmp -o run -- \
  python3 tools/compact_bench.py 20000 3600 3 > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
cat $out/compact.jsonl
find $out/prof_cmp -name '*kernel_stats.csv' -exec cp {} $out/compact_kernel_stats.csv \;
cut -d, -f1-4 $out/compact_kernel_stats.csv | head -14
timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 --pinned > $out/compact_pinned.jsonl 2> $out/compact_pinned.err || exit 1
cat $out/compact_pinned.jsonl
timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 --scan-order > $out/compact_scan.jsonl 2> $out/compact_scan.err || exit 1
cat $out/compact_scan.jsonl
TSDBHIP_TRACE=1 timeout -k 10 300 python3 tools/rollup_read_bench.py --steps 3 > $out/rollup_trace.jsonl 2> $out/rollup_trace.err || { tail $out/rollup_trace.err; exit 1; }
tail -40 $out/rollup_trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_ro -o run -- \
  python3 tools/rollup_read_bench.py > $out/rollup.jsonl 2> $out/rollup.err || { tail $out/rollup.err; exit 1; }
cat $out/rollup.jsonl
find $out/prof_ro -name '*kernel_stats.csv' -exec cp {} $out/rollup_kernel_stats.csv \;
cut -d, -f1-4 $out/rollup_kernel_stats.csv | head -14
# config 2 headline: tile-size A/B (old threshold 8192 tiles vs the tail-aware default)
for v in 8192 32768; do
  TSDBHIP_TILE_MIN=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pmc --no-config3 > $out/bench_tile$v.json 2> $out/bench_tile$v.err || { tail $out/bench_tile$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/bench_tile$v.json')); print('tile_min', $v, d['value'], d['ms_per_step'], d['roofline'])"
done
