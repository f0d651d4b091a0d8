#!/bin/bash
# compaction: parity tests and the bench under a kernel trace
set -o pipefail
tag=${1:-r04d}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_compaction.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_cmp -o run -- \
  python3 tools/compact_bench.py 20000 3600 3 > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
cat $out/compact.jsonl
find $out/prof_cmp -name '*kernel_stats.csv' -exec cp {} $out/compact_kernel_stats.csv \;
cut -d, -f1-4 $out/compact_kernel_stats.csv | head -12
timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 --pinned > $out/compact_pinned.jsonl 2> $out/compact_pinned.err
cat $out/compact_pinned.jsonl
timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 3 --scan-order > $out/compact_scan.jsonl 2> $out/compact_scan.err
cat $out/compact_scan.jsonl
