#!/bin/bash
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
TSDBHIP_TRACE=1 timeout -k 10 300 python3 -u tools/compact_bench.py 20000 3600 3 --pinned > $out/compact_pinned.jsonl 2> $out/compact_pinned.trace \
  || { tail $out/compact_pinned.trace; exit 1; }
TSDBHIP_TRACE=1 timeout -k 10 300 python3 -u tools/compact_bench.py 20000 3600 3 > $out/compact.jsonl 2> $out/compact.trace \
  || { tail $out/compact.trace; exit 1; }
grep "load_cells" $out/compact.trace | tail -9; grep "load_cells" $out/compact_pinned.trace | tail -9
bash tools/runs/check.sh $tag tests/test_gpu_fast.py tests/test_gpu_fullsize.py tests/test_gpu_multidev.py
