#!/bin/bash
set -o pipefail
out=gpurun_out/r04y2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 300 --timeout-method thread -k "hwin or rows" > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python3 tools/c3day_bench.py > $out/c3day.jsonl 2> $out/c3day.err || { tail $out/c3day.err; exit 1; }
cat $out/c3day.jsonl
