#!/bin/bash
# result assembly from page-locked staging, over host threads for large results
set -o pipefail
out=gpurun_out/r04ad; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
TSDBHIP_TRACE=1 timeout -k 10 300 python3 tools/c3day_trace.py > $out/trace.out 2> $out/trace.txt || { tail $out/trace.txt; exit 1; }
tail -8 $out/trace.txt
timeout -k 10 300 python3 tools/c3day_bench.py > $out/c3day.jsonl 2> $out/c3day.err || { tail $out/c3day.err; exit 1; }
cat $out/c3day.jsonl
