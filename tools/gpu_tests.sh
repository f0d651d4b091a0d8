#!/bin/bash
# One GPU-box pass over chosen test files, then (optionally) the bench and a kernel trace.
# usage: tools/gpu_tests.sh <tag> <bench:0|1> <pytest args...>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=$1; bench=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 1000 python -u -m pytest "$@" -x -v --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
  rc=$?; grep -E "passed|failed|error" $out/pytest.log | tail -3
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $out/pytest.log | head -20; exit $rc; }
fi
[ "$bench" = "1" ] || exit 0
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-pmc --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?; cat $out/bench.json; [ $rc -eq 0 ] || { tail -20 $out/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > $out/prof_bench.json 2> $out/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -20 $out/prof.err; exit $rc; }
find $out/prof -name '*kernel_stats.csv' -exec head -8 {} \;
