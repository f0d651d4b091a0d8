#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, a kernel-trace profile.
# usage: tools/gpu_check.sh <tag>    (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== bench"
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err
rc=$?; cat $out/bench.json; [ $rc -eq 0 ] || { tail -20 $out/bench.err; exit $rc; }
echo "== rocprofv3 kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > $out/prof_bench.json 2> $out/prof.err
rc=$?; [ $rc -eq 0 ] || { tail -20 $out/prof.err; exit $rc; }
find $out/prof -name '*kernel_stats.csv' -exec head -6 {} \;
echo done
