#!/bin/bash
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?; tail -2 $out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $out/pytest_gpu.log | head; exit $rc; }
bash tools/ro_bench_prof.sh $1
