#!/bin/bash
# Round-3 closing run on one MI355X: the whole GPU suite, smoke(), then the measurement pass
# (tools/runs/r03_measure.sh).   usage: tools/runs/r03_final.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-r03q}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
rc=$?; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/runs/r03_measure.sh $tag
