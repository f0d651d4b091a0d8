#!/bin/bash
# round 4, GPU pass A: the tests touched this round, the bench line (with config 3), the
# config-3 percentile / ordered lines, and the --gpus 2 refusal on a one-GPU box.
set -o pipefail
out=gpurun_out/${1:-r04a}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_multidev.py tests/test_gpu_rollup_read.py tests/test_gpu_compaction.py \
  tests/test_gpu_fast.py tests/test_gpu_pct_group.py tests/test_gpu_ordered.py tests/test_gpu_multi.py \
  -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?; cat $out/bench.json; [ $rc -eq 0 ] || { tail -20 $out/bench.err; exit $rc; }
bash tools/c3_check.sh ${1:-r04a} || exit 1
timeout -k 10 120 python -u bench.py --gpus 2 > $out/bench2.json 2> $out/bench2.err
echo "gpus2 rc=$? $(tail -2 $out/bench2.err)"
