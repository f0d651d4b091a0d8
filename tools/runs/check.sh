#!/bin/bash
# Generic GPU pass: bash tools/runs/check.sh TAG [pytest args ...]
#   runs `pytest -m gpu` over the given selection (default: the whole GPU suite) into
#   gpurun_out/TAG/pytest_gpu.log, then (BENCH=1) the driver's bench command into bench.jsonl.
# Every GPU step runs under its own `timeout -k 10`; a failure ends the pass.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 ${PYTEST_LIMIT:-1500} python -u -m pytest "${sel[@]}" -m gpu -x -q --timeout ${TEST_TIMEOUT:-150} --timeout-method thread \
  > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest_gpu.log | head -20; exit $rc; }
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err \
    || { tail -20 $out/bench.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$out/bench.jsonl').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
print('cpu', json.dumps(d['cpu_baseline']))
print('c3', json.dumps(d['extra']['config3']))"
fi
