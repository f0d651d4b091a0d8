#!/bin/bash
# closing pass (rounds 4-5): full GPU suite, smoke, the driver's bench command, kernel trace of the bench
set -o pipefail
tag=${1:-r04full}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$out/bench.jsonl').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
print('c3', json.dumps(d['extra']['config3']['sum'])); print('c3 p99', json.dumps(d['extra']['config3'].get('p99')))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > $out/prof_bench.jsonl 2> $out/prof.err || { tail -20 $out/prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/bench_kernel_stats.csv \;
head -6 $out/bench_kernel_stats.csv | cut -c1-160
