#!/bin/bash
# final build: smoke, the driver's bench command, kernel trace of the bench
set -o pipefail
out=gpurun_out/r04final; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$out/bench.jsonl').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
print('c3', d['extra']['config3']['sum']['kernel_ms'], d['extra']['config3']['sum']['hbm_frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > $out/prof_bench.jsonl 2> $out/prof.err || { tail -20 $out/prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/bench_kernel_stats.csv \;
head -4 $out/bench_kernel_stats.csv | cut -c1-160
