#!/bin/bash
# k_hwin vs k_rows where both apply (TSDBHIP_HWIN=2 forces k_hwin): config 3's day shard at 10m / 1h
# and its 12 h half at 1m.   bash tools/runs/hwin_ab.sh TAG
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for h in 1 2; do
  TSDBHIP_HWIN=$h timeout -k 10 300 python3 -u tools/c3day_bench.py --only 1m,10m,1h > $out/day_h$h.jsonl 2> $out/day_h$h.err \
    || { tail $out/day_h$h.err; exit 1; }
  TSDBHIP_HWIN=$h timeout -k 10 300 python3 -u tools/c3day_bench.py --hours 12 --series 2500000 --only 1m,10m \
    > $out/half_h$h.jsonl 2> $out/half_h$h.err || { tail $out/half_h$h.err; exit 1; }
  echo "HWIN=$h"; cut -c1-200 $out/day_h$h.jsonl $out/half_h$h.jsonl
done
timeout -k 10 400 python3 -u tools/bench_configs.py --config 4 --steps 10 > $out/c4.jsonl 2> $out/c4.err || { tail -20 $out/c4.err; exit 1; }
python3 -c "
import json
for l in open('$out/c4.jsonl'):
    d=json.loads(l); print(d['query'], 'mean', round(d['ms_per_step'],1), 'median', round(d['step_ms_median'],1), 'eval', round(d['k_raw_eval_ms'],1), 'steps', d['steps_ms'])"
for mode in "" "--pinned"; do
  TSDBHIP_TRACE=1 timeout -k 10 300 python3 -u tools/compact_bench.py 20000 3600 3 $mode > $out/compact$mode.jsonl 2> $out/compact$mode.trace \
    || { tail $out/compact$mode.trace; exit 1; }
  cat $out/compact$mode.jsonl; tail -12 $out/compact$mode.trace
done
