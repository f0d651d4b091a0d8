#!/bin/bash
# k_sel_wave check: the percentile group-by / multi-device tests, then the md rehearsal with
# and without it (TSDBHIP_SEL_WAVE=0).  bash tools/runs/selwave_ab.sh TAG
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_pct_group.py tests/test_gpu_multidev.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for w in 1 0; do
  TSDBHIP_SEL_WAVE=$w TSDBHIP_BENCH_DEVICES=0,0 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 \
    --c3-series 1000000 --no-cpu-baseline --no-pmc > $out/md2_w$w.jsonl 2> $out/md2_w$w.err \
    || { tail -20 $out/md2_w$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$out/md2_w$w.jsonl').read().strip().splitlines()[-1])
v=d['extra']['config3_strong']['p99']
print('wave=$w p99 ms', round(v['ms_per_step'],2), 'select_ms', round(v['stages']['select_ms'],2))"
done
