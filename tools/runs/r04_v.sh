#!/bin/bash
# mid-rank search: phase-1 candidate bound 64 / 32 / 16 (TSDBHIP_PCT_CAND), config 5 median / p50 / p99
set -o pipefail
out=gpurun_out/r04v; mkdir -p $out
export TMPDIR=/tmp
for cnd in 16; do
  TSDBHIP_PCT_CAND=$cnd timeout -k 10 600 python -u -m pytest tests/test_gpu_pct.py -x -q --timeout 300 --timeout-method thread > $out/pytest_$cnd.log 2>&1
  rc=$?; tail -2 $out/pytest_$cnd.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_$cnd.log | head -30; exit $rc; }
done
for cnd in 64 32 16 64; do
  TSDBHIP_PCT_CAND=$cnd timeout -k 10 400 python -u tools/bench_configs.py --config 5 --fns median,p50 --no-extra > $out/c5_$cnd.jsonl 2> $out/c5_$cnd.err || { tail $out/c5_$cnd.err; exit 1; }
  python3 -c "
import json
for l in open('$out/c5_$cnd.jsonl'):
    d=json.loads(l); print('cand=$cnd', d.get('query'), round(d.get('ms_per_step',0),2), round(d.get('hbm_frac_of_8tbs',0),3))"
done
