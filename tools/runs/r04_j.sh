#!/bin/bash
# percentile key kernels after the lane_below / phase-2 rewrite: parity + config 5
set -o pipefail
tag=${1:-r04j}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pct.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
for m in 11 00; do
  TSDBHIP_PCT_VONLY=${m:0:1} TSDBHIP_PCT_V6=${m:1:1} timeout -k 10 400 python -u tools/bench_configs.py --config 5 --fns p99,median,p50 --no-extra > $out/c5_v$m.jsonl 2> $out/c5_v$m.err || { tail $out/c5_v$m.err; exit 1; }
  python3 -c "
import json
for l in open('$out/c5_v$m.jsonl'):
    d=json.loads(l); print('vonly,v6=$m', d.get('query'), round(d.get('ms_per_step',0),2), round(d.get('hbm_frac_of_8tbs',0),3))"
done
