#!/bin/bash
# k_short with 6 datapoints a lane for the vle class: parity suites, config 3 (10M x 360) A/B
set -o pipefail
out=gpurun_out/r04aa; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_pct.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
for m in 0 1 0 1; do
  TSDBHIP_SHORT6=$m timeout -k 10 300 python -u tools/bench_configs.py --config 3 --series 10000000 --groups 1000 --only sum,avg,p99 --steps 10 > $out/c3_$m.jsonl 2> $out/c3_$m.err || { tail $out/c3_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$out/c3_$m.jsonl'):
    d=json.loads(l); print('short6=$m', d.get('query'), round(d.get('ms_per_step',0),3), d.get('kernel_ms'))"
done
