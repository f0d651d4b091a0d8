#!/bin/bash
# 6 a lane for the vle class in k_rows / k_hwin: tests, config-3 day shard A/B
set -o pipefail
out=gpurun_out/r04ac; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
for m in 0 1; do
  TSDBHIP_SHORT6=$m timeout -k 10 300 python3 tools/c3day_bench.py > $out/c3day_$m.jsonl 2> $out/c3day_$m.err || { tail $out/c3day_$m.err; exit 1; }
  python3 -c "
import json
for l in open('$out/c3day_$m.jsonl'):
    d=json.loads(l); print('short6=$m', d['query'], round(d['ms_per_step'],2), round(d['fast_ms'],2))"
done
