#!/bin/bash
set -o pipefail
out=gpurun_out/r04z2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_pct.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
timeout -k 10 400 python -u tools/bench_configs.py --config 5 --fns p99,median,p50 --no-extra > $out/c5.jsonl 2> $out/c5.err || { tail $out/c5.err; exit 1; }
python3 -c "
import json
for l in open('$out/c5.jsonl'):
    d=json.loads(l); print(d.get('query'), round(d.get('ms_per_step',0),2), round(d.get('hbm_frac_of_8tbs',0),3))"
