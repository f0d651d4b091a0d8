#!/bin/bash
# k_hwin tests + the day-shard bench, A/B against opentsdb_amd/lib/libtsdbhip_base.so when present
set -o pipefail
out=gpurun_out/$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_fullsize.py -k "hwin or day_shard or multi" -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -2 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $out/pytest.log | head; exit $rc; }
timeout -k 10 300 python -u tools/c3day_bench.py --only 1m,1h --multi > $out/c3day.jsonl 2> $out/c3day.err || { tail $out/c3day.err; exit 1; }
if [ -f opentsdb_amd/lib/libtsdbhip_base.so ]; then
  TSDBHIP_LIB=opentsdb_amd/lib/libtsdbhip_base.so timeout -k 10 300 python -u tools/c3day_bench.py --only 1m,1h --multi > $out/c3day_base.jsonl 2> $out/c3day_base.err || { tail $out/c3day_base.err; exit 1; }
  timeout -k 10 300 python -u tools/c3day_bench.py --only 1m --multi > $out/c3day_2.jsonl 2> $out/c3day_2.err || { tail $out/c3day_2.err; exit 1; }
fi
python3 -c "
import json, glob
for f in sorted(glob.glob('$out/c3day*.jsonl')):
    for l in open(f): d=json.loads(l); print(f.split('/')[-1], d['query'], round(d['ms_per_step'],3), round(d.get('decode_downsample_ms',0),3), d.get('redo_tiles'))
"
