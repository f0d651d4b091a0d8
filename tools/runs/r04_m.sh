#!/bin/bash
# rollup fused stage: parity + bench
set -o pipefail
tag=${1:-r04m}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_rollup_read.py tests/test_gpu_rollup.py tests/test_gpu_fast.py tests/test_gpu_multidev.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_ro -o run -- \
  python3 tools/rollup_read_bench.py --check > $out/rollup.jsonl 2> $out/rollup.err || { tail $out/rollup.err; exit 1; }
python3 -c "
import json
for l in open('$out/rollup.jsonl'):
    d=json.loads(l); print(d['query'], round(d['ms_per_step'],3), d.get('check'))"
find $out/prof_ro -name '*kernel_stats.csv' -exec cp {} $out/rollup_kernel_stats.csv \;
python3 - "$out" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + "/rollup_kernel_stats.csv")))[:9]:
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:10.1f}")
PY
TSDBHIP_RO_FUSE=0 timeout -k 10 300 python3 tools/rollup_read_bench.py > $out/rollup_nofuse.jsonl 2>/dev/null || exit 1
python3 -c "
import json
for l in open('$out/rollup_nofuse.jsonl'):
    d=json.loads(l); print('nofuse', d['query'], round(d['ms_per_step'],3))"
