#!/bin/bash
# percentile downsampling: parity (values-only key kernel) and config 5 p99 / median A/B
set -o pipefail
tag=${1:-r04f}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pct.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -30; exit $rc; }
for m in 11 10 00; do
  TSDBHIP_PCT_VONLY=${m:0:1} TSDBHIP_PCT_V6=${m:1:1} timeout -k 10 400 python -u tools/bench_configs.py --config 5 --fns p99,median,p50 --no-extra > $out/c5_v$m.jsonl 2> $out/c5_v$m.err || { tail $out/c5_v$m.err; exit 1; }
  python3 -c "
import json
for l in open('$out/c5_v$m.jsonl'):
    d=json.loads(l); print('vonly,v6=$m', d.get('query'), round(d.get('ms_per_step',0),2), round(d.get('hbm_frac_of_8tbs',0),3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c5 -o run -- \
  python3 tools/bench_configs.py --config 5 --fns p99,median --no-extra --steps 3 > $out/c5_prof.jsonl 2> $out/c5_prof.err || { tail $out/c5_prof.err; exit 1; }
find $out/prof_c5 -name '*kernel_stats.csv' -exec cp {} $out/c5_kernel_stats.csv \;
cut -d, -f1-4 $out/c5_kernel_stats.csv | head -12
