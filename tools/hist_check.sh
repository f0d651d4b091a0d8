#!/bin/bash
# histogram tests + bench + kernel trace: tools/hist_check.sh <tag>
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_hist.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $out/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/hist_bench.py --series 2000 --check > $out/check.json 2> $out/check.err || { tail -5 $out/check.err; exit 1; }
timeout -k 10 300 python -u tools/hist_bench.py > $out/b1m.json 2> $out/b1m.err || { tail -5 $out/b1m.err; exit 1; }
timeout -k 10 300 python -u tools/hist_bench.py --ds none > $out/braw.json 2> $out/braw.err || { tail -5 $out/braw.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/hist_bench.py --steps 3 > $out/prof.json 2> $out/prof.err || { tail -5 $out/prof.err; exit 1; }
python3 -c "
import json, csv
for f in ('check','b1m','braw'):
    d=json.loads(open('$out/'+f+'.json').read().strip().splitlines()[-1]); print(f, {k: d[k] for k in list(d)[:8]})
for r in csv.DictReader(open('$out/prof/run_kernel_stats.csv')):
    if 'k_hist' in r['Name']: print(r['Name'][:48], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
if [ -f opentsdb_amd/lib/libtsdbhip_base.so ]; then   # A/B: the same bench on a baseline build
  TSDBHIP_LIB=opentsdb_amd/lib/libtsdbhip_base.so timeout -k 10 300 python -u tools/hist_bench.py > $out/b1m_base.json 2> $out/b1m_base.err || { tail -5 $out/b1m_base.err; exit 1; }
  TSDBHIP_LIB=opentsdb_amd/lib/libtsdbhip_base.so timeout -k 10 300 python -u tools/hist_bench.py --ds none > $out/braw_base.json 2> $out/braw_base.err || { tail -5 $out/braw_base.err; exit 1; }
  timeout -k 10 300 python -u tools/hist_bench.py > $out/b1m_2.json 2> $out/b1m_2.err || { tail -5 $out/b1m_2.err; exit 1; }
  python3 -c "
import json
for f in ('b1m','b1m_base','b1m_2','braw','braw_base'):
    d=json.loads(open('$out/'+f+'.json').read().strip().splitlines()[-1]); print(f, round(d['ms_per_query'],3))
"
fi
