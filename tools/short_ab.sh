#!/bin/bash
# config 3 k_short A/B of two builds through bench.py's extra block: tools/short_ab.sh <tag> <lib_b>
set -o pipefail
out=gpurun_out/$1; B=$2; mkdir -p $out; export TMPDIR=/tmp
for run in a1 b1 a2 b2; do
  case $run in a*) L=opentsdb_amd/lib/libtsdbhip.so;; b*) L=$B;; esac
  TSDBHIP_LIB=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-pmc --no-cpu-baseline > $out/$run.json 2> $out/$run.err || { tail $out/$run.err; exit 1; }
done
python3 -c "
import json
for r in ('a1','b1','a2','b2'):
    d=json.load(open('$out/'+r+'.json')); e=d['extra']['config3']
    print(r, 'c2', round(d['ms_per_step'],3), 'c3 sum', round(e['sum']['ms_per_step'],3), 'kernel', round(e['sum']['kernel_ms'],3), 'multi', round(e['multi_avg_min_max_count_dev']['ms_per_step'],3), 'p99', round(e['p99']['ms_per_step'],3), 'parity', d['parity_ok'], e['parity']['ok'])
"
