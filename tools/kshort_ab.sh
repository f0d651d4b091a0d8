#!/bin/bash
# A/B of k_short builds on config 3 (rocprof kernel stats per build).  usage: tools/kshort_ab.sh <tag> <lib>...
tag=$1; shift
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  TSDBHIP_LIB=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_$n -o run -- python3 -u tools/bench_configs.py --config 3 --only sum,avg --steps 10 > gpurun_out/${tag}_$n.jsonl || exit 1
  echo "== $n"
  python3 - gpurun_out/${tag}_$n/run_kernel_stats.csv <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if 'k_short' in x['Name'] or 'k_index' in x['Name']:
        print(f"  {x['Name'][:44]:44s} avg {float(x['AverageNs'])/1e3:8.1f} us  sd {float(x['StdDev'])/1e3:6.1f}  n {x['Calls']}")
PY
done
