#!/bin/bash
# Round-3 measurement pass on one MI355X: the bench line, configs 3/4/5, the f-row benches and a
# kernel trace of the bench.   usage: tools/runs/r03_measure.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=${1:-r03m}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $out/$name.jsonl 2> $out/$name.err
  local rc=$?
  echo "== $name rc=$rc"; cut -c1-400 $out/$name.jsonl
  case $rc in 0) ;; *) tail -5 $out/$name.err; exit $rc;; esac
}
step bench 400 python -u bench.py
step c3 300 python -u tools/bench_configs.py --config 3 --only sum,p99,median
step c3_ordered 300 python -u tools/bench_configs.py --config 3 --ordered --only sum
step c5 400 python -u tools/bench_configs.py --config 5 --fns p99,median,p50,ep99r7
step c4 300 python -u tools/bench_configs.py --config 4
step rollup_read 400 python -u tools/rollup_read_bench.py --check
step compact 300 python -u tools/compact_bench.py
step compact_pinned 300 python -u tools/compact_bench.py --pinned
step hist 300 python -u tools/hist_bench.py
step hist_raw 300 python -u tools/hist_bench.py --ds none
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-config3 > $out/prof_bench.json 2> $out/prof.err
rc=$?; echo "== prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/prof.err; exit $rc; }
find $out/prof -name '*kernel_stats.csv' -exec head -6 {} \;
echo done
