#!/bin/bash
# Copy + kernel trace of tools/compact_bench.py (72M one-datapoint cells).  bash tools/runs/compact_prof.sh TAG
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 tools/compact_bench.py 20000 3600 2 ${MODE:-} > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
for f in $(find $out/prof -name '*stats.csv'); do cp $f $out/$(basename $f); done
find $out/prof -name '*memory_copy_trace.csv' -exec cp {} $out/memory_copy_trace.csv \;
rm -rf $out/prof
cat $out/compact.jsonl | cut -c1-300
ls $out; head -20 $out/*memory_copy_stats.csv
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$out/memory_copy_trace.csv")))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
t0=int(rows[0]["Start_Timestamp"])
for r in rows[:200:5]:
    s,e=int(r["Start_Timestamp"]),int(r["End_Timestamp"])
    print(r["Direction"], r.get("Size", r.get("Bytes","?")), round((s-t0)/1e6,3), round((e-s)/1e6,3))
PY
