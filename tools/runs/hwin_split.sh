#!/bin/bash
# k_hwin work-item split sweep (TSDBHIP_HWIN_SPLIT) on config 3's day shard.  bash tools/runs/hwin_split.sh TAG
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for sp in ${SPLITS:-4 6 8 12 24}; do
  TSDBHIP_HWIN_SPLIT=$sp timeout -k 10 300 python3 -u tools/c3day_bench.py --only 1m --multi --steps 5 > $out/split$sp.jsonl 2> $out/split$sp.err \
    || { tail $out/split$sp.err; exit 1; }
  echo "split $sp"; cat $out/split$sp.jsonl
done
