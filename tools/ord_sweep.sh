#!/bin/bash
# k_ordered slot-run width sweep on config 3 (sum:1m-avg ordered); outputs under gpurun_out/<tag>/
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
for kw in ${KWS:-default 8 15 30 60}; do
  if [ "$kw" = default ]; then unset TSDBHIP_ORD_KW; else export TSDBHIP_ORD_KW=$kw; fi
  timeout -k 10 300 python -u tools/bench_configs.py --config 3 --ordered --only sum > $out/c3_kw_$kw.jsonl 2> $out/c3_kw_$kw.err || { tail -5 $out/c3_kw_$kw.err; exit 1; }
  echo "kw=$kw $(cat $out/c3_kw_$kw.jsonl)"
done
