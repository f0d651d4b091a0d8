#!/bin/bash
# k_sel_reg block-shape A/B: bash tools/runs/sel_ab.sh TAG "T:OCC" ...
#   per variant: the percentile group-by GPU tests, then config 3 p99 / median:1m-avg  -> sel_<T>_<OCC>.jsonl
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  T=${v%%:*}; O=${v##*:}
  export TSDBHIP_SEL_T=$T TSDBHIP_SEL_OCC=$O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pct_group.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > $out/pytest_${T}_${O}.log 2>&1 || { tail -20 $out/pytest_${T}_${O}.log; exit 1; }
  tail -1 $out/pytest_${T}_${O}.log
  timeout -k 10 300 python3 -u tools/bench_configs.py --config 3 --only p99,median --steps 10 \
    > $out/sel_${T}_${O}.jsonl 2> $out/sel_${T}_${O}.err || { tail -20 $out/sel_${T}_${O}.err; exit 1; }
  python3 -c "
import json
for l in open('$out/sel_${T}_${O}.jsonl'):
    d=json.loads(l); print('$v', d['query'], 'ms', round(d['ms_per_step'],3), 'kernel', round(d.get('kernel_ms',0),3))"
done
