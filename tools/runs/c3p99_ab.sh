#!/bin/bash
# Config 3 p99 / median group-by A/B: bash tools/runs/c3p99_ab.sh TAG "NAME:ENV=VAL,ENV=VAL" ...
#   the percentile group-by GPU tests once, then per variant config 3 p99 / median:1m-avg -> <NAME>.jsonl
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pct_group.py tests/test_gpu_fast.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  ( [ "$envs" != "$v" ] && for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 python3 -u tools/bench_configs.py --config 3 --only sum,p99,median --steps 10 \
      > $out/$name.jsonl 2> $out/$name.err ) || { tail -20 $out/$name.err; exit 1; }
  python3 -c "
import json
for l in open('$out/$name.jsonl'):
    d=json.loads(l); print('$name', d['query'], 'ms', round(d['ms_per_step'],3), 'kernel', round(d.get('kernel_ms',0),3))"
done
