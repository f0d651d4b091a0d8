#!/bin/bash
# Rollup-read / config-5 A/B over environment variants: bash tools/runs/ro_ab.sh TAG "NAME:ENV=VAL,..." ...
#   the rollup-read GPU tests once, then per variant tools/rollup_read_bench.py -> <NAME>.jsonl
#   (C5=1: also tools/bench_configs.py --config 5 -> <NAME>_c5.jsonl)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollup_read.py tests/test_gpu_pct.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  ( [ "$envs" != "$v" ] && for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 python3 -u tools/rollup_read_bench.py > $out/$name.jsonl 2> $out/$name.err &&
    if [ "${C5:-0}" = 1 ]; then timeout -k 10 400 python3 -u tools/bench_configs.py --config 5 --steps 5 > $out/${name}_c5.jsonl 2>> $out/$name.err; fi
  ) || { tail -20 $out/$name.err; exit 1; }
  python3 -c "
import json, os
for f in ('$out/$name.jsonl', '$out/${name}_c5.jsonl'):
    if not os.path.exists(f): continue
    for l in open(f):
        d=json.loads(l); print('$name', d['query'], 'ms', round(d['ms_per_step'],3), 'dev', round(d.get('device_decode_downsample_ms', d.get('kernel_ms', 0)),3))"
done
