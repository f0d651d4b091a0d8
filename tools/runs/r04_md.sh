#!/bin/bash
# rehearsal of bench.py's multi-device path on one GPU (repeated devices, peer copies)
set -o pipefail
out=gpurun_out/r04md; mkdir -p $out
export TMPDIR=/tmp
TSDBHIP_BENCH_DEVICES=0,0 timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --c3-series 1000000 > $out/md2.jsonl 2> $out/md2.err || { tail -20 $out/md2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$out/md2.jsonl').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','n_gpus','devices','transport','rccl_ranks','exchange_ms','ms_per_step')})
print(json.dumps(d['extra'])[:1500])"
TSDBHIP_BENCH_DEVICES=0,0,0,0 timeout -k 10 400 python3 bench.py --gpus 4 --steps 5 --warmup 2 --no-config3 > $out/md4.jsonl 2> $out/md4.err || { tail -20 $out/md4.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$out/md4.jsonl').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','n_gpus','devices','transport','rccl_ranks','exchange_ms','ms_per_step')})"
