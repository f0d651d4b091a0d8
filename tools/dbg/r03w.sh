set -o pipefail
out=gpurun_out/r03w; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollup_read.py tests/test_gpu_rollup.py tests/test_gpu_rollup_shard.py -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; grep -E "^FAILED" $out/tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/rollup_read_bench.py --check > $out/rollup_read.jsonl 2> $out/rr.err; rc=$?; cut -c1-200 $out/rollup_read.jsonl; python3 -c "
import json
for l in open('$out/rollup_read.jsonl'):
    d=json.loads(l); print(d['query'], round(d['ms_per_step'],3), round(d['device_decode_downsample_ms'],3), d.get('check'))"; [ $rc -eq 0 ] || { tail -5 $out/rr.err; exit $rc; }
