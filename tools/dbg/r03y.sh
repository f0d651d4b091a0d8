set -o pipefail
out=gpurun_out/r03y; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_rollup_read.py tests/test_gpu_rollup.py -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; grep -E "^FAILED" $out/tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
for w in 1 0; do
TSDBHIP_SEQ_WAVE=$w timeout -k 10 300 python -u tools/seq_bench.py > $out/seq$w.jsonl 2> $out/seq$w.err; rc=$?; cut -c1-260 $out/seq$w.jsonl; [ $rc -eq 0 ] || { tail -5 $out/seq$w.err; exit $rc; }
done
timeout -k 10 300 python -u tools/rollup_read_bench.py > $out/rr.jsonl 2> $out/rr.err; rc=$?; python3 -c "
import json
for l in open('$out/rr.jsonl'):
    d=json.loads(l); print(d['query'], round(d['ms_per_step'],3), round(d['device_decode_downsample_ms'],3))"; [ $rc -eq 0 ] || { tail -5 $out/rr.err; exit $rc; }
