set -o pipefail
out=gpurun_out/r03x; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_rollup_read.py tests/test_gpu_rollup.py tests/test_gpu_rollup_shard.py -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; grep -E "^FAILED" $out/tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
for w in 1 0; do
TSDBHIP_SEQ_WAVE=$w timeout -k 10 300 python -u tools/rollup_read_bench.py --check > $out/rr$w.jsonl 2> $out/rr$w.err; rc=$?; echo "wave=$w"; python3 -c "
import json
for l in open('$out/rr$w.jsonl'):
    d=json.loads(l); print(d['query'], round(d['ms_per_step'],3), round(d['device_decode_downsample_ms'],3), d.get('check'))"; [ $rc -eq 0 ] || { tail -5 $out/rr$w.err; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rrprof -o run -- python3 tools/rollup_read_bench.py --steps 5 > $out/rrp.jsonl 2> $out/rrp.err; rc=$?; [ $rc -eq 0 ] || { tail -3 $out/rrp.err; exit $rc; }
head -5 $out/rrprof/run_kernel_stats.csv | cut -d, -f1-4
