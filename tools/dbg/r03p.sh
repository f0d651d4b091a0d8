set -o pipefail
out=gpurun_out/r03p; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_pct_group.py tests/test_gpu_fast.py tests/test_gpu_hist.py tests/test_gpu_fullsize.py -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; grep -E "^FAILED" $out/tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
for c in 1 0; do
  TSDBHIP_SEL_COLS=$c timeout -k 10 300 python -u tools/bench_configs.py --config 3 --only sum,p99,median > $out/c3_cols$c.jsonl 2> $out/c3_cols$c.err; rc=$?; echo "cols=$c"; cut -c1-300 $out/c3_cols$c.jsonl; [ $rc -eq 0 ] || { tail -5 $out/c3_cols$c.err; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3prof -o run -- python3 tools/bench_configs.py --config 3 --only p99 > $out/c3prof.jsonl 2> $out/c3prof.err; rc=$?; [ $rc -eq 0 ] || { tail -3 $out/c3prof.err; exit $rc; }
head -8 $out/c3prof/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 200 python -u tools/hist_bench.py > $out/hist.json 2> $out/hist.err; rc=$?; cut -c1-300 $out/hist.json; [ $rc -eq 0 ] || { tail -3 $out/hist.err; exit $rc; }
