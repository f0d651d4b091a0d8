set -o pipefail
out=gpurun_out/r03zz; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_raw.py tests/test_gpu_pct_raw.py tests/test_gpu_raw_unsorted.py tests/test_gpu_fullsize.py -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; grep -E "^FAILED" $out/tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/bench_configs.py --config 4 > $out/c4.jsonl 2> $out/c4.err; rc=$?; cut -c1-330 $out/c4.jsonl; [ $rc -eq 0 ] || { tail -5 $out/c4.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c4prof -o run -- python3 tools/raw_prof.py 100000 2 sum,p99 > $out/c4prof.jsonl 2> $out/c4prof.err; rc=$?; cat $out/c4prof.jsonl; [ $rc -eq 0 ] || { tail -3 $out/c4prof.err; exit $rc; }
head -10 $out/c4prof/run_kernel_stats.csv | cut -d, -f1-4
