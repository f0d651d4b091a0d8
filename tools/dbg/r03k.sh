set -o pipefail
out=gpurun_out/r03k; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_hist.py tests/test_gpu_rollup_read.py tests/test_gpu_rollup.py tests/test_gpu_rollup_shard.py -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -2 $out/tests.log; grep -E "^FAILED" $out/tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/rollup_read_bench.py --check > $out/rollup_read.jsonl 2> $out/rr.err; rc=$?; cut -c1-330 $out/rollup_read.jsonl; [ $rc -eq 0 ] || { tail -5 $out/rr.err; exit $rc; }
timeout -k 10 300 python -u bench.py --value-kind 4 --no-pmc --no-cpu-baseline --no-config3 --steps 5 > $out/bench_f64.json 2> $out/bench_f64.err; rc=$?; cut -c1-700 $out/bench_f64.json; [ $rc -eq 0 ] || { tail -5 $out/bench_f64.err; exit $rc; }
TSDBHIP_SEQ=0 timeout -k 10 300 python -u bench.py --value-kind 4 --no-pmc --no-cpu-baseline --no-config3 --steps 2 --warmup 1 > $out/bench_f64_grid.json 2> $out/bench_f64_grid.err; cut -c1-300 $out/bench_f64_grid.json
TSDBHIP_TRACE=1 timeout -k 10 300 python3 tools/compact_bench.py 20000 3600 2 --pinned > $out/cp.json 2> $out/cp.err; cat $out/cp.json; grep "trace load_cells" $out/cp.err | tail -7
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/hp -o run -- python3 tools/hist_bench.py --steps 3 > $out/hp.json 2> $out/hp.err; rc=$?; cut -c1-250 $out/hp.json; [ $rc -eq 0 ] || { tail -5 $out/hp.err; exit $rc; }
find $out/hp -name '*kernel_stats.csv' -exec head -6 {} \; | cut -c1-200
