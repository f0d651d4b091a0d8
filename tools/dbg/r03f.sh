set -o pipefail
out=gpurun_out/r03f; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hist.py -q --timeout 200 --timeout-method thread > $out/hist_tests.log 2>&1; rc=$?; tail -2 $out/hist_tests.log; grep -E "^FAILED" $out/hist_tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
for v in 0 1; do
  TSDBHIP_HIST_PIPE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/hp$v -o run -- python3 tools/hist_bench.py --steps 3 > $out/hp$v.json 2> $out/hp$v.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $out/hp$v.err; exit $rc; }
  echo "pipe=$v"; cut -c1-200 $out/hp$v.json
  find $out/hp$v -name '*kernel_stats.csv' -exec head -9 {} \;
done
TSDBHIP_HIST_WINDOW=0 timeout -k 10 200 python3 tools/hist_bench.py > $out/old_kernel.json 2>&1; cut -c1-200 $out/old_kernel.json
