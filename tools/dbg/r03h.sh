set -o pipefail
out=gpurun_out/r03h; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hist.py -q --timeout 200 --timeout-method thread > $out/hist_tests.log 2>&1; rc=$?; tail -2 $out/hist_tests.log; grep -E "^FAILED" $out/hist_tests.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
for v in 0 1; do
  TSDBHIP_HIST_LAYOUT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/hl$v -o run -- python3 tools/hist_bench.py --steps 3 > $out/hl$v.json 2> $out/hl$v.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $out/hl$v.err; exit $rc; }
  echo "layout=$v"; cut -c1-200 $out/hl$v.json
  find $out/hl$v -name '*kernel_stats.csv' -exec head -5 {} \; | cut -c1-200
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rr -o run -- python3 tools/rollup_read_bench.py --series 200000 --steps 2 > $out/rr.jsonl 2> $out/rr.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $out/rr.err; exit $rc; }
cut -c1-300 $out/rr.jsonl; find $out/rr -name '*kernel_stats.csv' -exec head -12 {} \; | cut -c1-200
timeout -k 10 200 python3 -X faulthandler tools/compact_bench.py 2000 3600 2 --pinned > $out/cp.json 2> $out/cp.err; rc=$?; echo "pinned rc=$rc"; cat $out/cp.json; tail -30 $out/cp.err
