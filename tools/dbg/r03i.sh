set -o pipefail
out=gpurun_out/r03i; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?; tail -3 $out/pytest_gpu.log; grep -E "^FAILED" $out/pytest_gpu.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/rollup_read_bench.py > $out/rollup_read.jsonl 2> $out/rr.err; rc=$?; cut -c1-420 $out/rollup_read.jsonl; [ $rc -eq 0 ] || { tail -5 $out/rr.err; exit $rc; }
timeout -k 10 300 python -u tools/bench_configs.py --config 2 --only sum > $out/c2.jsonl 2> $out/c2.err; cut -c1-300 $out/c2.jsonl
