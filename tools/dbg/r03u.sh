set -o pipefail
out=gpurun_out/r03u; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rrprof -o run -- python3 tools/rollup_read_bench.py --steps 5 > $out/rr.jsonl 2> $out/rr.err; rc=$?; cut -c1-200 $out/rr.jsonl; [ $rc -eq 0 ] || { tail -3 $out/rr.err; exit $rc; }
head -14 $out/rrprof/run_kernel_stats.csv | cut -d, -f1-4
