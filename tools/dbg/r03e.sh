set -o pipefail
out=gpurun_out/r03e; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" $out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; cat $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/histprof -o run -- python3 tools/hist_bench.py --steps 3 > $out/histprof.json 2> $out/histprof.err; rc=$?; [ $rc -eq 0 ] || { tail -5 $out/histprof.err; exit $rc; }
find $out/histprof -name '*kernel_stats.csv' -exec head -12 {} \;
