set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 500 python -u -m pytest tests/test_gpu_hist.py tests/test_gpu_rollup_shard.py tests/test_gpu_compaction.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03d/tests.log 2>&1; rc=$?; tail -4 gpurun_out/r03d/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/hist_bench.py > gpurun_out/r03d/hist_bench.json 2> gpurun_out/r03d/hist_bench.err; rc=$?; cat gpurun_out/r03d/hist_bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03d/hist_bench.err; exit $rc; }
timeout -k 10 300 python -u tools/hist_bench.py --ds none > gpurun_out/r03d/hist_bench_raw.json 2>> gpurun_out/r03d/hist_bench.err; cat gpurun_out/r03d/hist_bench_raw.json
