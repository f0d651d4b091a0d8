#!/bin/bash
# Round-3 PMC passes (each counter group its own run, kernel trace only): config 4's raw union
# kernels, config 3's percentile group-by selection, the windowed histogram accumulation.
# usage: tools/runs/r03_pmc.sh <tag>   (outputs under gpurun_out/pmc_<tag>_*/, summaries printed)
set -o pipefail
tag=${1:-r03}
export TMPDIR=/tmp
bash tools/pmc_run.sh ${tag}_c4 python3 tools/raw_prof.py 100000 1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_c4 k_raw | tee gpurun_out/pmc_${tag}_c4/summary.txt
bash tools/pmc_run.sh ${tag}_c4p99 python3 tools/raw_prof.py 100000 1 p99 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_c4p99 k_raw | tee gpurun_out/pmc_${tag}_c4p99/summary.txt
bash tools/pmc_run.sh ${tag}_c3p99 python3 tools/bench_configs.py --config 3 --only p99 --steps 1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_c3p99 k_sel | tee gpurun_out/pmc_${tag}_c3p99/summary.txt
bash tools/pmc_run.sh ${tag}_hist python3 tools/hist_bench.py --steps 1 --warmup 0 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_hist k_hist | tee gpurun_out/pmc_${tag}_hist/summary.txt
