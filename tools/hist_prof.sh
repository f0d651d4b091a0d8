#!/bin/bash
# Histogram-path profile on the GPU box: kernel trace + one PMC pass over tools/hist_bench.py.
set -o pipefail
out=gpurun_out/${1:-histprof}; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/hist_bench.py --steps 3 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $out/pmc1 -o run -- python3 tools/hist_bench.py --steps 1 --warmup 0 > $out/pmc1.log 2>&1 || { tail -5 $out/pmc1.log; exit 1; }
find $out/trace -name '*kernel_stats.csv' -exec head -6 {} \;
python3 tools/pmc_summary.py $out/pmc1 k_hist | tee $out/pmc1_summary.txt
