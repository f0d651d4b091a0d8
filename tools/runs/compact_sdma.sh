#!/bin/bash
# Compaction wall time: the runtime's copy engines vs blit kernels (HSA_ENABLE_SDMA=0), pageable / pinned.
set -o pipefail
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for sd in 1 0; do for mode in "" "--pinned"; do
  HSA_ENABLE_SDMA=$sd timeout -k 10 300 python3 -u tools/compact_bench.py 20000 3600 3 $mode > $out/c_sdma$sd$mode.jsonl 2> $out/c_sdma$sd$mode.err \
    || { tail $out/c_sdma$sd$mode.err; exit 1; }
  echo "SDMA=$sd $mode"; cut -c1-330 $out/c_sdma$sd$mode.jsonl
done; done
