#!/bin/bash
# Profile bench.py on the GPU box: kernel trace + stats, then separate PMC passes
# (counters never combined with runtime/sys traces).
# usage: tools/prof.sh <tag> [bench args...]
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $*"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $out/$name -o run -- $B > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|134|137|139) echo "fatal rc in $name, stopping"; exit $rc;; esac
  return 0
}
run trace --kernel-trace --stats
run pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace
run pmc2 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace
run pmc3 --pmc FETCH_SIZE --kernel-trace
run pmc4 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace
echo done
