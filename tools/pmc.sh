#!/bin/bash
# PMC passes over an arbitrary python command (each counter group in its own run, never
# combined with runtime/sys traces).   usage: tools/pmc.sh <tag> <python args...>
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $out/$name -o run -- python3 "${ARGS[@]}" > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|134|137|139) echo "fatal rc in $name, stopping"; exit $rc;; esac
  return 0
}
ARGS=("$@")
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
echo done
