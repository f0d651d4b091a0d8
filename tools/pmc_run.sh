#!/bin/bash
# PMC passes (one counter group per run, never combined with traces) over a command.
# usage: tools/pmc_run.sh <tag> <command...>     outputs under gpurun_out/pmc_<tag>/
tag=$1; shift
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
            ${PMC_LDS:+"SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $out/p$i -o run -- "$@" > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done
