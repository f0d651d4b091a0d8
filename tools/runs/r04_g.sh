#!/bin/bash
# config 2 headline kernel: PMC passes (one counter group per run, kernel trace only)
set -o pipefail
tag=${1:-r04g}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD" \
            "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $out/p$i -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --no-config3 > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $out/p$i.log; [ $i -eq 3 ] && continue; exit $rc; }
done
python3 tools/pmc_summary.py $out k_fast 2>&1 | head -40 || true
