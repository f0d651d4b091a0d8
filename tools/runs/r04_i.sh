#!/bin/bash
# config 5 k_pct_rows instruction mix: PMC passes (one counter group per run, kernel trace only)
set -o pipefail
tag=${1:-r04i}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for fn in p99 median; do
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $out/$fn/p$i -o run -- \
    python3 tools/bench_configs.py --config 5 --fns $fn --no-extra --steps 2 > $out/$fn.p$i.log 2>&1
  rc=$?
  echo "$fn pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $out/$fn.p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $out/$fn k_pct_rows 2>&1 | tee $out/$fn.summary.txt | head -30
done
