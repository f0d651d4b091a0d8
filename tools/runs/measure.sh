#!/bin/bash
# Measurement pass: bash tools/runs/measure.sh TAG [c3] [c3day] [md] [c4] [pmc_hwin]
#   c3        tools/bench_configs.py --config 3 --only sum,p99,median (10M series x 1 h)  -> c3.jsonl
#   c3day     tools/c3day_bench.py --multi (config 3's day on one GPU's share)  -> c3day.jsonl
#   md        bench.py --gpus 2 / 4 over repeated device 0 (the multi-device context rehearsal,
#             config 2 weak + config 3 strong at 1M series)                     -> md2.jsonl, md4.jsonl
#   c4        tools/bench_configs.py --config 4 (steps listed) and a TSDBHIP_TRACE=1 rerun -> c4*.jsonl
#   pmc_hwin  rocprofv3 PMC passes over the day's sum:1m-avg (k_hwin)           -> pmc_hwin/summary.txt
#   ro        tools/rollup_read_bench.py --check (default and TSDBHIP_RO_PACK=0), traced rerun -> ro*.jsonl
#   ro_prof   rocprofv3 --kernel-trace --stats over tools/rollup_read_bench.py    -> ro_prof/
#   ro_api    rocprofv3 --hip-trace --stats over tools/rollup_read_bench.py (host API time) -> ro_api/
#   c3_prof   rocprofv3 --kernel-trace --stats over config 3 p99:1m-avg            -> c3_prof/
#   c4_prof   rocprofv3 --kernel-trace --stats over config 4 (sum, p99)           -> c4_prof/
#   pmc_c4    PMC passes (LDS pass included) over config 4 (k_raw_top, k_raw_eval)     -> pmc_c4_summary.txt
#   pmc_c3p99 PMC passes (LDS pass included) over config 3's sum / p99:1m-avg   -> pmc_c3p99_summary.txt
# Every GPU step under its own timeout; the first failure ends the pass.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    c3)
      timeout -k 10 400 python3 -u tools/bench_configs.py --config 3 --only sum,p99,median --steps 10 \
        > $out/c3.jsonl 2> $out/c3.err || { tail -20 $out/c3.err; exit 1; }
      python3 -c "
import json
for l in open('$out/c3.jsonl'):
    d=json.loads(l); print(d['query'], 'ms', round(d['ms_per_step'],3), 'kernel', round(d.get('kernel_ms',0),3))" ;;
    c3day)
      timeout -k 10 400 python3 -u tools/c3day_bench.py --multi > $out/c3day.jsonl 2> $out/c3day.err \
        || { tail -20 $out/c3day.err; exit 1; }
      cat $out/c3day.jsonl ;;
    md)
      for n in 2 4; do
        devs=$(python3 -c "print(','.join(['0']*$n))")
        TSDBHIP_BENCH_DEVICES=$devs timeout -k 10 600 python3 -u bench.py --gpus $n --steps 5 --warmup 2 \
          --c3-series 1000000 --no-cpu-baseline --no-pmc > $out/md$n.jsonl 2> $out/md$n.err \
          || { tail -20 $out/md$n.err; exit 1; }
        python3 -c "
import json
d=json.loads(open('$out/md$n.jsonl').read().strip().splitlines()[-1])
print($n, 'value', d['value'], 'ms', d['ms_per_step'], 'stages', d.get('stages'))
for k,v in d['extra']['config3_strong'].items():
    if isinstance(v, dict): print('  ', k, json.dumps(v))"
      done ;;
    c4)
      timeout -k 10 400 python3 -u tools/bench_configs.py --config 4 --steps 10 > $out/c4.jsonl 2> $out/c4.err \
        || { tail -20 $out/c4.err; exit 1; }
      TSDBHIP_TRACE=1 timeout -k 10 400 python3 -u tools/bench_configs.py --config 4 --steps 6 > $out/c4_trace.jsonl \
        2> $out/c4_trace.txt || { tail -20 $out/c4_trace.txt; exit 1; }
      python3 -c "
import json
for l in open('$out/c4.jsonl'):
    d=json.loads(l); print(d['query'], 'mean', round(d['ms_per_step'],1), 'median', round(d['step_ms_median'],1), 'eval', round(d['k_raw_eval_ms'],1), 'steps', d['steps_ms'], 'dev', d['device_steps_ms'])" ;;
    ro)
      timeout -k 10 300 python3 -u tools/rollup_read_bench.py --check > $out/ro.jsonl 2> $out/ro.err \
        || { tail -20 $out/ro.err; exit 1; }
      TSDBHIP_RO_PACK=0 timeout -k 10 300 python3 -u tools/rollup_read_bench.py > $out/ro_nopack.jsonl 2> $out/ro_nopack.err \
        || { tail -20 $out/ro_nopack.err; exit 1; }
      TSDBHIP_TRACE=1 timeout -k 10 300 python3 -u tools/rollup_read_bench.py --steps 3 > $out/ro_trace.jsonl \
        2> $out/ro_trace.txt || { tail -20 $out/ro_trace.txt; exit 1; }
      python3 -c "
import json
for f in ('ro', 'ro_nopack'):
    for l in open('$out/' + f + '.jsonl'):
        d=json.loads(l); print(f, d['query'], 'ms', round(d['ms_per_step'],3), 'dev', round(d.get('device_decode_downsample_ms',0),3), d.get('check',''))" ;;
    ro_prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/ro_prof -o run -- python3 tools/rollup_read_bench.py \
        --steps 5 > $out/ro_prof.log 2>&1 || { tail -20 $out/ro_prof.log; exit 1; }
      python3 tools/prof_top.py $out/ro_prof 12 ;;
    ro_api)
      timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d $out/ro_api -o run -- python3 tools/rollup_read_bench.py \
        --steps 20 > $out/ro_api.log 2>&1 || { tail -20 $out/ro_api.log; exit 1; }
      head -25 $out/ro_api/run_hip_api_stats.csv ;;
    c3_prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c3_prof -o run -- python3 tools/bench_configs.py \
        --config 3 --only p99 --steps 5 > $out/c3_prof.log 2>&1 || { tail -20 $out/c3_prof.log; exit 1; }
      python3 tools/prof_top.py $out/c3_prof 12 ;;
    c4_prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c4_prof -o run -- python3 tools/bench_configs.py \
        --config 4 --steps 3 > $out/c4_prof.log 2>&1 || { tail -20 $out/c4_prof.log; exit 1; }
      python3 tools/prof_top.py $out/c4_prof 12 ;;
    pmc_c4)
      PMC_LDS=1 bash tools/pmc_run.sh ${tag}_c4 python3 tools/bench_configs.py --config 4 --steps 1 || exit $?
      python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_c4 k_raw | tee $out/pmc_c4_summary.txt ;;
    pmc_c3p99)
      PMC_LDS=1 bash tools/pmc_run.sh ${tag}_c3p99 python3 tools/bench_configs.py --config 3 --only sum,p99 --steps 1 \
        || exit $?
      python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_c3p99 | tee $out/pmc_c3p99_summary.txt ;;
    pmc_hwin)
      bash tools/pmc_run.sh ${tag}_hwin python3 tools/c3day_bench.py --only 1m --steps 1 || exit $?
      python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_hwin k_hwin | tee $out/pmc_hwin_summary.txt ;;
  esac
done
