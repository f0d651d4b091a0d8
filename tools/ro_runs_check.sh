set -o pipefail
out=gpurun_out/r06ak; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollup_read.py tests/test_gpu_md_rollup.py tests/test_gpu_options.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/rollup_read_bench.py --check > $out/rollup_runs.jsonl 2> $out/rr.err || { tail $out/rr.err; exit 1; }
timeout -k 10 200 python -u tools/rollup_read_bench.py --opt RO_RUNS=0 > $out/rollup_pairs.jsonl 2> $out/rp.err || { tail $out/rp.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/rollup_read_bench.py > $out/prof.jsonl 2> $out/prof.err || { tail $out/prof.err; exit 1; }
python3 -c "
import json
for f in ('rollup_runs','rollup_pairs'):
    for l in open('$out/'+f+'.jsonl'): d=json.loads(l); print(f, d['query'], round(d['ms_per_step'],3), d.get('check',''))
"
grep -E "k_ro_|k_emit_reg" $out/prof/run_kernel_stats.csv | cut -d, -f1-4
