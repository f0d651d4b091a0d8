#!/bin/bash
# round 4, GPU pass B: RCCL next to torch, the tests touched so far, the bench line, config 3/4
# lines and the compaction bench.
set -o pipefail
tag=${1:-r04b}; out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "
from opentsdb_amd import engine as E
print('lib count', E.device_count())
e = E.Engine(devices=[0], transport=E.MD_RCCL); print('rccl ok before torch'); e.close()
import torch; print('torch count', torch.cuda.device_count())
try:
    e = E.Engine(devices=[0], transport=E.MD_RCCL); print('rccl ok after torch count'); e.close()
except Exception as ex: print('rccl FAILS after torch count:', ex)
" > $out/rccl.txt 2>&1; cat $out/rccl.txt | tail -4
timeout -k 10 1100 python -u -m pytest tests/test_gpu_multidev.py tests/test_gpu_rollup_read.py tests/test_gpu_compaction.py \
  tests/test_gpu_pct_raw.py tests/test_gpu_fast.py tests/test_gpu_pct_group.py tests/test_gpu_ordered.py tests/test_gpu_multi.py \
  -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $out/bench.json 2> $out/bench.err
rc=$?; cut -c1-600 $out/bench.json; [ $rc -eq 0 ] || { tail -20 $out/bench.err; exit $rc; }
bash tools/c3_check.sh $tag || exit 1
timeout -k 10 400 python -u tools/bench_configs.py --config 4 > $out/c4.jsonl 2> $out/c4.err || { tail $out/c4.err; exit 1; }
cut -c1-400 $out/c4.jsonl
timeout -k 10 300 python -u tools/compact_bench.py > $out/compact.jsonl 2> $out/compact.err || { tail $out/compact.err; exit 1; }
cat $out/compact.jsonl
timeout -k 10 120 python -u bench.py --gpus 2 > $out/bench2.json 2> $out/bench2.err
echo "gpus2 rc=$? $(tail -2 $out/bench2.err)"
