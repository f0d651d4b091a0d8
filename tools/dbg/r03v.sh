set -o pipefail
out=gpurun_out/r03v; mkdir -p $out; export TMPDIR=/tmp
for s in 1 0; do
TSDBHIP_SEQ=$s timeout -k 10 300 python3 tools/rollup_read_bench.py --steps 5 > $out/rr$s.jsonl 2> $out/rr$s.err; rc=$?; echo "seq=$s"; python3 -c "
import json
for l in open('$out/rr$s.jsonl'):
    d=json.loads(l); print(d['query'], round(d['ms_per_step'],3), round(d['device_decode_downsample_ms'],3), round(d['group_reduce_ms'],3))"; [ $rc -eq 0 ] || { tail -3 $out/rr$s.err; exit $rc; }
done
TSDBHIP_TRACE=1 timeout -k 10 300 python3 tools/rollup_read_bench.py --steps 1 > $out/rrt.jsonl 2> $out/rrt.err; rc=$?; tail -30 $out/rrt.err | cut -c1-200
