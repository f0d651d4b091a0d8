#!/bin/bash
# bench.py's launch forms rehearsed on a one-GPU box, each with its parity blocks:
#   n1    : the default line (N=1, config 3 block)
#   rccl1 : torch.distributed.run, one rank, the RCCL (nccl) process group forced on
#   gloo2 : torch.distributed.run, two ranks sharing GPU 0 over gloo (the exchange code of N>1)
#   md2   : the one-process multi-device context over GPU 0 repeated twice (peer copies)
#   md4   : the same over GPU 0 repeated four times
# usage: tools/bench_rehearse.sh <tag> [steps...]   (outputs under gpurun_out/<tag>/)
set -o pipefail
tag=$1; shift
steps=${*:-n1 rccl1 gloo2 md2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
TR="python -u -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
C="--steps 5 --warmup 2 --no-pmc --no-cpu-baseline --c3-series 2000000 --c5-series 1000000"
for s in $steps; do
  echo "== $s"
  case $s in
    n1)    timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-pmc --no-cpu-baseline > $out/$s.jsonl 2> $out/$s.err ;;
    rccl1) TSDBHIP_BENCH_FORCE_DIST=1 timeout -k 10 400 $TR --nproc-per-node 1 --master-port 29511 bench.py $C > $out/$s.jsonl 2> $out/$s.err ;;
    gloo2) TSDBHIP_BENCH_DIST=gloo TSDBHIP_BENCH_DEVICES=0,0 timeout -k 10 500 $TR --nproc-per-node 2 --master-port 29512 \
             bench.py --gpus 2 --series 500000 $C > $out/$s.jsonl 2> $out/$s.err ;;
    md2)   TSDBHIP_BENCH_DEVICES=0,0 timeout -k 10 500 python -u bench.py --gpus 2 --transport copy $C > $out/$s.jsonl 2> $out/$s.err ;;
    md4)   TSDBHIP_BENCH_DEVICES=0,0,0,0 timeout -k 10 500 python -u bench.py --gpus 4 --transport copy $C > $out/$s.jsonl 2> $out/$s.err ;;
  esac
  rc=$?
  python3 - $out/$s.jsonl <<'PY' || true
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l); p = d.get("parity") or {}
    print(" value %.3e ms %.3f parity_ok %s checked %s max_rel %.2g" % (d["value"], d["ms_per_step"], d.get("parity_ok"), p.get("checked"), p.get("max_rel_err", -1)))
    if p.get("straddle"): print(" straddle ok", p["straddle"]["ok"], p["straddle"].get("max_rel_err"))
    for k, v in (d.get("extra") or {}).items():
        pp = v.get("parity") or {}
        print(" ", k, "parity", pp.get("ok"), pp.get("checked"), {q: round(x.get("ms_per_step", -1), 3) for q, x in v.items() if isinstance(x, dict) and "ms_per_step" in x})
PY
  [ $rc -eq 0 ] || { echo "$s exited $rc"; tail -25 $out/$s.err; exit $rc; }
done
echo done
