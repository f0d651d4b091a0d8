set -o pipefail
out=gpurun_out/r03fc; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?; tail -2 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $out/bench.jsonl 2> $out/bench.err; rc=$?; cut -c1-200 $out/bench.jsonl; exit $rc
