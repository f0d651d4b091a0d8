set -o pipefail
out=gpurun_out/r03e; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?; tail -3 $out/pytest_gpu.log; grep -E "^FAILED" $out/pytest_gpu.log | head
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; cat $out/smoke.log; [ $rc -eq 0 ] || exit $rc



