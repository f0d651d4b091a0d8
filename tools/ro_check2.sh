set -o pipefail
out=gpurun_out/r06aw; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollup_read.py tests/test_gpu_md_rollup.py tests/test_gpu_fast.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -2 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $out/pytest.log | head; exit $rc; }
bash tools/ro_bench_prof.sh r06aw
