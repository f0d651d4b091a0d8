set -o pipefail
out=gpurun_out/histb1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/hist_bench.py --series 2000 --check > $out/check.json 2> $out/check.err || { tail -5 $out/check.err; exit 1; }
cat $out/check.json
timeout -k 10 300 python -u tools/hist_bench.py > $out/b1m.json 2> $out/b1m.err || { tail -5 $out/b1m.err; exit 1; }
cat $out/b1m.json
timeout -k 10 300 python -u tools/hist_bench.py --ds none > $out/braw.json 2> $out/braw.err || { tail -5 $out/braw.err; exit 1; }
cat $out/braw.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 tools/hist_bench.py --steps 3 > $out/prof.json 2> $out/prof.err || { tail -5 $out/prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec head -12 {} \;
