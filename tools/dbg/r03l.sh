set -o pipefail
out=gpurun_out/r03l; mkdir -p $out; export TMPDIR=/tmp
for cfg in "52 16" "52 4" "80 16" "80 4" "160 16"; do
  set -- $cfg
  TSDBHIP_HIST_WLDS=$1 TSDBHIP_HIST_SU=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/h_$1_$2 -o run -- python3 tools/hist_bench.py --steps 3 > $out/h_$1_$2.json 2> $out/h_$1_$2.err; rc=$?; [ $rc -eq 0 ] || { tail -3 $out/h_$1_$2.err; exit $rc; }
  echo "wlds=$1 su=$2 $(python3 -c "import json;print(round(json.load(open('$out/h_$1_$2.json'))['ms_per_query'],3))") ms; accw: $(grep k_hist_accw $out/h_$1_$2/run_kernel_stats.csv | cut -d, -f4)"
done
