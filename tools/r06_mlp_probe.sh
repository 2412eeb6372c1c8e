# combiner MLP launch-grouping probe: throughput and per-launch trace for
# each value of the mlp_wgrad_split knob given as arguments
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mlp_probe
mkdir -p $O
for v in "$@"; do
  timeout -k 10 240 python3 -u tools/perf_c5_mlp.py --samples 8000000 --epochs 2 --tune mlp_wgrad_split=$v > $O/perf_$v.json 2>&1 || { echo PERFFAIL $v; exit 11; }
  tail -1 $O/perf_$v.json
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o tr -- python3 tools/perf_c5_mlp.py --samples 1000000 --epochs 1 --tune mlp_wgrad_split=$v > $O/tr_$v.log 2>&1 || { echo TRFAIL $v; exit 12; }
  f=$(find $O/tr_$v -name '*kernel_trace.csv')
  python3 tools/mlp_trace_summary.py $f > $O/trace_$v.txt && cat $O/trace_$v.txt
  rm -rf $O/tr_$v
done
