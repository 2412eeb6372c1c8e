# combiner MLP probe builds (results wrong by construction): the WGRAD
# launch's duration without its accumulator stores (st1) and without any of
# its tile stores (st2), against the product build, from kernel traces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mlp_stprobe
mkdir -p $O
for v in base st1 st2; do
  if [ $v = base ]; then L=""; else L=tools/_ab/mlp_$v.so; fi
  HGX_LIB_PATH=$L timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o tr -- python3 tools/perf_c5_mlp.py --samples 1000000 --epochs 1 > $O/tr_$v.log 2>&1 || { echo TRFAIL $v; exit 12; }
  f=$(find $O/tr_$v -name '*kernel_trace.csv')
  python3 tools/mlp_trace_summary.py $f > $O/trace_$v.txt && echo $v && cat $O/trace_$v.txt
  rm -rf $O/tr_$v
done
