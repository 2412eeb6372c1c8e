#!/bin/bash
# r05 counter passes (each its own rocprofv3 run, one counter per pass,
# under timeout -s KILL): the C4 d = 256 trainer step (FETCH_SIZE,
# WRITE_SIZE, kernel trace for the plain vs MULTI step form) and the C5
# combiner MLP launches (FETCH_SIZE, WRITE_SIZE per kernel).
# Usage: tools/pmc_r05.sh OUTDIR [d256|mlp|all]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_r05}
PART=${2:-all}
mkdir -p $O
if [ $PART != mlp ]; then
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 420 rocprofv3 --pmc $C -d $O/d256_$C -o run --output-format csv -- \
    python3 tools/train_d256_pmc_prog.py > $O/d256_$C.log 2>&1 || { echo "d256 pmc $C failed rc=$?"; exit 16; }
  echo "d256 $C ok"
done
F=$(find $O/d256_FETCH_SIZE -name '*counter_collection.csv' | head -1)
W=$(find $O/d256_WRITE_SIZE -name '*counter_collection.csv' | head -1)
python tools/pmc_train_summary.py "$F" "$W" $O/pmc_train_d256.json 256 5 "tools/train_d256_pmc_prog.py" > /dev/null || exit 19
rm -rf $O/d256_FETCH_SIZE $O/d256_WRITE_SIZE
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/d256_trace -o run --output-format csv -- \
  python3 tools/train_d256_pmc_prog.py > $O/d256_trace.log 2>&1 || { echo "d256 trace failed"; exit 17; }
find $O/d256_trace -name '*kernel_stats.csv' -exec cp {} $O/d256_kernel_stats.csv \;
rm -rf $O/d256_trace
echo "d256 trace ok"
fi
if [ $PART != d256 ]; then
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $O/mlp_$C -o run --output-format csv -- \
    python3 tools/perf_c5_mlp.py --samples 256000 --rows 1000000 --epochs 1 > $O/mlp_$C.log 2>&1 || { echo "mlp pmc $C failed rc=$?"; exit 18; }
  F=$(find $O/mlp_$C -name '*counter_collection.csv' | head -1)
  python tools/pmc_kernel_summary.py "$F" $C $O/pmc_mlp_$C.json > /dev/null || exit 20
  rm -rf $O/mlp_$C
  echo "mlp $C ok"
done
fi
