#!/bin/bash
# C4 alg-dist: PMC passes of the kernels the bench runs (separate runs), then
# the hot/cold non-temporal gather experiment (debug build tools/_ab/dbg.so).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/alg_r02
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "TCC_EA0_[A-Z0-9_]*" $O/counters.txt | sort -u > $O/tcc_ea.txt || true
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc$i -o run --output-format csv -- \
    python3 tools/perf_alg.py c4 10 2 > $O/pmc$i.log 2>&1 || { echo "pmc pass $i ($C) failed rc=$?"; }
  echo "pass $i done"
done
python tools/pmc_alg_summary.py $O/pmc_alg_c4.json $(find $O -name '*counter_collection.csv') > /dev/null || echo summary-failed
rm -rf $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4
for H in 2147483647 0 40000 80000 170000 400000; do
  echo "== HOT=$H" >> $O/hot.log
  HGX_LIB_PATH=tools/_ab/dbg.so HGX_ALG_HOT=$H timeout -k 10 120 python tools/perf_alg.py c4 10 20 >> $O/hot.log 2>&1 || exit 20
done
echo "== HOT_E=0" >> $O/hot.log
HGX_LIB_PATH=tools/_ab/dbg.so HGX_ALG_HOT_E=0 timeout -k 10 120 python tools/perf_alg.py c4 10 20 >> $O/hot.log 2>&1 || exit 21
echo all-ok
