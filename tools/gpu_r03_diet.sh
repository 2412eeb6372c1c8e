#!/bin/bash
# r03: train_prep from the sort's registers (runs.so) and with 4 workgroups
# per CU (diet.so), early row-0 sums at float2 rows (r0e2.so): tests, prep
# phase trace, A/B against the radix-sort library (libhgx.so).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_diet}
mkdir -p $O
T="tests/test_gpu_train.py tests/test_gpu_streaming.py"
for v in diet r0e2; do
  HGX_LIB_PATH=tools/_ab/$v.so timeout -k 10 500 python -u -m pytest $T -v --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1; echo "tests $v rc=$?"; tail -1 $O/tests_$v.log
done
HGX_LIB_PATH=tools/_ab/trace.so timeout -k 10 300 python -u tools/trace_train.py 128 hobe > $O/trace_prep.log 2>&1 || { echo TRACEFAIL; tail -20 $O/trace_prep.log; exit 13; }
head -5 $O/trace_prep.log
L=hypergraphembedding_amd/libhgx.so
AB_N=6000000 timeout -k 10 500 python -u tools/ab_train.py 128 hobe $L tools/_ab/runs.so tools/_ab/diet.so tools/_ab/r0e2.so > $O/ab_128.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_128.log; exit 14; }
cat $O/ab_128.log
AB_N=3000000 timeout -k 10 400 python -u tools/ab_train.py 256 rand $L tools/_ab/diet.so tools/_ab/r0e2.so > $O/ab_256.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_256.log; exit 15; }
cat $O/ab_256.log
