#!/bin/bash
# r03: block radix sort in train_prep (libhgx.so) and early row-0 atomics
# (tools/_ab/r0e.so): trainer tests on both, prep phase trace, A/B.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_rsort}
mkdir -p $O
T="tests/test_gpu_train.py tests/test_gpu_streaming.py"
timeout -k 10 500 python -u -m pytest $T -x -v --timeout 200 --timeout-method thread > $O/tests_rsort.log 2>&1 || { echo TESTFAIL rsort; tail -30 $O/tests_rsort.log; exit 11; }
tail -1 $O/tests_rsort.log
HGX_LIB_PATH=tools/_ab/r0e.so timeout -k 10 500 python -u -m pytest $T -x -v --timeout 200 --timeout-method thread > $O/tests_r0e.log 2>&1 || { echo TESTFAIL r0e; tail -30 $O/tests_r0e.log; }
tail -1 $O/tests_r0e.log
HGX_LIB_PATH=tools/_ab/trace.so timeout -k 10 300 python -u tools/trace_train.py 128 hobe > $O/trace_prep.log 2>&1 || { echo TRACEFAIL; tail -20 $O/trace_prep.log; exit 13; }
head -8 $O/trace_prep.log
L=hypergraphembedding_amd/libhgx.so
AB_N=6000000 timeout -k 10 400 python -u tools/ab_train.py 128 hobe tools/_ab/prev.so $L tools/_ab/r0e.so > $O/ab_128.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_128.log; exit 14; }
cat $O/ab_128.log
AB_N=3000000 timeout -k 10 400 python -u tools/ab_train.py 256 rand tools/_ab/prev.so $L tools/_ab/r0e.so > $O/ab_256.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_256.log; exit 15; }
cat $O/ab_256.log
