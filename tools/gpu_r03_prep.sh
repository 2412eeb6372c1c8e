#!/bin/bash
# r03: train_prep phase trace (diagnostic build) and the prep change A/B.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_prep}
mkdir -p $O
HGX_LIB_PATH=tools/_ab/trace.so timeout -k 10 300 python -u tools/trace_train.py 128 hobe > $O/trace_prep.log 2>&1 || { echo TRACEFAIL; tail -20 $O/trace_prep.log; exit 11; }
head -8 $O/trace_prep.log
L=hypergraphembedding_amd/libhgx.so
AB_N=6000000 timeout -k 10 400 python -u tools/ab_train.py 128 hobe tools/_ab/prev.so $L > $O/ab_prep.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_prep.log; exit 12; }
cat $O/ab_prep.log
