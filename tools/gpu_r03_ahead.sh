#!/bin/bash
# r03: trimmed train_place zero fill (libhgx.so vs tools/_ab/noplace.so) and
# chunk preparation one chunk ahead on the batch stream (tuning
# train_prep_overlap = 2): trainer tests, interleaved A/B.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_ahead}
mkdir -p $O
L=hypergraphembedding_amd/libhgx.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_streaming.py -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 11; }
tail -1 $O/tests.log
AB_N=6000000 timeout -k 10 300 python -u tools/ab_train.py 128 hobe tools/_ab/noplace.so $L $L:train_prep_overlap=2 > $O/ab_128.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_128.log; exit 12; }
cat $O/ab_128.log
AB_N=3000000 timeout -k 10 300 python -u tools/ab_train.py 256 rand tools/_ab/noplace.so $L $L:train_prep_overlap=2 > $O/ab_256.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_256.log; exit 13; }
cat $O/ab_256.log
