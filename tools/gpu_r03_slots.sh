#!/bin/bash
# r03: row-0 slot count (HGX_R0_SLOTS 4 / 8 / 16) with the early row-0 sums:
# trainer tests on the variants, interleaved A/B.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_slots}
mkdir -p $O
for v in s4 s16; do
  HGX_LIB_PATH=tools/_ab/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1; echo "tests $v rc=$?"; tail -1 $O/tests_$v.log
done
L=hypergraphembedding_amd/libhgx.so
AB_N=6000000 timeout -k 10 300 python -u tools/ab_train.py 128 hobe $L tools/_ab/s4.so tools/_ab/s16.so > $O/ab_128.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_128.log; exit 12; }
cat $O/ab_128.log
AB_N=3000000 timeout -k 10 300 python -u tools/ab_train.py 256 rand $L tools/_ab/s4.so tools/_ab/s16.so > $O/ab_256.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_256.log; exit 13; }
cat $O/ab_256.log
