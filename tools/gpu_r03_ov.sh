#!/bin/bash
# r03: CU-mask probe, overlapped chunk preparation (trainer tests + A/B of the
# whole epoch's rate), then the HEAD check (GPU suite, smoke, bench line).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_ov}
mkdir -p $O
timeout -k 10 120 tools/_ab/cumask_probe > $O/cumask_probe.log 2>&1; echo "probe rc=$?"; cat $O/cumask_probe.log
cat $O/cumask_probe.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread > $O/train_tests.log 2>&1 || { echo TRAINTESTFAIL; tail -30 $O/train_tests.log; exit 11; }
tail -1 $O/train_tests.log
L=hypergraphembedding_amd/libhgx.so
AB_N=6000000 timeout -k 10 400 python -u tools/ab_train.py 128 hobe $L $L:train_prep_overlap=1 $L:train_prep_overlap=1,train_prep_cus=16 $L:train_prep_overlap=1,train_prep_cus=32 $L:train_prep_overlap=1,train_prep_cus=64 > $O/ab_ov.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_ov.log; exit 12; }
cat $O/ab_ov.log
bash tools/gpu_r03_head.sh ${1:-r03_ov}_head || exit 13
tail -1 gpurun_out/${1:-r03_ov}_head/bench.json | cut -c1-400
