#!/bin/bash
# r03: trainer phase trace on the shipped geometry (float2 x 64 lanes, d=128,
# C3 HOBE records; diagnostic build tools/_ab/dbg.so), the push form at
# 64-B rows, the combiner learnability test.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_trace}
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_mlp.py -x -v --timeout 150 --timeout-method thread > $O/mlp_tests.log 2>&1 || { echo MLPFAIL; tail -30 $O/mlp_tests.log; exit 11; }
echo mlp-ok
HGX_LIB_PATH=tools/_ab/dbg.so timeout -k 10 300 python -u tools/trace_train.py 128 hobe > $O/trace_d128_hobe.log 2>&1 || { echo TRACEFAIL; tail -20 $O/trace_d128_hobe.log; exit 12; }
head -12 $O/trace_d128_hobe.log
HGX_LIB_PATH=tools/_ab/dbg.so timeout -k 10 300 python -u tools/trace_train.py 256 > $O/trace_d256_rand.log 2>&1 || { echo TRACEFAIL2; tail -20 $O/trace_d256_rand.log; exit 13; }
head -6 $O/trace_d256_rand.log
timeout -k 10 300 python -u tools/perf_alg_push.py c4 20 2 16 > $O/ab_c4_ks16.jsonl 2>&1 || { echo ABFAIL; tail -20 $O/ab_c4_ks16.jsonl; exit 14; }
tail -1 $O/ab_c4_ks16.jsonl
