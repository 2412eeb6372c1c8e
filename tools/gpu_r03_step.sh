#!/bin/bash
# r03: trainer step changes (16-B row-0 partial loads, batched head
# reductions): trainer + streaming + sharded tests, then interleaved A/B
# against the previous build, and the train_tb=512 tuning.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_step}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_streaming.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 11; }
echo tests-ok
timeout -k 10 300 python -u tools/ab_train.py 128 hobe tools/_ab/step3.so tools/_ab/step4.so > $O/ab_d128_hobe.log 2>&1 || { echo AB1FAIL; tail $O/ab_d128_hobe.log; exit 12; }
cat $O/ab_d128_hobe.log
timeout -k 10 300 python -u tools/ab_train.py 256 rand tools/_ab/step3.so tools/_ab/step4.so > $O/ab_d256_rand.log 2>&1 || { echo AB2FAIL; tail $O/ab_d256_rand.log; exit 13; }
cat $O/ab_d256_rand.log
