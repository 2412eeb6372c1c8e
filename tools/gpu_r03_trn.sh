#!/bin/bash
# r03: trainer / streaming / configs / full-size / sharded GPU tests on the
# current tree (write-through row stores at both geometries).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_trn}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_streaming.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py tests/test_gpu_lp_combine.py tests/test_gpu_embedding.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 11; }
tail -2 $O/tests.log
