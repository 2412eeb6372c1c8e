#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
rm -f $O/sweep_alg.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_embedding.py -x -q --timeout 120 --timeout-method thread > $O/t_train.log 2>&1 || exit 11
timeout -k 10 60 python tools/perf_train.py 128 >> $O/sweep_alg.txt 2>&1 || exit 12
timeout -k 10 60 python tools/perf_train.py 256 >> $O/sweep_alg.txt 2>&1 || exit 12
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit 14
echo ok
