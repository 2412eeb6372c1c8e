#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
rm -f $O/sweep_alg.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > $O/t_train.log 2>&1 || exit 11
for v in "HGX_TRAIN_PIPE=1" "HGX_TRAIN_PIPE=0" "HGX_TRAIN_PIPE=2"; do
  echo "== $v" >> $O/sweep_alg.txt
  env $v timeout -k 10 60 python tools/perf_train.py 128 >> $O/sweep_alg.txt 2>&1 || exit 12
done
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit 14
echo ok
