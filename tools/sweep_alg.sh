#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
rm -f $O/sweep_alg.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_algdist_probs.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py tests/test_gpu_embedding.py -x -q --timeout 120 --timeout-method thread > $O/t_alg.log 2>&1 || exit 11
for v in "HGX_ALG_QUAD=1" "HGX_ALG_QUAD=0" "HGX_ALG_SAMPLE_FLUSH=0" "HGX_ALG_QLPI=4" "HGX_ALG_QLPI=16"; do
  echo "== $v" >> $O/sweep_alg.txt
  env $v timeout -k 10 60 python tools/perf_alg.py c3 10 20 >> $O/sweep_alg.txt 2>&1 || exit 12
done
for v in "HGX_ALG_QUAD=1" "HGX_ALG_QUAD=0"; do
  echo "== c4 $v" >> $O/sweep_alg.txt
  env $v timeout -k 10 120 python tools/perf_alg.py c4 10 5 >> $O/sweep_alg.txt 2>&1 || exit 13
done
echo ok
