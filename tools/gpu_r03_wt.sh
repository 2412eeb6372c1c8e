#!/bin/bash
# r03: write-through (sc1) row stores in the trainer step vs plain stores,
# interleaved A/B in one process (tools/ab_train.py).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_wt}
mkdir -p $O
timeout -k 10 300 python -u tools/ab_train.py 128 hobe tools/_ab/step3.so tools/_ab/wt1.so > $O/ab_d128_hobe.log 2>&1 || { echo AB1FAIL; tail $O/ab_d128_hobe.log; exit 12; }
cat $O/ab_d128_hobe.log
bash tools/gpu_r03_mlpwt.sh ${1:-r03_wt}_mlp || exit 14
timeout -k 10 300 python -u tools/ab_train.py 256 rand tools/_ab/step3.so tools/_ab/wt1.so tools/_ab/wt3.so > $O/ab_d256_rand.log 2>&1 || { echo AB2FAIL; tail $O/ab_d256_rand.log; exit 13; }
cat $O/ab_d256_rand.log
