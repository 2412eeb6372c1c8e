#!/bin/bash
# Interleaved A/B of trainer builds under tools/_ab (one process per
# workload, tools/ab_train.py). Usage: tools/ab_r02b.sh OUTTAG lib1.so lib2.so ...
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${1}
shift
mkdir -p $O
for w in "128 hobe" "128 rand" "256 rand"; do
  timeout -k 10 300 python -u tools/ab_train.py $w "$@" >> $O/ab.log 2>&1 || exit 3
done
echo ok
