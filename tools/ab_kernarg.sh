#!/bin/bash
# Interleaved A/B of the HIP runtime's kernel-argument placement
# (HIP_FORCE_DEV_KERNARG=0 / 1) on the trainer step, d=128 and d=256,
# 4M random records (tools/perf_train.py). Diagnostic only.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${1:-kernarg}
mkdir -p $O
for r in 1 2 3; do
  for v in 0 1; do
    for d in 128 256; do
      echo "== round $r HIP_FORCE_DEV_KERNARG=$v d=$d" >> $O/ab.log
      HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 python -u tools/perf_train.py $d >> $O/ab.log 2>&1 || exit 3
    done
  done
done
echo ok
