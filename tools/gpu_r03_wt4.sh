#!/bin/bash
# r03: 16-byte write-through row stores at d = 256 (asm, A/B build) vs plain.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_wt4}
mkdir -p $O
timeout -k 10 300 python -u tools/ab_train.py 256 rand tools/_ab/cur.so tools/_ab/wt4.so > $O/ab_d256_rand.log 2>&1 || { echo AB2FAIL; tail $O/ab_d256_rand.log; exit 13; }
cat $O/ab_d256_rand.log
