#!/bin/bash
# r03: which part of the two-stream overlapped preparation slows the step
# chain (tools/ovl_probe.hip), then the trainer A/B with per-XCD CU masks.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_ov2}
mkdir -p $O
timeout -k 10 180 tools/_ab/ovl_probe > $O/ovl_probe.log 2>&1; echo "probe rc=$?"; cat $O/ovl_probe.log
L=hypergraphembedding_amd/libhgx.so
AB_N=6000000 timeout -k 10 400 python -u tools/ab_train.py 128 hobe $L $L:train_prep_overlap=1 $L:train_prep_overlap=1,train_prep_cus=32 > $O/ab_ov.log 2>&1 || { echo ABFAIL; tail -20 $O/ab_ov.log; exit 12; }
cat $O/ab_ov.log
