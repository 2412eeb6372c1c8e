#!/bin/bash
# r03: ablations + phase trace of the current step (debug build)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_abl2}
mkdir -p $O
HGX_LIB_PATH=tools/_ab/dbg.so timeout -k 10 400 python -u tools/ablate_train.py 128 > $O/ablate_d128.jsonl 2>&1 || { echo ABLFAIL; tail -20 $O/ablate_d128.jsonl; exit 11; }
cat $O/ablate_d128.jsonl
HGX_LIB_PATH=tools/_ab/dbg.so timeout -k 10 300 python -u tools/trace_train.py 128 hobe > $O/trace_d128_hobe.log 2>&1 || { echo TRACEFAIL; tail -20 $O/trace_d128_hobe.log; exit 12; }
head -6 $O/trace_d128_hobe.log
