#!/bin/bash
# r03: trainer ablations (debug build), then the multi-rank bench rehearsal.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_abl}
mkdir -p $O
HGX_LIB_PATH=tools/_ab/dbg.so timeout -k 10 400 python -u tools/ablate_train.py 128 > $O/ablate_d128.jsonl 2>&1 || { echo ABLFAIL; tail -20 $O/ablate_d128.jsonl; exit 11; }
cat $O/ablate_d128.jsonl
bash tools/gpu_r03_mgpu.sh ${1:-r03_abl}_mgpu || exit 12
