#!/bin/bash
# r03 close: one full C4 HOBE d=256 epoch (every row, row-range chunks) and
# the C5 combiner throughput on the final tree.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_c4c5}
mkdir -p $O
timeout -k 10 900 python -u tools/perf_hobe_c4_full.py > $O/c4_full_epoch.jsonl 2> $O/c4_full_epoch.err || { echo C4FAIL; tail -20 $O/c4_full_epoch.err; exit 11; }
tail -1 $O/c4_full_epoch.jsonl
timeout -k 10 300 python -u tools/perf_c5_mlp.py > $O/c5_mlp.jsonl 2> $O/c5_mlp.err || { echo C5FAIL; tail -20 $O/c5_mlp.err; exit 12; }
tail -2 $O/c5_mlp.jsonl
