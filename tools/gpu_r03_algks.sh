#!/bin/bash
# r03: per-kernel times of the C4 alg-dist sweep at 48-B vs 64-B rows
# (tools/perf_alg_ks.py under rocprofv3 kernel trace).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_algks}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/perf_alg_ks.py c4 10 1 > $O/ks.json 2> $O/ks.err || exit 11
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/ \;
rm -rf $O/prof
echo ok
