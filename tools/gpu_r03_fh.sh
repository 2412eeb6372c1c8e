#!/bin/bash
# r03: write-through float2 trainer rows + fused MLP head: trainer / MLP GPU
# tests, then the C5 combiner throughput (fused vs separate head launch).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_fh}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py tests/test_gpu_streaming.py tests/test_gpu_lp_combine.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 11; }
tail -2 $O/tests.log
timeout -k 10 240 python -u tools/perf_c5_mlp.py --samples 4000000 --epochs 2 > $O/c5_fused.jsonl 2>&1 || { echo C5FAIL; tail $O/c5_fused.jsonl; exit 12; }
tail -1 $O/c5_fused.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/perf_c5_mlp.py --samples 2000000 --epochs 1 > $O/c5_prof.jsonl 2>&1 || { echo PROFFAIL; exit 13; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/c5_kernel_stats.csv \;
rm -rf $O/prof
cut -d, -f1-4 $O/c5_kernel_stats.csv | head -8
