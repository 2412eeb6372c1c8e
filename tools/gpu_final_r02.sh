#!/bin/bash
# End-of-round check of the final tree: GPU test suite, smoke(), the C5
# combiner throughput and the rocprofv3 kernel stats of that run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02_close
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/gpu_tests.log; exit 11; }
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 12; }
echo smoke-ok
timeout -k 10 240 python -u tools/perf_c5_mlp.py > $O/c5_mlp.jsonl 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 tools/perf_c5_mlp.py --samples 2000000 --epochs 1 > $O/c5_prof.jsonl 2>&1 || exit 14
find $O/p -name "*kernel_stats.csv" -exec cp {} $O/c5_kernel_stats.csv \;
rm -rf $O/p
echo all-ok
