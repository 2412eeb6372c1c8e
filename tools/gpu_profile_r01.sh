#!/bin/bash
# One GPU session: the GPU test suite, trainer perf, bench line, rocprofv3 kernel
# stats of the bench, FETCH/WRITE PMC passes of the trainer (separate runs).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1 || exit 11
timeout -k 10 120 python tools/perf_train.py 128 > $O/perf_train.log 2>&1 || exit 12
timeout -k 10 120 python tools/perf_train.py 256 >> $O/perf_train.log 2>&1 || exit 13
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 14
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python bench.py --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err || exit 15
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python tools/perf_train.py 128 400000 > $O/pmc_fetch.log 2>&1 || exit 16
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python tools/perf_train.py 128 400000 > $O/pmc_write.log 2>&1 || exit 17
# keep the summaries only (gpurun copies back at most 64 MiB)
F=$(find $O/pmc_fetch -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc_write -name '*counter_collection.csv' | head -1)
python tools/pmc_train_summary.py "$F" "$W" $O/pmc_train.json 128 1 > /dev/null || exit 18
find $O/prof_bench -name '*stats.csv' -exec cp {} $O/ \;
rm -rf $O/pmc_fetch $O/pmc_write $O/prof_bench
echo all-ok
