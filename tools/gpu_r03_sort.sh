#!/bin/bash
# r03: chunk preparation LDS-batched bitonic sort in train_prep on a side stream: trainer GPU tests, then
# the bench's C3 line with the previous and the LDS-batched bitonic sort in train_prep library, alternated.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_sort}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_streaming.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 11; }
tail -1 $O/tests.log
for r in 1 2; do
  for b in prev sort; do
    HGX_LIB_PATH=tools/_ab/$b.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-c4 --no-extra > $O/bench_${b}_$r.json 2> $O/bench_${b}_$r.err || { echo FAIL $b; tail $O/bench_${b}_$r.err; exit 12; }
    echo "$b run $r: $(tail -1 $O/bench_${b}_$r.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["per_launch_us"])')"
  done
done
