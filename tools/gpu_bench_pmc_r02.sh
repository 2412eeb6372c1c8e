#!/bin/bash
# The bench line, then FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) of
# bench.py itself (one epoch, no CPU/C4/extra legs), summarised per trainer
# batch step into $O/pmc_train.json. Usage: tools/gpu_bench_pmc_r02.sh [tag]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r02}
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 14
echo bench-ok
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-c4 --no-extra \
    > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed rc=$?"; exit 16; }
  echo pmc-$C-ok
done
F=$(find $O/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)
python tools/pmc_train_summary.py "$F" "$W" $O/pmc_train.json 128 2 > /dev/null || exit 18
rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE
echo all-ok
