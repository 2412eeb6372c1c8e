#!/bin/bash
# Round evidence: GPU test suite, bench line, rocprofv3 kernel stats of the
# bench, FETCH/WRITE PMC passes of bench.py (separate runs) summarised per
# batch step. Usage: tools/gpu_round.sh TAG [tests|bench|all]  (the GPU
# suite alone takes ~11 min: run the two parts as separate gpurun calls)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-round}
mkdir -p $O
PART=${2:-all}
if [ $PART != bench ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; exit 11; }
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; exit 12; }
echo smoke-ok
fi
[ $PART = tests ] && exit 0
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 14
echo bench-ok
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --no-cpu --no-c4-full > $O/bench_prof.json 2> $O/bench_prof.err || exit 15
find $O/prof_bench -name '*stats.csv' -exec cp {} $O/ \;
rm -rf $O/prof_bench
echo prof-ok
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-c4 --no-extra \
    > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed rc=$?"; exit 16; }
done
F=$(find $O/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)
W=$(find $O/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)
python tools/pmc_train_summary.py "$F" "$W" $O/pmc_train.json 128 6 > /dev/null || exit 18
rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE
# the --gpus N path rehearsed on one GPU: bench.py starts its 2 ranks itself
# (gloo on cuda:0; not a scaling measurement: both ranks share one GPU)
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 1 --warmup 0 --one-device --dist-backend gloo --no-cpu --no-extra > $O/bench_2rank_gloo.json 2> $O/bench_2rank_gloo.err || { echo G2FAIL; exit 19; }
echo all-ok
