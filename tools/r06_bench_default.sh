# the default bench line as the driver runs it (now with the whole-C4 leg at
# N = 1), wall time measured around it
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_bench_default}
mkdir -p $O
t0=$(date +%s)
timeout -k 10 900 python -u bench.py --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -5 $O/bench.err; exit 14; }
echo "bench wall s: $(( $(date +%s) - t0 ))" | tee $O/wall.txt
