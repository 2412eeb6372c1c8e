# closing evidence of r06: the default bench line, then the same command under
# rocprofv3 (kernel stats); TAG = output directory
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_final}
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; exit 14; }
echo bench-ok
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --no-cpu --no-c4-full > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROFFAIL; exit 15; }
find $O/prof_bench -name '*stats.csv' -exec cp {} $O/ \;
rm -rf $O/prof_bench
echo prof-ok
