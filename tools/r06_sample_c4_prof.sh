# per-kernel time of the C4 HOBE sampler on a 10% row slice (rocprofv3 stats)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sample_c4_prof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/sample_c4_probe.py 0.1 > $O/probe.json 2> $O/probe.err || { echo FAIL; tail $O/probe.err; exit 11; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/ \;
rm -rf $O/prof
cat $O/probe.json
