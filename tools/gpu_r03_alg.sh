#!/bin/bash
# r03: alg-dist push form -- parity tests, interleaved A/B at C4 and C3,
# rocprofv3 kernel stats of both forms at C4.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_alg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_algdist_probs.py tests/test_gpu_mlp.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 11; }
echo tests-ok
timeout -k 10 300 python -u tools/perf_alg_push.py c4 20 3 > $O/ab_c4.jsonl 2>&1 || { echo ABFAIL; tail -20 $O/ab_c4.jsonl; exit 12; }
cat $O/ab_c4.jsonl
timeout -k 10 200 python -u tools/perf_alg_push.py c3 20 3 > $O/ab_c3.jsonl 2>&1 || { echo ABFAIL3; tail -20 $O/ab_c3.jsonl; exit 13; }
tail -1 $O/ab_c3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python3 tools/perf_alg_push.py c4 5 1 > $O/prof.log 2>&1 || { echo PROFFAIL; tail -20 $O/prof.log; exit 14; }
find $O/p -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/p
head -30 $O/kernel_stats.csv | cut -c1-220
