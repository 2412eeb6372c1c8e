set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_mtc3_prof
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mt.py tests/test_gpu_jaccard.py -x -q --timeout 300 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MTFAIL; exit 10; }
echo mt-tests-ok
timeout -k 10 300 python3 -u tools/mt_c3_hobe.py --no-oracle > $O/mt_c3_hobe.json 2> $O/mt_c3_hobe.err || { echo MTC3FAIL; exit 13; }
echo mtc3-ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u tools/mt_c3_hobe.py --no-oracle > $O/mt_c3_hobe_prof.json 2> $O/mt_c3_hobe_prof.err || { echo PROFFAIL; exit 14; }
find $O/prof -name '*stats.csv' -exec cp {} $O/ \;
rm -rf $O/prof
echo prof-ok
