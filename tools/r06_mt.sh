set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_mt2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mt.py tests/test_gpu_jaccard.py -x -v --timeout 300 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MTFAIL; exit 10; }
echo mt-tests-ok
