# r06: the numpy-seeded sampler tests, then the round evidence (bench, rocprof
# stats, PMC passes, the 2-rank launcher rehearsal)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_round
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_jaccard.py tests/test_gpu_mt.py -x -v --timeout 200 --timeout-method thread > $O/mt_tests.log 2>&1 || { echo MTFAIL; exit 10; }
echo mt-tests-ok
bash tools/gpu_round.sh r06_round bench
