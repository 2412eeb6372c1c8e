set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05load2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_store.py -x -v --timeout 120 --timeout-method thread > $O/store_tests.log 2>&1 || exit 10
timeout -k 10 400 python -u tools/perf_hobe_c4_full.py --N 2000000 --E 1000000 --chunk 268435456 > $O/plain.jsonl 2> $O/plain.err || exit 11
