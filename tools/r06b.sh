set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mt.py tests/test_gpu_store.py -x -v --timeout 200 --timeout-method thread --durations=10 > $O/mt_store_tests.log 2>&1 || { echo TESTFAIL; exit 11; }
echo tests-ok
timeout -k 10 600 python3 -u bench.py --gpus 2 --one-device --dist-backend gloo --no-cpu --no-extra --steps 2 > $O/bench_2rank_launcher.json 2> $O/bench_2rank_launcher.err || { echo BENCHFAIL; exit 12; }
echo bench-ok
