set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCHFAIL; exit 2; }
echo done
