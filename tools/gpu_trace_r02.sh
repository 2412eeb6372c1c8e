set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 300"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_streaming.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_train.log 2>&1 || { echo TESTFAIL; exit 1; }
$T python tools/ab_train.py 128 rand tools/_ab/old.so tools/_ab/new.so > gpurun_out/ab.log 2>&1 || exit 2
$T python tools/ab_train.py 128 hobe tools/_ab/old.so tools/_ab/new.so >> gpurun_out/ab.log 2>&1 || exit 3
timeout -k 10 400 python tools/perf_hobe_c4.py > gpurun_out/c4.log 2>&1 || exit 4
echo done
