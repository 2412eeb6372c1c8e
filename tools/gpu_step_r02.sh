set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 120"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_streaming.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_train.log 2>&1 || { echo TESTFAIL; exit 1; }
$T python tools/perf_train.py 128 > gpurun_out/perf.log 2>&1 || exit 2
$T python tools/perf_train.py 256 >> gpurun_out/perf.log 2>&1 || exit 3
HGX_STEP_TB=128 HGX_LIB_PATH=tools/_ab/dbg.so $T python tools/perf_train.py 128 >> gpurun_out/perf.log 2>&1 || exit 4
HGX_STEP_TB=256 HGX_LIB_PATH=tools/_ab/dbg.so $T python tools/perf_train.py 256 >> gpurun_out/perf.log 2>&1 || exit 5
HGX_LIB_PATH=tools/_ab/dbg.so $T python tools/trace_train.py 128 > gpurun_out/trace_new.log 2>&1 || exit 6
HGX_LIB_PATH=tools/_ab/old.so $T python tools/trace_train.py 128 > gpurun_out/trace_old.log 2>&1 || exit 7
HGX_LIB_PATH=tools/_ab/old.so $T python tools/perf_train.py 128 > gpurun_out/perf_old.log 2>&1 || exit 8
echo done
