# float2 x 64-lane step geometry at d=128: trainer parity tests, then an
# interleaved A/B against the pre-change library and the other geometries,
# and a phase trace of the default
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py > gpurun_out/vw_tests.log 2>&1 || { tail -40 gpurun_out/vw_tests.log; exit 1; }
tail -3 gpurun_out/vw_tests.log
L=hypergraphembedding_amd/libhgx.so
for kind in rand hobe; do
  timeout -k 10 200 python -u tools/ab_train.py 128 $kind tools/_ab/pre_vw.so $L:train_lanes=32 $L:train_tb=256 $L:train_tb=512 > gpurun_out/vw_ab_$kind.log 2>&1 || { cat gpurun_out/vw_ab_$kind.log; exit 1; }
  cat gpurun_out/vw_ab_$kind.log
done
timeout -k 10 200 python -u tools/trace_train.py 128 hobe > gpurun_out/vw_trace.log 2>&1 || { cat gpurun_out/vw_trace.log; exit 1; }
head -8 gpurun_out/vw_trace.log
