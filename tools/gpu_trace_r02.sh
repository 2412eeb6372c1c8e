set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 300"
HGX_LIB_PATH=tools/_ab/dbg.so $T python tools/trace_train.py 128 > gpurun_out/trace_ovl.log 2>&1 || exit 2
HGX_TRAIN_OVERLAP=0 HGX_LIB_PATH=tools/_ab/dbg.so $T python tools/trace_train.py 128 > gpurun_out/trace_novl.log 2>&1 || exit 2
echo done
