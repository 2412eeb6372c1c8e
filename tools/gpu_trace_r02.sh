set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10 300"
HGX_STEP_TB=128 $T python tools/ab_train.py 128 rand tools/_ab/old.so tools/_ab/dbg.so tools/_ab/one.so > gpurun_out/ab.log 2>&1 || exit 2
$T python tools/ab_train.py 256 rand tools/_ab/old.so tools/_ab/v2.so >> gpurun_out/ab.log 2>&1 || exit 3
$T python tools/ab_train.py 256 hobe tools/_ab/old.so tools/_ab/v2.so >> gpurun_out/ab.log 2>&1 || exit 3
echo done
