set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05rccl
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -k "rccl" > $O/tests.log 2>&1 || exit 10
