# targeted GPU check after a sampler-default change: the stream pin, the C4
# tests and their deferred oracle checks, then smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c4check
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_stream_pin.py tests/test_gpu_c4.py tests/test_gpu_samplers.py tests/test_gpu_zz_deferred.py -x -v --timeout 700 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -5 $O/tests.log; exit 11; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; exit 12; }
echo smoke-ok
