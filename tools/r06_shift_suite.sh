# after a deliberate sampler-stream change: regenerate the pinned stream
# shas on this box, then the whole GPU suite and smoke against them
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/shift_suite
mkdir -p $O
timeout -k 10 300 python3 -u tests/golden/make_stream_sha.py $O/stream_sha.json > $O/make_sha.log 2>&1 || { echo SHAFAIL; tail $O/make_sha.log; exit 10; }
cp $O/stream_sha.json tests/golden/stream_sha.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -5 $O/gpu_tests.log; exit 11; }
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; exit 12; }
echo smoke-ok
