#!/bin/bash
# r03: the GPU suite from a given test on (after a fix), then smoke().
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_rest}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 --deselect tests/test_gpu_c4.py --deselect tests/test_gpu_fullsize.py > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 12; }
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 13; }
echo smoke-ok
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -20 $O/bench.err; exit 14; }
echo bench-ok
tail -c 3000 $O/bench.json
