#!/bin/bash
# HEAD check on a fresh box: GPU suite, smoke, bench line. Usage: tools/gpu_r03_head.sh TAG
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_head}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; exit 11; }
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; exit 12; }
echo smoke-ok
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 14
echo bench-ok
