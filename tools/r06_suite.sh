# GPU suite + smoke on one box (round evidence); TAG = output directory
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -5 $O/gpu_tests.log; exit 11; }
echo tests-ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; exit 12; }
echo smoke-ok
