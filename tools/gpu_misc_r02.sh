#!/bin/bash
# r02 late checks: trainer A/B of tools/_ab builds, the C1 HOBE end-to-end
# GPU test, the 2-rank bench rehearsal (gloo, one device).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/misc
bash tools/ab_r02b.sh misc/ab tools/_ab/base.so tools/_ab/pf.so || exit 3
echo ab-ok
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k c1_hobe -x -v --timeout 240 --timeout-method thread > gpurun_out/misc/c1hobe.log 2>&1 || { echo C1HOBE_FAIL; tail -30 gpurun_out/misc/c1hobe.log; exit 4; }
echo c1hobe-ok
bash tools/gpu_mgpu_r02.sh
