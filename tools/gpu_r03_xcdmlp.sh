#!/bin/bash
# r03: XCD-grouped tile order in the MLP GEMM launches vs the identity
# order: MLP tests, then tools/perf_c5_mlp.py per build, alternated.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_xcdmlp}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 11; }
tail -1 $O/tests.log
for r in 1 2; do
  for b in noxcd xcd; do
    HGX_LIB_PATH=tools/_ab/$b.so timeout -k 10 240 python -u tools/perf_c5_mlp.py --samples 4000000 --epochs 2 > $O/c5_${b}_$r.jsonl 2>&1 || { echo FAIL $b; tail $O/c5_${b}_$r.jsonl; exit 12; }
    echo "$b run $r: $(tail -1 $O/c5_${b}_$r.jsonl | python -c 'import json,sys; d=json.load(sys.stdin); print(d["samples_per_s"], d["tflops"])')"
  done
done
