#!/bin/bash
# r03: the C5 combiner MLP with write-through (sc1) epilogue stores vs plain
# stores: tools/perf_c5_mlp.py per build, alternated (base, wt, base, wt).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_mlpwt}
mkdir -p $O
for r in 1 2; do
  for b in base mlpwt; do
    HGX_LIB_PATH=tools/_ab/$b.so timeout -k 10 240 python -u tools/perf_c5_mlp.py --samples 4000000 --epochs 2 > $O/c5_${b}_$r.jsonl 2>&1 || { echo FAIL $b; tail $O/c5_${b}_$r.jsonl; exit 11; }
    echo "$b run $r: $(tail -1 $O/c5_${b}_$r.jsonl | python -c 'import json,sys; d=json.load(sys.stdin); print(d["samples_per_s"], d["tflops"])')"
  done
done
