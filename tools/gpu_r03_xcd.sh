#!/bin/bash
# r03: one-XCD persistent batch skeleton vs launch per batch; alg-dist row
# width 12 vs 16 at C3 and C4.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/${1:-r03_xcd}
mkdir -p $O
timeout -k 10 120 tools/xcd_persist 4000 > $O/xcd_persist.jsonl 2>&1 || { echo XCDFAIL; tail $O/xcd_persist.jsonl; exit 11; }
cat $O/xcd_persist.jsonl
timeout -k 10 200 python -u tools/perf_alg_ks.py c3 20 3 > $O/ks_c3.json 2>&1 || { echo KS3FAIL; tail $O/ks_c3.json; exit 12; }
cat $O/ks_c3.json
timeout -k 10 300 python -u tools/perf_alg_ks.py c4 20 3 > $O/ks_c4.json 2>&1 || { echo KS4FAIL; tail $O/ks_c4.json; exit 13; }
cat $O/ks_c4.json
timeout -k 10 300 python -u tools/ab_train.py 128 hobe tools/_ab/base.so tools/_ab/gfirst.so > $O/ab_gfirst.log 2>&1 || { echo ABFAIL; tail $O/ab_gfirst.log; exit 14; }
cat $O/ab_gfirst.log
