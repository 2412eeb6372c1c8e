# combiner MLP: plain vs write-through output stores (HGX_MLP_WT), interleaved
# A/B of the C5 perf tool, then the MLP tests on the write-through build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mlp_wt
mkdir -p $O
for r in 1 2; do
  for v in base wt1; do
    if [ $v = base ]; then L=""; else L=tools/_ab/mlp_$v.so; fi
    HGX_LIB_PATH=$L timeout -k 10 240 python3 -u tools/perf_c5_mlp.py --samples 8000000 --epochs 2 > $O/perf_${v}_$r.json 2>&1 || { echo PERFFAIL $v; exit 11; }
    echo $v $r; tail -1 $O/perf_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['samples_per_s'])"
  done
done
HGX_LIB_PATH=tools/_ab/mlp_wt1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_lp_combine.py -x -q --timeout 300 --timeout-method thread > $O/mlp_tests_wt1.log 2>&1 || { echo TESTFAIL; tail -20 $O/mlp_tests_wt1.log; exit 12; }
tail -2 $O/mlp_tests_wt1.log
