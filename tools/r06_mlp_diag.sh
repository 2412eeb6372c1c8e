set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mlp_diag
mkdir -p $O
HGX_LIB_PATH=tools/_ab/mlp_diag.so timeout -k 10 240 python3 -u tools/perf_c5_mlp.py --samples 2000000 --epochs 1 > $O/diag.log 2>&1 || { echo FAIL; tail $O/diag.log; exit 11; }
cat $O/diag.log
