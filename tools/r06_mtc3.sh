set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_mtc3
mkdir -p $O
timeout -k 10 900 python3 -u tools/mt_c3_hobe.py > $O/mt_c3_hobe.json 2> $O/mt_c3_hobe.err || { echo MTC3FAIL; exit 13; }
echo mtc3-ok
