set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_mtc3_prof
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u tools/mt_c3_hobe.py --no-oracle > $O/mt_c3_hobe.json 2> $O/mt_c3_hobe.err || { echo PROFFAIL; exit 13; }
find $O/prof -name '*stats.csv' -exec cp {} $O/ \;
rm -rf $O/prof
echo prof-ok
