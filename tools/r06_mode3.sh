# C4 HOBE sampling on a 10% row slice: the auto rule's threshold
# (sample_mode3_shift: uniform columns when W >= the column count * 2^shift)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mode3
mkdir -p $O
for d in "$@"; do
  timeout -k 10 170 python3 -u tools/perf_hobe_c4.py --frac 0.1 --no-train --mode3 0 --mode3-shift $d > $O/shift_$d.json 2> $O/shift_$d.err || { echo FAIL $d; tail -3 $O/shift_$d.err; exit 11; }
  tail -1 $O/shift_$d.json
done
