# C4 HOBE sampling on a 10% row slice: node-row / edge-row 3-hop proposal
# thresholds set apart (args: pairs NODE_SHIFT:EDGE_SHIFT)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mode3e
mkdir -p $O
for p in "$@"; do
  n=${p%:*}; e=${p#*:}
  timeout -k 10 170 python3 -u tools/perf_hobe_c4.py --frac 0.1 --no-train --mode3-shift $n --mode3-shift-e $e > $O/s_${n}_${e}.json 2> $O/s_${n}_${e}.err || { echo FAIL $p; tail -3 $O/s_${n}_${e}.err; exit 11; }
  echo $p; tail -1 $O/s_${n}_${e}.json
done
