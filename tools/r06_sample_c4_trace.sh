# per-dispatch durations of the C4 HOBE sampler's kernels on a 10% row slice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sample_c4_trace
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/sample_c4_probe.py 0.1 > $O/probe.json 2> $O/probe.err || { echo FAIL; tail $O/probe.err; exit 11; }
f=$(find $O/tr -name '*kernel_trace.csv')
python3 - "$f" > $O/dispatches.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
  d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
  if d > 1.0:
    print(f"{d:10.2f} ms  {r['Kernel_Name'][:70]}")
PY
rm -rf $O/tr
cat $O/dispatches.txt
