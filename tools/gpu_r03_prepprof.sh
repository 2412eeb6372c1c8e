#!/bin/bash
# r03: kernel times of the trainer's chunk preparation (train_prep /
# train_place) for two builds, rocprofv3 kernel trace of one bench epoch.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_prepprof}
mkdir -p $O
for b in prev sort; do
  HGX_LIB_PATH=tools/_ab/$b.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-c4 --no-extra > $O/b_$b.json 2> $O/b_$b.err || { echo FAIL $b; exit 11; }
  find $O/p_$b -name '*kernel_stats.csv' -exec cp {} $O/ks_$b.csv \;
  rm -rf $O/p_$b
  python3 -c "
import csv
for r in csv.DictReader(open('$O/ks_$b.csv')):
  if 'train_' in r['Name'] or 'shuffle' in r['Name']: print('$b', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"
done
