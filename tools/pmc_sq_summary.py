"""Mean SQ counter values per launch of the trainer step kernel from a
rocprofv3 --pmc counter_collection.csv (diagnostic A/B of builds).
Usage: python tools/pmc_sq_summary.py CSV [KERNEL_SUBSTRING]"""
import csv, sys
import numpy as np
path = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "train_"
vals = {}
for r in csv.DictReader(open(path)):
  if key not in r["Kernel_Name"]:
    continue
  vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k in sorted(vals):
  print(f"{k:28s} {np.mean(vals[k]):14.1f}  (n={len(vals[k])})")
