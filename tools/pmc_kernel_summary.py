"""Per-kernel mean of one rocprofv3 --pmc counter (counter_collection.csv):
python tools/pmc_kernel_summary.py CSV COUNTER OUT_JSON"""
import csv
import json
import sys

path, counter, out = sys.argv[1], sys.argv[2], sys.argv[3]
acc = {}
for r in csv.DictReader(open(path)):
  if r["Counter_Name"] != counter:
    continue
  k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
  k = k[5:] if k.startswith("void ") else k
  k = k.split("(")[0]
  s, n = acc.get(k, (0.0, 0))
  acc[k] = (s + float(r["Counter_Value"]), n + 1)
res = {k: {"mean": s / n, "launches": n} for k, (s, n) in acc.items()}
json.dump({"counter": counter, "unit": "KB (FETCH_SIZE / WRITE_SIZE)", "kernels": res},
          open(out, "w"), indent=1)
print(json.dumps(res, indent=1)[:2000])
