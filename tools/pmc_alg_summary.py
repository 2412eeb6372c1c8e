"""Summarise rocprofv3 --pmc passes of tools/perf_alg.py into a JSON of
per-kernel median counters and durations. Usage:
  python tools/pmc_alg_summary.py OUT_JSON CSV [CSV ...]"""
import collections, csv, json, re, sys
import numpy as np

out, paths = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in paths:
  for r in csv.DictReader(open(p)):
    name = r["Kernel_Name"]
    m = re.search(r"::(\w+)(<[^(]*>)?\(", name)
    short = (m.group(1) + (m.group(2) or "")) if m else name[:60]
    if not any(t in short for t in ("algdist", "seg_partial", "long_finish")):
      continue
    acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    acc[short]["duration_us"].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
res = {k: {c: float(np.median(v)) for c, v in d.items()} for k, d in acc.items()}
for k, d in res.items():
  if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
    d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
json.dump({"note": ("median per launch; FETCH_SIZE/WRITE_SIZE in KB as reported "
                    "(random 16-B-per-lane gathers: FETCH calibration unknown, "
                    "see DESIGN.md); duration from the counter pass"),
           "kernels": res}, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
