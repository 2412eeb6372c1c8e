"""Summarise the reject_rows per-row diagnostics (a -DHGX_DEBUG_KNOBS build,
HGX_REJ_DIAG_OUT=file): per pattern and mode, rows, rounds and time (ticks
of s_memrealtime, 100 MHz), and the slowest rows. Diagnostic only.

  python tools/rej_diag_summary.py DIAG.bin [first N records]"""
import json
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 8)
names = {2: "nn", 3: "ee", 4: "nne", 5: "een"}
modes = {0: "2hop-paths", 1: "3hop-paths", 2: "uniform-cols"}
out = {"rows": int(a.shape[0])}
# keep the first pass over the patterns (the probe samples twice)
seen, cut = set(), a.shape[0]
for i, p in enumerate(a[:, 0]):
  if p in seen and i > 0 and a[i - 1, 0] != p:
    cut = i
    break
  seen.add(int(p))
a = a[:cut]
out["rows_first_pass"] = int(a.shape[0])
groups = []
for p in sorted(set(a[:, 0].tolist())):
  for m in sorted(set(a[a[:, 0] == p, 2].tolist())):
    s = a[(a[:, 0] == p) & (a[:, 2] == m)]
    us = s[:, 7] / 100.0
    groups.append({
        "pattern": names.get(p, p), "mode": modes.get(m, "deferred%d" % m),
        "rows": int(s.shape[0]), "row_us_sum": round(float(us.sum()), 1),
        "row_us_p50": round(float(np.median(us)), 1),
        "row_us_p99": round(float(np.quantile(us, 0.99)), 1),
        "row_us_max": round(float(us.max()), 1),
        "rounds_mean": round(float(s[:, 6].mean()), 2),
        "rounds_max": int(s[:, 6].max()),
        "n1_p50": int(np.median(s[:, 3])), "W_p50": int(np.median(s[:, 5]))})
out["groups"] = groups
slow = a[np.argsort(-a[:, 7])[:20]]
out["slowest"] = [{"pattern": names.get(int(r[0])), "row": int(r[1]),
                   "mode": int(r[2]), "n1": int(r[3]), "q": int(r[4]),
                   "W": int(r[5]), "rounds": int(r[6]), "us": r[7] / 100.0}
                  for r in slow]
print(json.dumps(out, indent=1))
