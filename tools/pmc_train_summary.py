"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (of bench.py, or
tools/perf_train.py) into profiles/<round>_pmc_train.json: HBM bytes per
batch step (train_step, or train_fwd_bwd + train_update), gfx950 FETCH
correction x2 (MI355X_MICROARCH.md, HBM section). Usage:
  python tools/pmc_train_summary.py FETCH_CSV WRITE_CSV OUT_JSON d ROUND [CMD]"""
import csv, json, sys
import numpy as np

fetch_csv, write_csv, out, d = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])


def per_kernel(path, counter):
  vals = {}
  for r in csv.DictReader(open(path)):
    if r["Counter_Name"] != counter:
      continue
    name = r["Kernel_Name"]
    for key in ("train_fwd_bwd", "train_update", "train_step", "train_flush"):
      if key in name:
        vals.setdefault(key, []).append(float(r["Counter_Value"]))
        if key == "train_step":  # the light / MULTI pending-slot forms
          form = "train_step[MULTI]" if "true>" in name else "train_step[plain]"
          vals.setdefault(form, []).append(float(r["Counter_Value"]))
  return {k: float(np.mean(v)) for k, v in vals.items()}, \
      {k: len(v) for k, v in vals.items()}


f, nf = per_kernel(fetch_csv, "FETCH_SIZE")
w, nw = per_kernel(write_csv, "WRITE_SIZE")
# per batch step: every batch runs train_step (or K1 + K2); the flush runs
# once per epoch (and before a restart), so it is averaged over batches
steps = max(nf.get("train_step", 0) + nf.get("train_fwd_bwd", 0), 1)
def per_step(vals, counts):
  return sum(vals[k] * counts[k] for k in vals if "[" not in k) / steps
hbm = 1024 * (2 * per_step(f, nf) + per_step(w, nw))
alg = 256 * (224 * d + 68)
res = {
    "round": int(sys.argv[5]) if len(sys.argv) > 5 else 1,
    "command": ("rocprofv3 --pmc FETCH_SIZE (pass 1) / "
                "--pmc WRITE_SIZE (pass 2) --output-format csv -- python3 "
                + (sys.argv[6] if len(sys.argv) > 6 else
                   "bench.py --steps 1 --warmup 0 --no-cpu --no-c4 --no-extra")),
    "note": ("Per batch of 256 records at d=%d, summed over "
             "the per-batch kernels (train_step, or train_fwd_bwd + train_update, and the "
             "deferred-row flush once per epoch), per batch step. FETCH_SIZE / "
             "WRITE_SIZE are KB; gfx950 correction: FETCH doubled (wide 16-B-per-"
             "lane reads are tallied at half), WRITE as is. Infinity-Cache hits "
             "are counted by these counters." % d),
    "launches": {"fetch": nf, "write": nw},
    "fetch_kb_per_batch": f,
    "write_kb_per_batch": w,
    "hbm_bytes_per_batch": int(round(hbm)),
    "algorithmic_bytes_per_batch": alg,
}
forms = {k: int(round(1024 * (2 * f[k] + w.get(k, 0.0))))
         for k in f if k.startswith("train_step[")}
if forms:
  res["hbm_bytes_per_batch_by_form"] = forms
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
