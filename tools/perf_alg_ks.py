"""A/B of the alg-dist coordinate row width (tuning alg_ks: 12 = 48-B rows,
16 = 64-B rows aligned to the 64-B memory sectors), interleaved in one
process. `python tools/perf_alg_ks.py [c3|c4] [iters] [rounds]`."""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph, random_hypergraph

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
inc = random_hypergraph() if cfg == "c3" else powerlaw_hypergraph()
ctx = _hgx.Context(0)
ctx.upload(inc)
rs = np.random.RandomState(0)
x0 = rs.random_sample((inc.N, 10)).astype(np.float32)
y0 = rs.random_sample((inc.E, 10)).astype(np.float32)
b_iter = 8.0 * inc.nnz + (8.0 + 12.0 * 10) * (inc.N + inc.E)
res, out = {12: [], 16: []}, {}
for r in range(rounds):
  for ks in (12, 16):
    ctx.set_tuning("alg_ks", ks)
    ctx.alg_set(x0, y0)
    ctx.alg_run(iters)
    ms, _ = ctx.alg_stats()
    res[ks].append(ms / iters)
    if r == 0:
      out[ks] = ctx.alg_get()
med = {k: float(np.median(v)) for k, v in res.items()}
print(json.dumps({"cfg": cfg, "iters": iters,
                  "ms_per_iter": {k: round(v, 4) for k, v in med.items()},
                  "gbps": {k: round(b_iter / v / 1e6, 1) for k, v in med.items()},
                  "runs": {k: [round(x, 4) for x in v] for k, v in res.items()},
                  "max_abs_diff": max(float(np.abs(out[12][0] - out[16][0]).max()),
                                      float(np.abs(out[12][1] - out[16][1]).max()))}),
      flush=True)
