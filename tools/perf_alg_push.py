"""A/B of the alg-dist edge half: gather (alg_push 0) vs push form
(alg_push 1), interleaved in one process on one graph.
`python tools/perf_alg_push.py [c3|c4] [iters] [rounds]`: device ms per
iteration of each mode and the max-abs difference of their results."""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph, random_hypergraph

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ks = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # alg_ks tuning (0: 12)
inc = random_hypergraph() if cfg == "c3" else powerlaw_hypergraph()
ctx = _hgx.Context(0)
ctx.set_tuning("alg_ks", ks)
ctx.upload(inc)
rs = np.random.RandomState(0)
x0 = rs.random_sample((inc.N, 10)).astype(np.float32)
y0 = rs.random_sample((inc.E, 10)).astype(np.float32)
b_iter = 8.0 * inc.nnz + (8.0 + 12.0 * 10) * (inc.N + inc.E)
res = {0: [], 1: []}
out = {}
for r in range(rounds):
  for mode in (0, 1):
    ctx.set_tuning("alg_push", mode)
    ctx.alg_set(x0, y0)
    t = time.perf_counter()
    ctx.alg_run(iters)
    wall = time.perf_counter() - t
    ms, _ = ctx.alg_stats()
    res[mode].append(ms / iters)
    print(json.dumps({"cfg": cfg, "push": mode, "round": r, "ks": ks,
                      "ms_per_iter": round(ms / iters, 4),
                      "gbps": round(b_iter / (ms / iters) / 1e6, 1),
                      "wall_s": round(wall, 3)}), flush=True)
    if r == 0:
      out[mode] = ctx.alg_get()
d = max(float(np.abs(out[0][0] - out[1][0]).max()),
        float(np.abs(out[0][1] - out[1][1]).max()))
print(json.dumps({"cfg": cfg, "ks": ks, "median_ms_per_iter": {m: round(float(np.median(v)), 4)
                                                      for m, v in res.items()},
                  "max_abs_diff_push_vs_gather": d}), flush=True)
