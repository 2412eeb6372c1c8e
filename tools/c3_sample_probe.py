"""HOBE sampling of C3 (random 100k/50k, S = 200, K = 5) timed `reps` times
after one warm call (A/B of builds via HGX_LIB_PATH). Diagnostic only."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx  # noqa: E402
from hypergraphembedding_amd.synthetic import random_hypergraph  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
inc = random_hypergraph(seed=0)
ctx = _hgx.Context(0)
rs = np.random.RandomState(0)
x0, y0 = rs.random_sample((inc.N, 10)), rs.random_sample((inc.E, 10))
ts = []
for r in range(reps + 1):
  ctx.upload(inc)  # a fresh incidence each time (filters rebuilt, as in bench.py)
  ctx.alg_set(x0, y0)
  ctx.alg_run(20)
  ctx.synchronize()
  t = time.perf_counter()
  n = ctx.sample_hobe(4000, 5, 200)
  ctx.synchronize()
  if r:
    ts.append(time.perf_counter() - t)
print(json.dumps({"records": n, "sample_s": [round(v, 4) for v in ts],
                  "median_s": round(float(np.median(ts)), 4)}))
ctx.close()
