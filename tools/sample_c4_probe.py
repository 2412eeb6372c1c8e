"""HOBE sampling of the C4 power-law graph alone (bench.py's hobe_d256
slice: a seeded `frac` of node rows and edge rows at S = 200, K = 5), for a
per-dispatch kernel trace of the sampler (rocprofv3 --kernel-trace):
reject_rows / expand_rows run per pattern in the order nn, ee, nne, een;
then the probabilities (hobe_nn_kernel, hobe_wave_kernel). Diagnostic.

  python tools/sample_c4_probe.py [frac=0.02]"""
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx  # noqa: E402
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph  # noqa: E402

frac = float(sys.argv[1]) if len(sys.argv) > 1 else 0.02
big = powerlaw_hypergraph(seed=0)
ctx = _hgx.Context(0)
ctx.upload(big)
rs4 = np.random.RandomState(1)
ctx.alg_set(rs4.random_sample((big.N, 10)).astype(np.float32),
            rs4.random_sample((big.E, 10)).astype(np.float32))
ctx.alg_run(20)
rsq = np.random.RandomState(2)
nq = np.where(rsq.random_sample(big.N) < frac, 200, 0).astype(np.int32)
eq = np.where(rsq.random_sample(big.E) < frac, 200, 0).astype(np.int32)
for rep in range(2):
  ctx.synchronize()
  t = time.perf_counter()
  n = ctx.sample_hobe(4000, 5, 200, node_q=nq, edge_q=eq)
  ctx.synchronize()
  dt = time.perf_counter() - t
  print(json.dumps({"rep": rep, "records": n, "sample_s": round(dt, 3),
                    "stats": list(ctx.sample_stats()),
                    "uniform_rows": ctx.sample_uniform_rows()}), flush=True)
idx, tgt = ctx.records_get()
h = hashlib.sha256()
h.update(idx.tobytes())
h.update(tgt.tobytes())
print(json.dumps({"records_sha256": h.hexdigest()}), flush=True)
ctx.close()
