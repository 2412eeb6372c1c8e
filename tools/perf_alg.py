"""alg-dist timing: `python tools/perf_alg.py [c3|c4] [k] [iters]`.
Prints device ms per iteration and algorithmic GB/s (B_iter = 8 nnz +
(8 + 12k)(N + E))."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph, random_hypergraph

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
t = time.time()
inc = random_hypergraph() if cfg == "c3" else powerlaw_hypergraph()
print(f"{cfg}: N={inc.N} E={inc.E} nnz={inc.nnz} max edge {inc.edge_size().max()} "
      f"gen {time.time() - t:.1f}s", flush=True)
ctx = _hgx.Context(0)
t = time.time()
ctx.upload(inc)
print(f"upload {time.time() - t:.1f}s", flush=True)
rs = np.random.RandomState(0)
x0 = rs.random_sample((inc.N, k)).astype(np.float32)
y0 = rs.random_sample((inc.E, k)).astype(np.float32)
for i in range(3):
  ctx.alg_set(x0, y0)
  ctx.alg_run(iters)
  ms, by = ctx.alg_stats()
  print(f"k={k} {iters} it: {ms:.2f} ms  {by / ms / 1e6:.1f} GB/s  "
        f"{ms / iters * 1e3:.1f} us/iter", flush=True)
