import sys, time, numpy as np
sys.path.insert(0, '.')
from hypergraphembedding_amd import _hgx
from hypergraphembedding_amd.synthetic import random_hypergraph
inc = random_hypergraph()
ctx = _hgx.Context(0)
ctx.upload(inc)
rs = np.random.RandomState(0)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
ctx.alg_set(rs.random_sample((inc.N, k)), rs.random_sample((inc.E, k)))
for i in range(3):
  ctx.alg_run(20); ms, by = ctx.alg_stats(); print(f'k={k} algdist 20 it: {ms:.2f} ms  {by/ms/1e6:.1f} GB/s  {ms/20*1e3:.1f} us/iter', flush=True)
