import sys, time, numpy as np
sys.path.insert(0, '.')
from hypergraphembedding_amd import _hgx
from hypergraphembedding_amd.synthetic import random_hypergraph
t = time.time(); inc = random_hypergraph(); print('gen', time.time() - t, inc.N, inc.E, inc.nnz, flush=True)
ctx = _hgx.Context(0)
t = time.time(); ctx.upload(inc); print('upload', time.time() - t, flush=True)
rs = np.random.RandomState(0)
t = time.time(); ctx.alg_set(rs.random_sample((inc.N, 10)), rs.random_sample((inc.E, 10))); print('alg_set', time.time() - t, flush=True)
for i in range(3):
  ctx.alg_run(20); ms, by = ctx.alg_stats(); print(f'algdist 20 it: {ms:.2f} ms  {by/ms/1e6:.1f} GB/s  {ms/20*1e3:.1f} us/iter', flush=True)
t = time.time(); nq = np.full(inc.N, 200, np.int32); eq = np.full(inc.E, 200, np.int32)
n = ctx.sample_fobe(1, 5, nq, eq); print('fobe', n, time.time() - t, flush=True)
t = time.time(); n = ctx.sample_hobe(1, 5, 200); print('hobe', n, time.time() - t, flush=True)
ctx.model_init(128, inc.N + 2, inc.E + 2, seed=1)
for ep in range(2):
  l = ctx.train(batch=256, max_epochs=1, loss=1, act=1, shuffle_seed=ep)
  ms, rec, bat = ctx.train_stats()
  print(f"train epoch {ms:.1f} ms  {rec/ms*1e3/1e6:.2f} Mrec/s  {ms*1e3/bat:.2f} us/batch  loss {l}", flush=True)
