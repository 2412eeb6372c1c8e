import sys, time, numpy as np
sys.path.insert(0, '.')
from hypergraphembedding_amd import _hgx
rs = np.random.RandomState(0)
N, E, K, d = 100000, 50000, 5, int(sys.argv[1]) if len(sys.argv) > 1 else 128
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
R = 4 + 2 * K
idx = np.zeros((n, R), np.int32)
kind = rs.randint(0, 3, n)
m0, m1, m2 = kind == 0, kind == 1, kind == 2
idx[m0, 0] = rs.randint(1, N + 1, m0.sum()); idx[m0, 2] = rs.randint(1, N + 1, m0.sum())
idx[m1, 1] = rs.randint(1, E + 1, m1.sum()); idx[m1, 3] = rs.randint(1, E + 1, m1.sum())
idx[m2, 0] = rs.randint(1, N + 1, m2.sum()); idx[m2, 3] = rs.randint(1, E + 1, m2.sum())
idx[m2, 4:4 + K] = rs.randint(1, N + 1, (m2.sum(), K)); idx[m2, 4 + K:] = rs.randint(1, E + 1, (m2.sum(), K))
tgt = np.zeros((n, 3), np.float32); tgt[np.arange(n), kind] = rs.uniform(0, 1, n)
ctx = _hgx.Context(0)
ctx.records_set(idx, tgt)
ctx.model_init(d, N + 2, E + 2, seed=1)
for ep in range(2):
  t = time.time()
  l = ctx.train(batch=256, max_epochs=1, loss=1, act=1, shuffle_seed=ep)
  wall = time.time() - t
  ms, rec, bat = ctx.train_stats()
  print(f"d={d} n={n} epoch wall {wall:.3f}s dev {ms:.1f}ms  {rec/ms*1e3/1e6:.2f} Mrec/s  {ms*1e3/bat:.2f} us/batch  loss {l}")
  print("  path (fused, split):", ctx.train_path_stats())
