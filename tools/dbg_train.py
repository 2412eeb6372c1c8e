import sys, numpy as np
sys.path.insert(0, 'oracle'); sys.path.insert(0, '.')
import oracle as O
from hypergraphembedding_amd import _hgx
z = np.load('tests/golden/hobe_small.npz')
idx, tgt, K = z['idx'], z['tgt'], int(z['K'])
ctx = _hgx.Context(0)
for (n, batch, d) in [(64*63, 64, 8), (64*64, 64, 8), (64*64+10, 64, 8), (64*66, 64, 8), (64*20, 8, 8)]:
  rs = np.random.RandomState(0)
  I, T = idx[:n], tgt[:n]
  nrows = 120; erows = 45
  nt = rs.uniform(-0.05, 0.05, (nrows, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (erows, d)).astype(np.float32)
  perms = np.arange(n)[None, :]
  ont, oet, ol, _, _ = O.train(I, T, K, nt, et, 1, 1, batch=batch, max_epochs=1, perms=perms)
  ctx.records_set(I, T); ctx.model_init(d, nrows, erows, node_tab=nt, edge_tab=et)
  gl = ctx.train(batch=batch, max_epochs=1, loss=1, act=1, perms=perms)
  gnt, get_ = ctx.model_get()
  dn = np.abs(gnt - ont).max(1); de = np.abs(get_ - oet).max(1)
  print(n, batch, 'loss', ol, gl, 'maxdiff N', dn.max(), 'E', de.max())
  print('  node rows differing', np.nonzero(dn > 1e-6)[0][:20], 'edge rows', np.nonzero(de > 1e-6)[0][:20])
  dN0 = gnt - nt; oN0 = ont - nt
  r = np.argmax(dn)
  print('  worst node row', r, 'gpu delta', dN0[r][:4], 'oracle delta', oN0[r][:4])
