"""Diagnostics for the MLP engine vs oracle/mlpref.c (GPU): with
HGX_MLP_GRAD_AT=k (both sides) batch k stores its raw gradients in the
weights; compare them bit for bit, layer by layer."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O
from hypergraphembedding_amd import _hgx
from test_gpu_mlp import glorot, make_case

ctx = _hgx.Context(0)
for kind, I, D in ((0, 40, 0), (1, 40, 24)):
  n = 256 * 3
  rng, nt, et, nr, er, lab = make_case(kind, I, D, n, 3)
  m = _hgx.Mlp(ctx, kind, I, D)
  w0 = glorot(m.shapes, rng, 0.1)
  m.set_tables(nt, et)
  m.set_samples(nr, er, lab)
  p = rng.permutation(n)[None, :]
  for at in (0, 1, 2):
    os.environ["HGX_MLP_GRAD_AT"] = str(at)
    m.set_weights(w0)
    m.fit(max_epochs=1, min_delta=-1e30, seed=77, perms=p)
    wg = m.get_weights()
    wc, _ = O.mlp_fit(kind, I, D, w0, nt, et, nr, er, lab, p, min_delta=-1e30, seed=77)
    off = 0
    for q, (kk, nn) in enumerate(m.shapes):
      for nm, cnt in (("W", kk * nn), ("b", nn)):
        a, b = wg[off:off + cnt], wc[off:off + cnt]
        idx = np.nonzero(a != b)[0]
        print(f"kind {kind} grad@{at} layer {q} {nm}: ndiff {len(idx)}/{cnt}",
              "" if not len(idx) else f"idx {idx[:4]} g {a[idx[:3]]} c {b[idx[:3]]} rel {np.abs(a[idx]-b[idx]).max()/np.abs(b).max():.2g}")
        off += cnt
  m.close()
