"""The BASELINE.json configurations end to end on the GPU:

C1  youtube_tiny FOBE d=16: the reference's record stream (the oracle's
    MT19937 replica, sha-pinned to fixtures made by the reference), trained on
    the device for up to 10 epochs with EarlyStopping on the oracle's batch
    order; per-row cosine vs the CPU restatement (SURVEY §8c tolerance:
    p50 >= 0.9999, p1 >= 0.999) and the same epochs run.
C1  youtube_tiny HOBE d=16: device alg-dist -> device probabilities on the
    reference's pair stream -> device training, vs the reference coordinates
    and the CPU restatement (same tolerance).
C2  random 100k/50k FOBE d=128: exact per-row counts and pair validity on
    sampled rows, trainer determinism and a decreasing loss.
C5  the N_E_SUPERVISED combiner on two d=256 embeddings (FOBE, HOBE) of a
    row slice of the power-law 10M/5M graph: the dense-MLP engine bit-exact
    vs oracle/mlpref.c on a sample of the combiner's samples, then two
    epochs over all of the slice's samples (positives + 5x negatives).
"""

import hashlib

import numpy as np
import pytest

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
  from hypergraphembedding_amd import _hgx
  c = _hgx.Context(0)
  yield c
  c.close()


def _sha(idx, tgt):
  h = hashlib.sha256()
  h.update(np.ascontiguousarray(idx, np.int32).tobytes())
  h.update(np.ascontiguousarray(tgt, np.float32).tobytes())
  return h.hexdigest()


def _row_cos(a, b):
  num = (a * b).sum(1)
  den = np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1)
  return num / np.maximum(den, 1e-30)


def test_c1_fobe_end_to_end_cosine(ctx, tiny_inc):
  from hypergraphembedding_amd import _hgx
  z = golden("fobe_tiny.npz")
  K, S = int(z["K"]), int(z["S"])
  inc = tiny_inc
  idx, tgt = O.fobe_sample(O.Rng(int(z["seed"])), inc,
                           np.full(inc.N, S, np.int32),
                           np.full(inc.E, S, np.int32), K)
  assert idx.shape[0] == int(z["n"]) and _sha(idx, tgt) == str(z["sha"])
  n, d = idx.shape[0], 16
  rs = np.random.RandomState(11)
  perms = np.stack([rs.permutation(n) for _ in range(10)])
  nt = rs.uniform(-0.05, 0.05, (inc.N + 1, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (inc.E + 1, d)).astype(np.float32)
  ont, oet, ol, _, _ = O.train(idx, tgt, K, nt, et, O.LOSS_KLD, O.ACT_SIGMOID,
                               batch=256, max_epochs=10, perms=perms,
                               min_delta=1e-3)
  ctx.upload(inc)
  ctx.records_set(idx, tgt)
  ctx.model_init(d, inc.N + 1, inc.E + 1, node_tab=nt, edge_tab=et)
  gl = ctx.train(batch=256, max_epochs=10, loss=_hgx.LOSS_KLD,
                 act=_hgx.ACT_SIGMOID, min_delta=1e-3, perms=perms)
  gnt, get_ = ctx.model_get()
  assert len(gl) == len(ol), (gl, ol)  # EarlyStopping stopped at the same epoch
  np.testing.assert_allclose(gl, ol, rtol=1e-4)
  for g, o in ((gnt[1:], ont[1:]), (get_[1:], oet[1:])):
    c = _row_cos(g, o)
    assert np.percentile(c, 50) >= 0.9999 and np.percentile(c, 1) >= 0.999, \
        (np.percentile(c, 50), np.percentile(c, 1))


def test_c1_hobe_end_to_end_cosine(ctx, tiny_inc):
  """HG2V_ALG_DIST d=16 on youtube_tiny through every device stage: alg-dist
  (k=10, 20 iterations) from the reference's init vs the reference's own
  coordinates; the reference's HOBE pair stream (oracle MT19937 replica with
  the reference's coordinates: 755,267 records, the count measured from the
  reference) whose nn/ee/ne probabilities the device
  recomputes from ITS coordinates; then up to 10 epochs + EarlyStopping
  (MSE / ReLU heads) on the device vs the CPU restatement trained on the
  reference stream, same init and batch order: same epochs, per-row cosine
  p50 >= 0.9999, p1 >= 0.999."""
  from hypergraphembedding_amd import _hgx
  z = golden("algdist_tiny.npz")
  inc = tiny_inc
  r = O.Rng(int(z["seed"]))
  x0, y0 = r.random((inc.N, 10)), r.random((inc.E, 10))
  ctx.upload(inc)
  gx, gy = ctx.alg_dist(x0, y0, 20)  # coordinates stay resident
  assert np.abs(gx - z["x_20"]).max() <= 1e-4
  assert np.abs(gy - z["y_20"]).max() <= 1e-4
  K, S = 5, 200
  idx, tgt = O.hobe_sample(O.Rng(7), inc, z["x_20"], z["y_20"], S, K)
  assert idx.shape[0] == 755_267
  nn = (idx[:, 0] > 0) & (idx[:, 2] > 0)
  ee = (idx[:, 1] > 0) & (idx[:, 3] > 0)
  ne = (idx[:, 0] > 0) & (idx[:, 3] > 0)
  assert (nn.sum(), ee.sum(), ne.sum()) == (718_589, 138, 36_540)
  gt = np.zeros_like(tgt)
  gt[nn, 0] = ctx.hobe_probs(_hgx.HOBE_NN, idx[nn, 0] - 1, idx[nn, 2] - 1)
  gt[ee, 1] = ctx.hobe_probs(_hgx.HOBE_EE, idx[ee, 1] - 1, idx[ee, 3] - 1)
  gt[ne, 2] = ctx.hobe_probs(_hgx.HOBE_NE, idx[ne, 0] - 1, idx[ne, 3] - 1)
  assert np.abs(gt - tgt).max() <= 5e-4  # coordinates agree to 1e-4
  n, d = idx.shape[0], 16
  rs = np.random.RandomState(11)
  perms = np.stack([rs.permutation(n) for _ in range(10)])
  nt = rs.uniform(-0.05, 0.05, (inc.N + 1, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (inc.E + 1, d)).astype(np.float32)
  ont, oet, ol, _, _ = O.train(idx, tgt, K, nt, et, O.LOSS_MSE, O.ACT_RELU,
                               batch=256, max_epochs=10, perms=perms,
                               min_delta=1e-3)
  ctx.records_set(idx, gt)
  ctx.model_init(d, inc.N + 1, inc.E + 1, node_tab=nt, edge_tab=et)
  gl = ctx.train(batch=256, max_epochs=10, loss=_hgx.LOSS_MSE,
                 act=_hgx.ACT_RELU, min_delta=1e-3, perms=perms)
  gnt, get_ = ctx.model_get()
  assert len(gl) == len(ol), (gl, ol)  # EarlyStopping stopped at the same epoch
  np.testing.assert_allclose(gl, ol, rtol=1e-3)
  for g, o in ((gnt[1:], ont[1:]), (get_[1:], oet[1:])):
    c = _row_cos(g, o)
    assert np.percentile(c, 50) >= 0.9999 and np.percentile(c, 1) >= 0.999, \
        (np.percentile(c, 50), np.percentile(c, 1))


def test_c2_fobe_fullsize_counts_and_training(ctx):
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import random_hypergraph
  inc = random_hypergraph(seed=0)
  S, K = 200, 5
  ctx.upload(inc)
  n = ctx.sample_fobe(31, K, np.full(inc.N, S, np.int32),
                      np.full(inc.E, S, np.int32))
  idx, tgt = ctx.records_get()
  assert idx.shape == (n, 4 + 2 * K) and np.all(tgt == 1.0 * (tgt > 0))
  ln, le, rn, re = (idx[:, i] for i in range(4))
  nn = (ln > 0) & (rn > 0)
  ee = (le > 0) & (re > 0)
  ne = (ln > 0) & (re > 0) & (rn == 0)
  assert int(nn.sum() + ee.sum() + ne.sum()) == n
  cnt_nn = np.bincount(ln[nn] - 1, minlength=inc.N)
  cnt_ee = np.bincount(le[ee] - 1, minlength=inc.E)
  # BooleanSamples ne block: node rows (v, e in E(v)) then edge rows
  n_ne_node = int(np.minimum(np.diff(inc.rp_n), S).sum())
  ne_v, ne_e = ln[ne] - 1, re[ne] - 1
  assert int(ne.sum()) == n_ne_node + int(np.minimum(np.diff(inc.rp_e), S).sum())
  cnt_ne_n = np.bincount(ne_v[:n_ne_node], minlength=inc.N)
  rs = np.random.RandomState(0)
  for v in rs.choice(inc.N, 64, replace=False):
    mids = inc.col_n[inc.rp_n[v]:inc.rp_n[v + 1]]
    row = np.unique(np.concatenate([inc.col_e[inc.rp_e[m]:inc.rp_e[m + 1]] for m in mids]))
    assert cnt_nn[v] == min(S, row.size)
    got = rn[nn][ln[nn] - 1 == v] - 1
    assert np.unique(got).size == got.size and np.isin(got, row).all()
    assert cnt_ne_n[v] == min(S, mids.size)
  for e in rs.choice(inc.E, 64, replace=False):
    mids = inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]
    row = np.unique(np.concatenate([inc.col_n[inc.rp_n[m]:inc.rp_n[m + 1]] for m in mids]))
    assert cnt_ee[e] == min(S, row.size)
    got = re[ee][le[ee] - 1 == e] - 1
    assert np.unique(got).size == got.size and np.isin(got, row).all()
  tabs = []
  for _ in range(2):
    ctx.model_init(128, inc.N + 1, inc.E + 1, seed=5)
    ctx.train(batch=256, max_epochs=1, loss=_hgx.LOSS_KLD, act=_hgx.ACT_SIGMOID,
              min_delta=-1e30, shuffle_seed=9)
    tabs.append(ctx.model_get())
  assert np.array_equal(tabs[0][0], tabs[1][0])
  assert np.array_equal(tabs[0][1], tabs[1][1])
  ctx.model_init(128, inc.N + 1, inc.E + 1, seed=5)
  losses = ctx.train(batch=256, max_epochs=3, loss=_hgx.LOSS_KLD,
                     act=_hgx.ACT_SIGMOID, min_delta=-1e30, shuffle_seed=9)
  assert len(losses) == 3 and losses[2] < losses[1] < losses[0]


def _c4_row_slice(n_rows=20_000):
  """Node rows [0, n_rows) of the power-law 10M/5M graph with the edges they
  touch (edge ids compressed in order)."""
  from hypergraphembedding_amd.hypergraph_util import Incidence
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  g = powerlaw_hypergraph(seed=0)
  rp = g.rp_n[:n_rows + 1].copy()
  cols = g.col_n[:rp[-1]]
  eids, c = np.unique(cols, return_inverse=True)
  return Incidence(n_rows, eids.size, rp, c.astype(np.int32))


def test_c5_combiner_on_c4_row_slice(ctx):
  from hypergraphembedding_amd import _hgx
  inc = _c4_row_slice()
  assert inc.edge_size().max() > 1000  # power-law edges survive the slice
  ctx.upload(inc)
  d, S, K = 256, 50, 5
  tabs = []
  # FOBE (KLD / sigmoid) and HOBE (MSE / relu) embeddings, one epoch each
  ctx.sample_fobe(1, K, np.full(inc.N, S, np.int32), np.full(inc.E, S, np.int32))
  ctx.model_init(d, inc.N + 1, inc.E + 1, seed=1)
  ctx.train(batch=256, max_epochs=1, loss=_hgx.LOSS_KLD, act=_hgx.ACT_SIGMOID,
            min_delta=-1e30, shuffle_seed=1)
  tabs.append(ctx.model_get())
  r = O.Rng(3)
  ctx.alg_set(r.random((inc.N, 10)), r.random((inc.E, 10)))
  ctx.alg_run(20)
  ctx.sample_hobe(2, K, S)
  ctx.model_init(d, inc.N + 1, inc.E + 1, seed=2)
  ctx.train(batch=256, max_epochs=1, loss=_hgx.LOSS_MSE, act=_hgx.ACT_RELU,
            min_delta=-1e30, shuffle_seed=2)
  tabs.append(ctx.model_get())
  # _concatenate_embeddings: [FOBE | HOBE] rows idx + 1 (combine_embeddings_util.py:15-24)
  nt = np.concatenate([tabs[0][0][1:], tabs[1][0][1:]], 1)
  et = np.concatenate([tabs[0][1][1:], tabs[1][1][1:]], 1)
  assert nt.shape == (inc.N, 2 * d)
  # samples (_sample_hypergraph, combine_embeddings_util.py:46-67): every
  # incidence labelled 1, then 5 x as many missing (node, edge) pairs
  pos_n = np.repeat(np.arange(inc.N, dtype=np.int32), np.diff(inc.rp_n))
  pos_e = inc.col_n.astype(np.int32)
  rs = np.random.RandomState(4)
  m = 5 * pos_n.size
  neg_n = rs.randint(0, inc.N, 2 * m).astype(np.int32)
  neg_e = rs.randint(0, inc.E, 2 * m).astype(np.int32)
  inc_key = np.sort(pos_n.astype(np.int64) * inc.E + pos_e)
  cand = neg_n.astype(np.int64) * inc.E + neg_e
  pos = np.minimum(np.searchsorted(inc_key, cand), inc_key.size - 1)
  keep = inc_key[pos] != cand
  neg_n, neg_e = neg_n[keep][:m], neg_e[keep][:m]
  node_row = np.concatenate([pos_n, neg_n])
  edge_row = np.concatenate([pos_e, neg_e])
  label = np.concatenate([np.ones(pos_n.size, np.float32),
                          np.zeros(neg_n.size, np.float32)])
  # (1) bit-exact vs the CPU restatement on a sample of those samples
  sel = rs.choice(label.size, 1200, replace=False)
  mlp = _hgx.Mlp(ctx, _hgx.MLP_NE_SUPERVISED, 2 * d, d)
  lims = [np.sqrt(6.0 / (k + n)) for k, n in mlp.shapes]
  w0 = np.concatenate([np.concatenate([rs.uniform(-l, l, k * n), np.zeros(n)])
                       for l, (k, n) in zip(lims, mlp.shapes)]).astype(np.float32)
  mlp.set_weights(w0)
  mlp.set_tables(nt, et)
  mlp.set_samples(node_row[sel], edge_row[sel], label[sel])
  perms = rs.permutation(sel.size)[None, :]
  mlp.fit(batch=256, max_epochs=1, min_delta=-1e30, seed=7, perms=perms)
  wc, _ = O.mlp_fit(_hgx.MLP_NE_SUPERVISED, 2 * d, d, w0, nt, et, node_row[sel],
                    edge_row[sel], label[sel], perms, batch=256, min_delta=-1e30,
                    seed=7)
  assert np.abs(mlp.get_weights() - wc).max() == 0.0
  # (2) two epochs over all of the slice's samples on the device
  mlp.set_weights(w0)
  mlp.set_samples(node_row, edge_row, label)
  losses = mlp.fit(batch=256, max_epochs=2, min_delta=-1e30, seed=8)
  assert label.size > 2_000_000 and len(losses) == 2
  # MSE of a sigmoid label head on 1/6 positives: finite, inside [0, 0.25]
  assert np.all(np.isfinite(losses)) and np.all((losses >= 0) & (losses <= 0.25))
  jn = mlp.predict(1, np.arange(inc.N, dtype=np.int32), None)
  assert jn.shape == (inc.N, d) and np.isfinite(jn).all()
  mlp.close()
