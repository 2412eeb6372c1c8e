"""Streaming the record stream in chunks (SURVEY §5 "stream samples in
chunks"; the reference materialises every record, embedding.py:277-284):
model state carries across one-epoch hgx_train calls, so an epoch split into
resident chunks is the same computation as the unchunked epoch; the record
store's epochs (tests/test_gpu_store.py) train the same records as a
resident stream, to the same quality."""

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
  from hypergraphembedding_amd import _hgx
  c = _hgx.Context(0)
  yield c
  c.close()


def test_chunked_epoch_equals_unchunked_bitwise(ctx):
  """C3 (random 100k/50k, HOBE d=128): one epoch over the whole resident
  stream in permutation P vs the same epoch as three resident chunks
  (consecutive slices of P, sizes multiples of the batch): identical tables
  bit for bit, and the chunk loss sums add up to the epoch's."""
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import random_hypergraph
  inc = random_hypergraph(seed=0)
  ctx.upload(inc)
  r = O.Rng(4)
  ctx.alg_set(r.random((inc.N, 10)), r.random((inc.E, 10)))
  ctx.alg_run(20)
  n = ctx.sample_hobe(17, 5, 200)
  idx, tgt = ctx.records_get()
  P = np.random.RandomState(5).permutation(n)
  kw = dict(batch=256, max_epochs=1, loss=_hgx.LOSS_MSE, act=_hgx.ACT_RELU,
            min_delta=-1e30)
  ctx.model_init(128, inc.N + 1, inc.E + 1, seed=21)
  ctx.train(perms=P[None, :], **kw)
  full = ctx.model_get()
  full_loss = ctx.train_loss_sum()
  cuts = [0, 256 * 40_000, 256 * 150_000, n]
  ctx.model_init(128, inc.N + 1, inc.E + 1, seed=21)
  lsum = 0.0
  for lo, hi in zip(cuts, cuts[1:]):
    sel = P[lo:hi]
    ctx.records_set(idx[sel], tgt[sel])
    ctx.train(perms=np.arange(hi - lo)[None, :], **kw)
    lsum += ctx.train_loss_sum()
  chunked = ctx.model_get()
  assert np.array_equal(full[0], chunked[0])
  assert np.array_equal(full[1], chunked[1])
  assert abs(lsum - full_loss) <= 1e-9 * abs(full_loss)


def _holdout(inc, frac, rs):
  """A random `frac` of the incidences removed (never a node's or an
  edge's last one): (train Incidence, removed (v, e), as many missing
  (v, e))."""
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.hypergraph_util import Incidence
  rows = np.repeat(np.arange(inc.N), np.diff(inc.rp_n))
  deg = np.diff(inc.rp_n).copy()
  size = np.diff(inc.rp_e).copy()
  keep = np.ones(inc.nnz, bool)
  for t in rs.permutation(inc.nnz)[:int(frac * inc.nnz)]:
    v, e = rows[t], inc.col_n[t]
    if deg[v] > 1 and size[e] > 1:
      keep[t] = False
      deg[v] -= 1
      size[e] -= 1
  rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
  col = inc.col_n[keep].astype(np.int32)
  rp_e, col_e = _hgx.csr_transpose(inc.N, inc.E, rp, col)
  train = Incidence(inc.N, inc.E, rp, col, rp_e, col_e)
  pos = (rows[~keep], inc.col_n[~keep])
  key = rows.astype(np.int64) * inc.E + inc.col_n
  cv = rs.randint(0, inc.N, 3 * pos[0].size)
  ce = rs.randint(0, inc.E, 3 * pos[0].size)
  miss = ~np.isin(cv.astype(np.int64) * inc.E + ce, key)
  neg = (cv[miss][:pos[0].size], ce[miss][:pos[0].size])
  return train, pos, neg


def _lp_accuracy(inc, nt, et, pos, neg, rs):
  """LP_NODE_EDGE_CLASSIFIER (evaluation_util.py:471-552) on arrays: the
  dense classifier trained on 200k training incidences and as many missing
  pairs, accuracy over the held-out incidences and as many missing pairs."""
  from hypergraphembedding_amd.dense_mlp import LP_CLASSIFIER, DenseModel
  rows = np.repeat(np.arange(inc.N), np.diff(inc.rp_n))
  pick = rs.choice(inc.nnz, 200_000, replace=False)
  key = rows.astype(np.int64) * inc.E + inc.col_n
  cv = rs.randint(0, inc.N, 300_000)
  ce = rs.randint(0, inc.E, 300_000)
  miss = ~np.isin(cv.astype(np.int64) * inc.E + ce, key)
  nr = np.concatenate([rows[pick], cv[miss][:200_000]]).astype(np.int32)
  er = np.concatenate([inc.col_n[pick], ce[miss][:200_000]]).astype(np.int32)
  lab = np.concatenate([np.ones(200_000), np.zeros(nr.size - 200_000)])
  m = DenseModel(LP_CLASSIFIER, nt.shape[1])
  m.set_tables(nt, et)
  m.fit(nr, er, lab.astype(np.float32), epochs=10, min_delta=1e-3)
  yp = m.predict_label(pos[0].astype(np.int32), pos[1].astype(np.int32)).ravel()
  yn = m.predict_label(neg[0].astype(np.int32), neg[1].astype(np.int32)).ravel()
  m.close()
  return float(((yp > 0.5).sum() + (yn <= 0.5).sum()) / (yp.size + yn.size))


@pytest.mark.timeout(900)
def test_store_streaming_matches_resident_training(ctx):
  """the record stream sampled in >= 4 strided row
  classes into the record store and trained in chunks of a quarter of the
  stream with the store's global shuffle (Hg2vModel.fit_store) vs resident
  with the device's global shuffle, on a 200k/100k power-law graph (edges
  numbered by popularity), three seeds, 8 epochs, the same records: mean
  final training loss within 1.25x and link-prediction accuracy within
  0.005 of resident (r04's windowed shuffle: 2.3x the loss, -0.014
  accuracy, profiles/r04/streaming/quality.log)."""
  from hypergraphembedding_amd import _hgx, embedding
  from hypergraphembedding_amd.hg2v_model import Hg2vModel
  from hypergraphembedding_amd.hg2v_sample import row_class_quota
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  full = powerlaw_hypergraph(N=200_000, E=100_000, mean_degree=8, seed=3)
  train, pos, neg = _holdout(full, 0.05, np.random.RandomState(0))
  S, K, d, EP = 50, 5, 32, 8
  ctx.upload(train)
  r = np.random.RandomState(1)
  ctx.alg_set(r.random_sample((train.N, 10)), r.random_sample((train.E, 10)))
  ctx.alg_run(20)
  n_all = ctx.sample_hobe(5, K, S)
  bn = np.full(train.N, 2 * S, np.int64)
  be = np.full(train.E, 2 * S, np.int64)
  budget = n_all // 4
  chunks = embedding._row_chunks(bn, be, budget)
  assert len(chunks) >= 4
  full_q = (np.full(train.N, S, np.int32), np.full(train.E, S, np.int32))
  res = {"resident": [], "store": []}
  for seed in range(3):
    for mode in res:
      m = Hg2vModel(train.N + 1, train.E + 1, d, K, _hgx.LOSS_MSE,
                    _hgx.ACT_RELU, ctx=ctx, seed=100 + seed)
      if mode == "resident":
        assert ctx.sample_hobe(1000 + seed, K, S) == n_all
        losses = m.fit(epochs=EP, min_delta=-1e30, shuffle_seed=7 + seed)
      else:
        stored = embedding.fill_store(
            ctx, train, lambda off, st: ctx.sample_hobe(
                1000 + seed, K, S, *(row_class_quota(q, off, st) for q in full_q)),
            bn, be, budget)
        assert stored == n_all
        losses = m.fit_store(budget, epochs=EP, min_delta=-1e30, seed=7 + seed)
        assert m.records_per_epoch == n_all
        assert len(m.chunk_stats) >= 4 * EP
      nt, et = m.get_weights()
      acc = _lp_accuracy(train, nt[1:], et[1:], pos, neg,
                         np.random.RandomState(50 + seed))
      res[mode].append((float(losses[-1]), acc))
      print(mode, seed, "losses", np.round(losses, 5).tolist(), "LP", round(acc, 4))
  for mode, v in res.items():
    print(mode, "final losses", [round(x[0], 5) for x in v],
          "LP accuracy", [round(x[1], 4) for x in v])
  loss = lambda mode: np.array([x[0] for x in res[mode]])
  acc = lambda mode: np.mean([x[1] for x in res[mode]])
  assert loss("store").mean() <= 1.25 * loss("resident").mean()
  assert abs(acc("store") - acc("resident")) <= 0.005
  assert acc("resident") > 0.55  # the embedding carries link information
