"""Streaming the record stream in chunks (SURVEY §5 "stream samples in
chunks"; the reference materialises every record, embedding.py:277-284):
model state carries across one-epoch hgx_train calls, so an epoch split into
resident chunks is the same computation as the unchunked epoch."""

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


def test_fit_streaming_embed_hobe_chunks(ctx):
  """EmbedHg2vAlgDist with a record budget below the stream size takes the
  streaming path (row-range chunks sampled and trained in turn): every
  record of the single-process stream is trained once per epoch, the loss
  decreases, and the embedding covers every node and edge."""
  from conftest import golden_incidence
  from hypergraphembedding_amd import embedding, _hgx
  from hypergraphembedding_amd.hg2v_model import Hg2vModel
  from hypergraphembedding_amd.runtime import get_context
  inc = golden_incidence("csr_small.npz")
  np.random.seed(3)
  emb = embedding.EmbedHg2vAlgDist(inc, 8, num_samples=20, epochs=3,
                                   records_budget=5000)
  assert emb.dim == 8 and emb.method_name == "HG2V_ALG_DIST"
  assert len(emb.node) == inc.N and len(emb.edge) == inc.E
  assert all(len(v.values) == 8 for v in emb.node.values())
  # the streaming fit itself: chunks cover the stream, loss goes down
  c = get_context()
  c.upload(inc)
  r = O.Rng(1)
  c.alg_set(r.random((inc.N, 10)), r.random((inc.E, 10)))
  c.alg_run(20)
  n_all = c.sample_hobe(9, 5, 20)
  chunks = embedding._row_chunks(inc, 40, 2000)
  assert len(chunks) >= 3

  def make(ci):
    (n0, n1), (e0, e1) = chunks[ci]
    nq = np.zeros(inc.N, np.int32)
    eq = np.zeros(inc.E, np.int32)
    nq[n0:n1] = 20
    eq[e0:e1] = 20
    return c.sample_hobe(9, 5, 20, node_q=nq, edge_q=eq)

  m = Hg2vModel(inc.N + 1, inc.E + 1, 16, 5, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                ctx=c, seed=2)
  losses = m.fit_streaming(make, len(chunks), epochs=4, min_delta=-1e30,
                           seed=0)
  assert m.records_per_epoch == n_all
  assert len(losses) == 4 and losses[-1] < losses[0]
