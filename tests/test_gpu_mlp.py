"""GPU parity of the dense MLP engine (hgx_mlp_*, csrc/hgx_mlp.hip) against
the CPU restatement (oracle/mlpref.c) on identical weights, samples, batch
order and dropout masks: the classifier of evaluation_util.py:471-505 and
the two combiners of combine_embeddings_util.py:80-174.

Bar: the trained weights and the predictions are BIT-EXACT. The restatement
runs every dot product in the device's reduction order (4 wave chains of
exact f32 fma steps, combined in a fixed order), the sigmoid uses the same
fma-written exp on both sides and Adagrad uses correctly rounded operations,
so nothing is left to a tolerance except the reported epoch loss (the
device sums loss partials per tile: relative 1e-5)."""

import numpy as np
import pytest

import oracle as O
from hypergraphembedding_amd import _hgx

pytestmark = pytest.mark.gpu


def glorot(shapes, rng, bias_scale=0.0):
  parts = []
  for k, n in shapes:
    lim = np.sqrt(6.0 / (k + n))
    parts += [rng.uniform(-lim, lim, k * n), rng.normal(0, bias_scale, n)]
  return np.concatenate(parts).astype(np.float32)


def make_case(kind, I, D, n, seed, rows=(300, 150)):
  rng = np.random.default_rng(seed)
  nt = rng.random((rows[0], I)).astype(np.float32)
  et = rng.random((rows[1], I)).astype(np.float32)
  nr = rng.integers(0, rows[0], n).astype(np.int32)
  er = rng.integers(0, rows[1], n).astype(np.int32)
  lab = (rng.random(n) < 1 / 6).astype(np.float32)
  return rng, nt, et, nr, er, lab


@pytest.fixture(scope="module")
def ctx():
  c = _hgx.Context(0)
  yield c
  c.close()


def run_both(ctx, kind, I, D, n, epochs, seed=3, bias_scale=0.1, batch=256):
  rng, nt, et, nr, er, lab = make_case(kind, I, D, n, seed)
  m = _hgx.Mlp(ctx, kind, I, D)
  w0 = glorot(m.shapes, rng, bias_scale)
  assert w0.size == O.mlp_num_weights(kind, I, D)
  m.set_weights(w0)
  np.testing.assert_array_equal(m.get_weights(), w0)
  m.set_tables(nt, et)
  m.set_samples(nr, er, lab)
  perms = np.stack([rng.permutation(n) for _ in range(epochs)])
  dseed = 77
  gl = m.fit(batch=batch, max_epochs=epochs, min_delta=-1e30, seed=dseed,
             perms=perms)
  wg = m.get_weights()
  wc, cl = O.mlp_fit(kind, I, D, w0, nt, et, nr, er, lab, perms, batch=batch,
                     min_delta=-1e30, seed=dseed)
  return m, (nt, et, nr, er), wg, wc, gl, cl


@pytest.mark.parametrize("kind,I,D", [(0, 40, 0), (1, 40, 24), (2, 40, 24),
                                      (0, 19, 0), (1, 70, 33)])
def test_fit_bit_exact(ctx, kind, I, D):
  m, (nt, et, nr, er), wg, wc, gl, cl = run_both(ctx, kind, I, D, 1500, 2)
  assert len(gl) == len(cl) == 2
  np.testing.assert_allclose(gl, cl, rtol=1e-5)
  diff = np.abs(wg - wc)
  assert diff.max() == 0.0, (diff.max(), int((diff > 0).sum()))
  # inference: label head and joint embeddings
  yg = m.predict(0, nr[:700], er[:700])
  yc = O.mlp_predict(kind, I, D, wc, nt, et, 0, nr[:700], er[:700])
  np.testing.assert_array_equal(yg, yc)
  if kind != 0:
    for out, rows in ((1, np.arange(nt.shape[0])), (2, np.arange(et.shape[0]))):
      jg = m.predict(out, rows if out == 1 else None, rows if out == 2 else None)
      jc = O.mlp_predict(kind, I, D, wc, nt, et, out,
                         rows if out == 1 else None, rows if out == 2 else None)
      np.testing.assert_array_equal(jg, jc)
  m.close()


def test_fit_bit_exact_c5_widths(ctx):
  """The C5 combiner shape: two 256-d embeddings (in 512) -> 256."""
  m, _, wg, wc, gl, cl = run_both(ctx, 1, 512, 256, 600, 1)
  assert np.abs(wg - wc).max() == 0.0
  np.testing.assert_allclose(gl, cl, rtol=1e-5)
  m.close()


@pytest.mark.parametrize("kind,I,D", [(1, 40, 24), (2, 40, 24), (1, 512, 256)])
def test_fused_head_equals_head_launch(ctx, kind, I, D):
  """Combiner training computes the label head inside the launch that forms
  the joint layers' deltas (tuning mlp_fuse_head, default 1) instead of in
  its own launch: the trained weights and epoch losses are bit for bit those
  of the separate head launch (and both equal oracle/mlpref.c above)."""
  rng, nt, et, nr, er, lab = make_case(kind, I, D, 700, 5)
  w0 = None
  res = []
  for fuse in (1, 0):
    ctx.set_tuning("mlp_fuse_head", fuse)
    try:
      m = _hgx.Mlp(ctx, kind, I, D)
      if w0 is None:
        w0 = glorot(m.shapes, np.random.default_rng(2), 0.1)
      m.set_weights(w0)
      m.set_tables(nt, et)
      m.set_samples(nr, er, lab)
      losses = m.fit(max_epochs=2, min_delta=-1e30, seed=4)
      res.append((m.get_weights(), np.asarray(losses)))
      m.close()
    finally:
      ctx.set_tuning("mlp_fuse_head", 1)
  np.testing.assert_array_equal(res[0][0], res[1][0])
  np.testing.assert_array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("kind,I,D,batch", [(1, 40, 24, 256), (2, 70, 33, 100),
                                            (1, 512, 256, 256), (2, 19, 7, 64)])
def test_prefetch_equals_gather(ctx, kind, I, D, batch):
  """Combiner training gathers batch b + 1's dropped-out input rows inside
  batch b's hidden-layer launch (tuning mlp_prefetch, default 1; 2: in the
  joint layers' launch); the first layer and its weight gradient then read
  them densely. Trained weights and epoch losses are bit for bit those of
  gathering in place (ragged last batch included: 900 samples)."""
  rng, nt, et, nr, er, lab = make_case(kind, I, D, 900, 6)
  w0 = None
  res = []
  for pf in (1, 2, 0):
    ctx.set_tuning("mlp_prefetch", pf)
    try:
      m = _hgx.Mlp(ctx, kind, I, D)
      if w0 is None:
        w0 = glorot(m.shapes, np.random.default_rng(3), 0.1)
      m.set_weights(w0)
      m.set_tables(nt, et)
      m.set_samples(nr, er, lab)
      losses = m.fit(batch=batch, max_epochs=2, min_delta=-1e30, seed=9)
      res.append((m.get_weights(), np.asarray(losses)))
      m.close()
    finally:
      ctx.set_tuning("mlp_prefetch", 1)
  for r in res[1:]:
    np.testing.assert_array_equal(res[0][0], r[0])
    np.testing.assert_array_equal(res[0][1], r[1])


def test_small_batches_and_single_sample(ctx):
  m, _, wg, wc, gl, cl = run_both(ctx, 2, 20, 12, 301, 1, batch=100)
  assert np.abs(wg - wc).max() == 0.0
  m.close()
  m, _, wg, wc, gl, cl = run_both(ctx, 0, 8, 0, 1, 3)
  assert np.abs(wg - wc).max() == 0.0
  m.close()


def test_device_shuffle_deterministic_and_learns(ctx):
  rng, nt, et, nr, er, _ = make_case(0, 16, 0, 4000, 11)
  # a learnable label: node row parity
  lab = (nr % 2).astype(np.float32)
  nt[:, 0] = (np.arange(nt.shape[0]) % 2)
  outs = []
  for _ in range(2):
    m = _hgx.Mlp(ctx, 0, 16)
    m.set_weights(glorot(m.shapes, np.random.default_rng(5)))
    m.set_tables(nt, et)
    m.set_samples(nr, er, lab)
    losses = m.fit(max_epochs=30, min_delta=1e-3, seed=9)
    outs.append((m.get_weights(), losses))
    st = m.stats()
    assert st["samples"] == 4000 * len(losses) and st["ms"] > 0
    m.close()
  np.testing.assert_array_equal(outs[0][0], outs[1][0])
  losses = outs[0][1]
  assert losses[-1] < losses[0]
  # EarlyStopping(min_delta=1e-3, patience=0): all but the last improved
  best = np.minimum.accumulate(losses)
  for e in range(1, len(losses) - 1):
    assert losses[e] + 1e-3 < best[e - 1]


def test_combiner_learns_planted_label(ctx):
  """The N_E_SUPERVISED combiner (kind 1: two towers, joint sigmoid layers,
  relu + sigmoid head; combine_embeddings_util.py:96-157) on a planted,
  learnable label (node feature 0 x edge feature 0 > 0.3, 17% positives):
  the epoch loss falls well below the constant predictor's MSE p(1 - p)
  and the device run equals oracle/mlpref.c bit for bit. (At in = 512 /
  d = 256 on random labels the head saturates instead: Keras-zero-init
  Adagrad's first step is lr * sign(g) on every weight, which drives the
  sigmoid to ~5e-9 within two batches -- tools/perf_c5_mlp.py's flat
  0.1667 loss is that, in the CPU restatement too.)"""
  rs = np.random.RandomState(0)
  ind, d, N, E, n = 16, 8, 2000, 1000, 30000
  nt = rs.uniform(-1, 1, (N, ind)).astype(np.float32)
  et = rs.uniform(-1, 1, (E, ind)).astype(np.float32)
  nr = rs.randint(0, N, n).astype(np.int32)
  er = rs.randint(0, E, n).astype(np.int32)
  lab = ((nt[nr, 0] * et[er, 0]) > 0.3).astype(np.float32)
  p = float(lab.mean())
  m = _hgx.Mlp(ctx, _hgx.MLP_NE_SUPERVISED, ind, d)
  w0 = glorot(m.shapes, np.random.default_rng(3))
  m.set_weights(w0)
  m.set_tables(nt, et)
  m.set_samples(nr, er, lab)
  epochs = 15
  perms = np.stack([rs.permutation(n) for _ in range(epochs)])
  losses = m.fit(max_epochs=epochs, min_delta=-1e30, seed=4, perms=perms)
  wc, lc = O.mlp_fit(_hgx.MLP_NE_SUPERVISED, ind, d, w0, nt, et, nr, er, lab,
                     perms, batch=256, min_delta=-1e30, seed=4)
  assert np.array_equal(m.get_weights(), wc)
  np.testing.assert_allclose(losses, lc, rtol=1e-5)
  assert len(losses) == epochs and losses[-1] < p * (1 - p) - 0.008, losses
  assert losses[-1] < losses[2] < losses[0]
  m.close()


def test_errors(ctx):
  with pytest.raises(AssertionError):
    _hgx.Mlp(ctx, 1, 16, 0)  # desired_dim > 0
  m = _hgx.Mlp(ctx, 0, 8)
  with pytest.raises(_hgx.HgxError):
    m.set_samples(np.zeros(3), np.zeros(3), np.zeros(3))  # tables first
  m.set_tables(np.zeros((4, 8)), np.zeros((2, 8)))
  with pytest.raises(AssertionError):
    m.set_samples(np.array([0, 4]), np.array([0, 1]), np.zeros(2))
  with pytest.raises(AssertionError):
    m.predict(1, np.arange(3))  # the classifier has no joint output
  m.close()
