"""GPU parity: the Keras-semantics Adagrad trainer vs the CPU oracle.

Same record stream (reference-generated golden records), same initial
tables, same per-epoch batch order (host permutations). The trainer is
"parity unpinned" against Keras itself (keras/tensorflow are absent), so the
oracle here is the restatement in oracle/hgref.c (hgref_train).

Tolerance: per-row cosine p50 >= 0.9999 and p1 >= 0.999 after
training, plus epoch losses within 1e-4 relative; fp32 summation order is
the only difference, so the observed agreement is far tighter.
"""

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


def _row_cos(a, b):
  a = a.astype(np.float64)
  b = b.astype(np.float64)
  num = (a * b).sum(1)
  den = np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1)
  ok = den > 0
  return num[ok] / den[ok]


def _run_both(ctx, idx, tgt, K, d, loss, act, batch, epochs, seed=0,
              min_delta=1e-3):
  rs = np.random.RandomState(seed)
  nrows = int(idx[:, [0, 2] + list(range(4, 4 + K))].max()) + 2
  erows = int(idx[:, [1, 3] + list(range(4 + K, 4 + 2 * K))].max()) + 2
  nt = rs.uniform(-0.05, 0.05, (nrows, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (erows, d)).astype(np.float32)
  perms = np.stack([rs.permutation(idx.shape[0]) for _ in range(epochs)])
  ont, oet, olosses, _, _ = O.train(idx, tgt, K, nt, et, loss, act,
                                    batch=batch, max_epochs=epochs, perms=perms,
                                    min_delta=min_delta)
  ctx.records_set(idx, tgt)
  ctx.model_init(d, nrows, erows, node_tab=nt, edge_tab=et)
  glosses = ctx.train(batch=batch, max_epochs=epochs, loss=loss, act=act,
                      perms=perms, min_delta=min_delta)
  gnt, get_ = ctx.model_get()
  return (ont, oet, olosses), (gnt, get_, glosses), (nt, et)


@pytest.fixture(params=[(32, 0), (64, 0), (64, 512)],
                ids=["lanes32", "lanes64", "lanes64-tb512"])
def lanes(ctx, request):
  """The fused step's geometry at padded d = 128: float4 x 32 lanes or float2
  x 64 lanes per record (tunings train_lanes / train_tb; d = 256 ignores the
  lanes, takes its 256-thread form)."""
  ctx.set_tuning("train_lanes", request.param[0])
  ctx.set_tuning("train_tb", request.param[1])
  yield request.param
  ctx.set_tuning("train_lanes", 0)
  ctx.set_tuning("train_tb", 0)


def _check(o, g, init):
  ont, oet, ol = o
  gnt, get_, gl = g
  assert ol.shape == gl.shape, (ol, gl)
  assert np.allclose(gl, ol, rtol=1e-4, atol=1e-7), (gl, ol)
  for a, b, i in ((gnt, ont, init[0]), (get_, oet, init[1])):
    c = _row_cos(a, b)
    assert np.percentile(c, 50) >= 0.9999
    assert np.percentile(c, 1) >= 0.999
    # the update actually happened
    assert not np.array_equal(a, i)


@pytest.mark.parametrize("d,batch", [(8, 64), (16, 256), (128, 256), (5, 37)])
def test_train_hobe_records_vs_oracle(ctx, d, batch, lanes):
  z = golden("hobe_small.npz")
  o, g, init = _run_both(ctx, z["idx"], z["tgt"], int(z["K"]), d, O.LOSS_MSE,
                         O.ACT_RELU, batch, epochs=3)
  _check(o, g, init)


@pytest.mark.parametrize("d,batch", [(16, 256), (128, 256), (256, 100), (2, 1)])
def test_train_fobe_records_vs_oracle(ctx, d, batch, lanes):
  """BooleanModel (KLD + sigmoid) on the reference's FOBE stream with
  negatives, every step geometry: d = 128 (C2's instantiation) as float4 x
  32 lanes and float2 x 64 lanes (256- and 512-thread workgroups)."""
  z = golden("fobe_small_ns.npz")
  idx, tgt = z["idx"], z["tgt"]
  if batch == 1:  # the reference test's batch_size=1 (test_embedding.py:193)
    idx, tgt = idx[:300], tgt[:300]
  o, g, init = _run_both(ctx, idx, tgt, int(z["K"]), d, O.LOSS_KLD,
                         O.ACT_SIGMOID, batch, epochs=2)
  _check(o, g, init)


def test_train_k5_synthetic_with_duplicates(ctx):
  """K=5 (the default), heavy row reuse inside a batch, last batch ragged."""
  rs = np.random.RandomState(7)
  n, K = 3000, 5
  idx = np.zeros((n, 4 + 2 * K), np.int32)
  kind = rs.randint(0, 3, n)
  idx[kind == 0, 0] = rs.randint(1, 30, (kind == 0).sum())
  idx[kind == 0, 2] = rs.randint(1, 30, (kind == 0).sum())
  idx[kind == 1, 1] = rs.randint(1, 12, (kind == 1).sum())
  idx[kind == 1, 3] = rs.randint(1, 12, (kind == 1).sum())
  m = kind == 2
  idx[m, 0] = rs.randint(1, 30, m.sum())
  idx[m, 3] = rs.randint(1, 12, m.sum())
  idx[m, 4:4 + K] = rs.randint(1, 30, (m.sum(), K))
  idx[m, 4 + K:] = rs.randint(1, 12, (m.sum(), K))
  tgt = np.zeros((n, 3), np.float32)
  tgt[np.arange(n), kind] = rs.uniform(0, 1, n).astype(np.float32)
  o, g, init = _run_both(ctx, idx, tgt, K, 32, O.LOSS_MSE, O.ACT_RELU, 256,
                         epochs=2)
  _check(o, g, init)


def test_train_early_stopping_and_device_shuffle(ctx):
  z = golden("hobe_small.npz")
  K = int(z["K"])
  ctx.records_set(z["idx"], z["tgt"])
  ctx.model_init(16, 200, 100, seed=5)
  losses = ctx.train(batch=64, max_epochs=10, loss=O.LOSS_MSE, act=O.ACT_RELU,
                     shuffle_seed=3, min_delta=1e9)
  # min_delta huge: epoch 1 improves on inf, epoch 2 cannot -> stop (Keras
  # EarlyStopping with patience=0)
  assert losses.size == 2
  losses = ctx.train(batch=64, max_epochs=4, loss=O.LOSS_MSE, act=O.ACT_RELU,
                     shuffle_seed=4, min_delta=-1.0)
  assert losses.size == 4
  ms, rec, bat = ctx.train_stats()
  assert rec == 4 * z["idx"].shape[0] and ms > 0
  del K


def test_train_rejects_out_of_range_rows(ctx):
  z = golden("hobe_small.npz")
  ctx.records_set(z["idx"], z["tgt"])
  ctx.model_init(8, 3, 3, seed=1)  # far too few rows
  with pytest.raises(AssertionError):
    ctx.train(batch=64, max_epochs=1)


def _mixed_reuse_records(rs, nb, B, K, hub_batches, wide=20000):
  """Records in batch order: batches in hub_batches draw every id from a
  handful of rows (records sharing rows across more than one workgroup: the
  batch cannot be packed and takes the two-kernel step), the others from a
  wide range (packable)."""
  n = nb * B
  idx = np.zeros((n, 4 + 2 * K), np.int32)
  kind = rs.randint(0, 3, n)
  for b in range(nb):
    lo, hi = (1, 6) if b in hub_batches else (1, wide)
    sl = slice(b * B, (b + 1) * B)
    kb = kind[sl]
    blk = idx[sl]
    m0, m1, m2 = kb == 0, kb == 1, kb == 2
    blk[m0, 0] = rs.randint(lo, hi, m0.sum())
    blk[m0, 2] = rs.randint(lo, hi, m0.sum())
    blk[m1, 1] = rs.randint(lo, hi, m1.sum())
    blk[m1, 3] = rs.randint(lo, hi, m1.sum())
    blk[m2, 0] = rs.randint(lo, hi, m2.sum())
    blk[m2, 3] = rs.randint(lo, hi, m2.sum())
    blk[m2, 4:4 + K] = rs.randint(lo, hi, (m2.sum(), K))
    blk[m2, 4 + K:] = rs.randint(lo, hi, (m2.sum(), K))
  tgt = np.zeros((n, 3), np.float32)
  tgt[np.arange(n), kind] = rs.uniform(0, 1, n).astype(np.float32)
  return idx, tgt


@pytest.mark.parametrize("d,loss,act", [(128, O.LOSS_MSE, O.ACT_RELU),
                                        (256, O.LOSS_KLD, O.ACT_SIGMOID)])
def test_fused_step_mixed_runs_vs_oracle_and_split(ctx, d, loss, act, lanes):
  """The one-launch deferred-row step (train_step) against the oracle and
  the two-kernel step. Hub batches (every id from 5 rows) make nearly every
  row of the batch a deferred row; consecutive hub batches chain them
  (pending slots, several per record); the wide batch after a hub batch
  flushes the hub rows it does not touch; a ragged last batch too."""
  rs = np.random.RandomState(11)
  K, B, nb = 5, 256, 12
  idx, tgt = _mixed_reuse_records(rs, nb, B, K, hub_batches={3, 4, 8})
  idx, tgt = idx[:-57], tgt[:-57]  # ragged last batch
  # in-order batches: the hub batches stay where they were put
  perms = np.arange(idx.shape[0])[None, :]
  nrows = int(idx[:, [0, 2] + list(range(4, 4 + K))].max()) + 2
  erows = int(idx[:, [1, 3] + list(range(4 + K, 4 + 2 * K))].max()) + 2
  nt = rs.uniform(-0.05, 0.05, (nrows, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (erows, d)).astype(np.float32)
  ont, oet, ol, _, _ = O.train(idx, tgt, K, nt, et, loss, act, batch=B,
                               max_epochs=1, perms=perms)
  ctx.records_set(idx, tgt)
  res = {}
  try:
    for mode in ("2", "0"):
      ctx.set_tuning("train_fused", 1 if mode == "2" else 0)
      ctx.model_init(d, nrows, erows, node_tab=nt, edge_tab=et)
      gl = ctx.train(batch=B, max_epochs=1, loss=loss, act=act, perms=perms)
      res[mode] = ctx.model_get() + (gl, ctx.train_path_stats())
  finally:
    ctx.set_tuning("train_fused", 1)
  fused, split = res["2"][3], res["0"][3]
  assert fused == (nb, 0), fused
  assert split == (0, nb), split
  for mode in ("2", "0"):
    gnt, get_, gl, _ = res[mode]
    assert np.allclose(gl, ol, rtol=1e-4, atol=1e-7), (mode, gl, ol)
    assert np.abs(gnt - ont).max() < 1e-5 and np.abs(get_ - oet).max() < 1e-5
  # the two device paths differ only in how the gradients of a row's slots
  # are summed (2^44 fixed point vs sequential fp32)
  for a, b in zip(res["2"][:2], res["0"][:2]):
    assert np.abs(a - b).max() < 1e-6


def test_fused_step_bitwise_deterministic(ctx, lanes):
  rs = np.random.RandomState(3)
  idx, tgt = _mixed_reuse_records(rs, 20, 256, 5, hub_batches=set())
  ctx.records_set(idx, tgt)
  out = []
  for _ in range(2):
    ctx.model_init(128, 20002, 20002, seed=9)
    ctx.train(batch=256, max_epochs=2, loss=O.LOSS_MSE, act=O.ACT_RELU,
              shuffle_seed=5, min_delta=-1.0)
    assert ctx.train_path_stats()[0] >= 36
    out.append(ctx.model_get())
  assert np.array_equal(out[0][0], out[1][0])
  assert np.array_equal(out[0][1], out[1][1])


def test_step_flush_overflow_and_pending_chains_vs_oracle(ctx, lanes):
  """Batch 0: 128 ne records with distinct rows, each twice (1536 rows with
  exactly two slots: all deferred); batch 1 touches none of them, so it
  flushes more rows than its 4 flush slots per record hold (the overflow
  list). Then hub batches back to back (every slot of a record pending, the
  slot-by-slot fold), a wide batch, and a ragged 3-record last batch after a
  hub batch. Against the oracle, in order, FOBE and HOBE heads."""
  rs = np.random.RandomState(21)
  K, B, d = 5, 256, 128
  R = 4 + 2 * K

  def batch(lo, hi, n=B):
    idx = np.zeros((n, R), np.int32)
    kind = rs.randint(0, 3, n)
    m0, m1, m2 = kind == 0, kind == 1, kind == 2
    idx[m0, 0] = rs.randint(lo, hi, m0.sum())
    idx[m0, 2] = rs.randint(lo, hi, m0.sum())
    idx[m1, 1] = rs.randint(lo, hi, m1.sum())
    idx[m1, 3] = rs.randint(lo, hi, m1.sum())
    idx[m2, 0] = rs.randint(lo, hi, m2.sum())
    idx[m2, 3] = rs.randint(lo, hi, m2.sum())
    idx[m2, 4:4 + K] = rs.randint(lo, hi, (m2.sum(), K))
    idx[m2, 4 + K:] = rs.randint(lo, hi, (m2.sum(), K))
    tgt = np.zeros((n, 3), np.float32)
    tgt[np.arange(n), kind] = rs.uniform(0, 1, n).astype(np.float32)
    return idx, tgt

  # batch 0: ne records, distinct node ids (ln + list) and edge ids (re +
  # list) over the 128 records, each record twice
  half = np.zeros((128, R), np.int32)
  nodes = rs.permutation(np.arange(1, 5000))[:128 * (1 + K)].reshape(128, 1 + K)
  edges = rs.permutation(np.arange(1, 5000))[:128 * (1 + K)].reshape(128, 1 + K)
  half[:, 0] = nodes[:, 0]
  half[:, 4:4 + K] = nodes[:, 1:]
  half[:, 3] = edges[:, 0]
  half[:, 4 + K:] = edges[:, 1:]
  t0 = np.zeros((B, 3), np.float32)
  t0[:, 2] = rs.uniform(0, 1, B).astype(np.float32)
  blocks = [(np.concatenate([half, half]), t0), batch(10000, 30000),
            batch(1, 6), batch(1, 6), batch(1, 6), batch(10000, 30000),
            batch(1, 6), batch(30000, 40000, 3)]
  idx = np.concatenate([b[0] for b in blocks])
  tgt = np.concatenate([b[1] for b in blocks])
  perms = np.arange(idx.shape[0])[None, :]
  nrows = int(idx[:, [0, 2] + list(range(4, 4 + K))].max()) + 2
  erows = int(idx[:, [1, 3] + list(range(4 + K, 4 + 2 * K))].max()) + 2
  nt = rs.uniform(-0.05, 0.05, (nrows, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (erows, d)).astype(np.float32)
  for loss, act in ((O.LOSS_MSE, O.ACT_RELU), (O.LOSS_KLD, O.ACT_SIGMOID)):
    pp = np.repeat(perms, 2, 0)
    ont, oet, ol, _, _ = O.train(idx, tgt, K, nt, et, loss, act, batch=B,
                                 max_epochs=2, perms=pp, min_delta=-1.0)
    ctx.records_set(idx, tgt)
    ctx.model_init(d, nrows, erows, node_tab=nt, edge_tab=et)
    gl = ctx.train(batch=B, max_epochs=2, loss=loss, act=act, perms=pp,
                   min_delta=-1.0)
    assert ctx.train_path_stats() == (2 * len(blocks), 0)
    # hub batches after hub batches: records naming two deferred rows of the
    # previous batch -> the MULTI form of the step
    assert ctx.train_multi_pending() > 0
    gnt, get_ = ctx.model_get()
    assert np.allclose(gl, ol, rtol=1e-4, atol=1e-7), (gl, ol)
    assert np.abs(gnt - ont).max() < 1e-5 and np.abs(get_ - oet).max() < 1e-5


def test_step_diverged_gradients_raise(ctx):
  """Gradients beyond the step's fixed-point range (a diverged run) raise
  FloatingPointError instead of wrapping silently."""
  rs = np.random.RandomState(2)
  idx, tgt = _mixed_reuse_records(rs, 4, 256, 5, hub_batches={1})
  nrows = int(idx[:, [0, 2] + list(range(4, 14))].max()) + 2
  erows = int(idx[:, [1, 3] + list(range(9, 14))].max()) + 2
  ctx.records_set(idx, tgt)
  ctx.model_init(128, nrows, erows,
                 node_tab=np.full((nrows, 128), 30.0, np.float32),
                 edge_tab=np.full((erows, 128), 30.0, np.float32))
  with pytest.raises(FloatingPointError):
    ctx.train(batch=256, max_epochs=1, loss=O.LOSS_MSE, act=O.ACT_RELU,
              perms=np.arange(idx.shape[0])[None, :])


@pytest.mark.parametrize("mode,cus", [(1, 0), (1, 32), (2, 0)])
def test_overlapped_preparation_bitwise_equal(ctx, mode, cus):
  """Chunk c + 1 prepared on a second stream while chunk c trains (tuning
  train_prep_overlap 1; train_prep_cus: disjoint CU masks) or on the same
  stream one chunk ahead (train_prep_overlap 2) gives the in-line
  preparation's tables and losses bit for bit. 2,100 batches = three chunks
  of up to 1,024 (both placed-buffer sets used, one reused), hub batches on
  both chunk boundaries (deferred rows and MULTI batches across chunks),
  device shuffle in-order first epoch, then shuffled."""
  rs = np.random.RandomState(5)
  K, B, nb = 5, 256, 2100
  idx, tgt = _mixed_reuse_records(rs, nb, B, K,
                                  hub_batches={1022, 1023, 1024, 2047, 2048})
  idx, tgt = idx[:-100], tgt[:-100]
  perms = np.stack([np.arange(idx.shape[0]), rs.permutation(idx.shape[0])])
  ctx.records_set(idx, tgt)
  out = []
  try:
    for ov in (0, mode):
      ctx.set_tuning("train_prep_overlap", ov)
      ctx.set_tuning("train_prep_cus", cus)
      ctx.model_init(128, 20002, 20002, seed=9)
      gl = ctx.train(batch=B, max_epochs=2, loss=O.LOSS_MSE, act=O.ACT_RELU,
                     perms=perms, min_delta=-1.0)
      out.append(ctx.model_get() + (gl, ctx.train_path_stats(),
                                    ctx.train_multi_pending()))
  finally:
    ctx.set_tuning("train_prep_overlap", 0)
    ctx.set_tuning("train_prep_cus", 0)
  assert out[0][3] == (2 * nb, 0), out[0][3]
  assert out[0][4] > 0
  assert out[0][3:] == out[1][3:]
  assert np.array_equal(out[0][2], out[1][2]), (out[0][2], out[1][2])
  assert np.array_equal(out[0][0], out[1][0])
  assert np.array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("d", [128, 256])
def test_padding_row_fixed_point_vs_split_step_and_oracle(ctx, d):
  """The padding row (row 0 of both tables) collects the gradients of every
  absent slot as 2^-44 fixed point: per record at 128-float rows (early
  row-0 sums), per workgroup at 256-float rows. Batches where nearly every
  slot is row 0 (node-node records: edge slots and both neighbour lists
  empty, 12 of 14 slots padding) and mixed batches, in order, against the
  two-kernel step's fp32 sums (train_fused 0) and the oracle."""
  rs = np.random.RandomState(31)
  K, B, nb = 5, 256, 10
  n = nb * B - 77
  idx = np.zeros((n, 4 + 2 * K), np.int32)
  kind = np.where(np.arange(n) < 6 * B, 0, rs.randint(0, 3, n))
  m0, m1, m2 = kind == 0, kind == 1, kind == 2
  idx[m0, 0] = rs.randint(1, 50000, m0.sum())
  idx[m0, 2] = rs.randint(1, 50000, m0.sum())
  idx[m1, 1] = rs.randint(1, 20000, m1.sum())
  idx[m1, 3] = rs.randint(1, 20000, m1.sum())
  idx[m2, 0] = rs.randint(1, 50000, m2.sum())
  idx[m2, 3] = rs.randint(1, 20000, m2.sum())
  idx[m2, 4:4 + K] = rs.randint(1, 50000, (m2.sum(), K))
  idx[m2, 4 + K:] = rs.randint(1, 20000, (m2.sum(), K))
  tgt = np.zeros((n, 3), np.float32)
  tgt[np.arange(n), kind] = rs.uniform(0, 1, n).astype(np.float32)
  perms = np.stack([np.arange(n), rs.permutation(n)])
  nt = rs.uniform(-0.05, 0.05, (50001, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (20001, d)).astype(np.float32)
  ont, oet, ol, _, _ = O.train(idx, tgt, K, nt, et, O.LOSS_MSE, O.ACT_RELU,
                               batch=B, max_epochs=2, perms=perms,
                               min_delta=-1.0)
  ctx.records_set(idx, tgt)
  res = {}
  try:
    for fused in (1, 0):
      ctx.set_tuning("train_fused", fused)
      ctx.model_init(d, 50001, 20001, node_tab=nt, edge_tab=et)
      gl = ctx.train(batch=B, max_epochs=2, loss=O.LOSS_MSE, act=O.ACT_RELU,
                     perms=perms, min_delta=-1.0)
      res[fused] = ctx.model_get() + (gl,)
  finally:
    ctx.set_tuning("train_fused", 1)
  for fused in (1, 0):
    gnt, get_, gl = res[fused]
    assert np.allclose(gl, ol, rtol=1e-4, atol=1e-7), (fused, gl, ol)
    assert np.abs(gnt - ont).max() < 1e-5 and np.abs(get_ - oet).max() < 1e-5
  for t in (0, 1):  # row 0 moved, and both steps agree on it
    assert not np.array_equal(res[1][t][0], (nt, et)[t][0])
    assert np.abs(res[1][t][0] - res[0][t][0]).max() < 1e-6
