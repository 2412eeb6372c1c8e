"""GPU parity: weighted-Jaccard samplers (HG2V_ADJ_JAC / HG2V_NEIGH_JAC).

Against the reference's own outputs (tests/golden/jaccard_small.npz, made
by running WeightedJaccardSamples) and the bit-exact oracle:
  * GetAllCentroids matrices: bit-exact;
  * probabilities of the reference's own pairs: bit-exact to its targets;
  * the device sampler: per-row counts equal to the reference's, every
    pair valid and distinct, neighbours from the right rows, and every
    probability bit-exact to the oracle for the device's pairs.
"""

import numpy as np
import pytest
import scipy.sparse as sp

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
  from hypergraphembedding_amd import _hgx
  c = _hgx.Context(0)
  yield c
  c.close()


def _features(z, inc, kind):
  if kind == "uniform":
    one = np.ones(inc.nnz, np.float32)
    return one, one
  return z["neigh_fn_v"], z["neigh_fe_v"]


def _quotas(z, inc, kind):
  S = int(z["S"])
  if kind == "uniform":
    return np.full(inc.N, S, np.int32), np.full(inc.E, S, np.int32)
  q = lambda w: np.array([int(float(x) * S) for x in w], np.int32)
  return q(z["neigh_node_weight"]), q(z["neigh_edge_weight"])


def _kinds(idx):
  nn = (idx[:, 0] > 0) & (idx[:, 2] > 0)
  ee = (idx[:, 1] > 0) & (idx[:, 3] > 0)
  ne = (idx[:, 0] > 0) & (idx[:, 3] > 0) & (idx[:, 2] == 0)
  return nn, ee, ne


def test_centroids_bit_exact(ctx, small_inc):
  z = golden("jaccard_small.npz")
  ctx.upload(small_inc)
  ctx.features_set(*_features(z, small_inc, "neigh"))
  for which, name in ((0, "cn"), (1, "ce")):
    p, j, v = ctx.jaccard_centroids(which)
    assert np.array_equal(p, z[name + "_p"])
    assert np.array_equal(j, z[name + "_j"])
    assert np.array_equal(v, z[name + "_v"])


@pytest.mark.parametrize("kind", ["uniform", "neigh"])
def test_probs_of_reference_pairs(ctx, small_inc, kind):
  z = golden("jaccard_small.npz")
  ctx.upload(small_inc)
  ctx.features_set(*_features(z, small_inc, kind))
  idx, tgt = z[kind + "_idx"], z[kind + "_tgt"]
  nn, ee, ne = _kinds(idx)
  got = ctx.jaccard_probs(0, idx[nn, 0] - 1, idx[nn, 2] - 1)
  assert np.array_equal(got, tgt[nn, 0])
  got = ctx.jaccard_probs(1, idx[ee, 1] - 1, idx[ee, 3] - 1)
  assert np.array_equal(got, tgt[ee, 1])
  got = ctx.jaccard_probs(2, idx[ne, 0] - 1, idx[ne, 3] - 1)
  assert np.array_equal(got, tgt[ne, 2])


@pytest.mark.parametrize("kind", ["uniform", "neigh"])
def test_sampler_vs_reference(ctx, small_inc, kind):
  z = golden("jaccard_small.npz")
  inc, K = small_inc, int(z["K"])
  fn, fe = _features(z, inc, kind)
  ctx.upload(inc)
  ctx.features_set(fn, fe)
  nq, eq = _quotas(z, inc, kind)
  n = ctx.sample_jaccard(31, K, nq, eq)
  idx, tgt = ctx.records_get()
  ridx = z[kind + "_idx"]
  assert n == ridx.shape[0]
  g, r = _kinds(idx), _kinds(ridx)
  for a, b in zip(g, r):
    assert np.array_equal(a, b)  # same kind blocks in the same order
  a, at = inc.to_scipy()
  a, at = a.astype(np.int32), at.astype(np.int32)
  nn, ee, ne = g
  for sel, lc, rc, pat, nrow in ((nn, 0, 2, a @ at, inc.N), (ee, 1, 3, at @ a, inc.E)):
    left, right = idx[sel, lc] - 1, idx[sel, rc] - 1
    assert np.array_equal(np.bincount(left, minlength=nrow),
                          np.bincount(ridx[sel, lc] - 1, minlength=nrow))
    assert np.all(np.asarray(sp.csr_matrix(pat)[left, right]).ravel() != 0)
    key = left.astype(np.int64) * (1 << 32) + right
    assert np.unique(key).size == key.size
  v, e = idx[ne, 0] - 1, idx[ne, 3] - 1
  assert np.all(np.asarray(sp.csr_matrix(a @ at @ a)[v, e]).ravel() != 0)
  assert np.all(np.asarray(at[np.repeat(e, K), (idx[ne, 4:4 + K] - 1).ravel()]).ravel())
  assert np.all(np.asarray(a[np.repeat(v, K), (idx[ne, 4 + K:] - 1).ravel()]).ravel())
  # probabilities of the device's own pairs: bit-exact to the oracle
  assert np.array_equal(tgt[nn, 0], O.jaccard_probs(0, idx[nn, 0] - 1, idx[nn, 2] - 1, inc, fn, fe))
  assert np.array_equal(tgt[ee, 1], O.jaccard_probs(1, idx[ee, 1] - 1, idx[ee, 3] - 1, inc, fn, fe))
  assert np.array_equal(tgt[ne, 2], O.jaccard_probs(2, v, e, inc, fn, fe))
  assert np.all(tgt[nn][:, 1:] == 0) and np.all(tgt[ee][:, [0, 2]] == 0)


def test_tiny_probs_and_centroids_vs_oracle(ctx, tiny_inc):
  """youtube_tiny has a 2217-member edge: long merges, big centroids."""
  inc = tiny_inc
  rs = np.random.RandomState(5)
  fn = rs.uniform(0.1, 1.0, inc.nnz).astype(np.float32)
  fe = rs.uniform(0.1, 1.0, inc.nnz).astype(np.float32)
  ctx.upload(inc)
  ctx.features_set(fn, fe)
  p, j, v = ctx.jaccard_centroids(0)
  op, oj, ov = O.centroids(inc.N, inc.rp_n, inc.col_n, inc.N, inc.rp_e, inc.col_e, fe)
  assert np.array_equal(p, op) and np.array_equal(j, oj) and np.array_equal(v, ov)
  p, j, v = ctx.jaccard_centroids(1)
  op, oj, ov = O.centroids(inc.E, inc.rp_e, inc.col_e, inc.E, inc.rp_n, inc.col_n, fn)
  assert np.array_equal(p, op) and np.array_equal(j, oj) and np.array_equal(v, ov)
  for kind, na, nb in ((0, inc.N, inc.N), (1, inc.E, inc.E), (2, inc.N, inc.E)):
    a = rs.randint(0, na, 3000)
    b = rs.randint(0, nb, 3000)
    assert np.array_equal(ctx.jaccard_probs(kind, a, b),
                          O.jaccard_probs(kind, a, b, inc, fn, fe))


@pytest.mark.parametrize("kind", ["uniform", "neigh"])
def test_sampler_mt_is_the_reference_stream(ctx, small_inc, kind):
  """rng="mt19937": np.random.seed(the fixture's seed), then the device
  sampler drawing numpy's stream returns WeightedJaccardSamples' own
  records (run_in_parallel=False), ids, neighbours and probabilities."""
  z = golden("jaccard_small.npz")
  inc, K = small_inc, int(z["K"])
  ctx.upload(inc)
  ctx.features_set(*_features(z, inc, kind))
  nq, eq = _quotas(z, inc, kind)
  np.random.seed(int(z[kind + "_seed"]))
  n = ctx.sample_jaccard_mt(K, nq, eq)
  idx, tgt = ctx.records_get()
  assert n == z[kind + "_idx"].shape[0]
  assert np.array_equal(idx, z[kind + "_idx"])
  assert np.array_equal(tgt, z[kind + "_tgt"])
