"""GPU parity for the FOBE/HOBE samplers.

The device draws with a counter-based generator, not numpy's MT19937 stream,
so parity with the reference (whose stream the oracle reproduces bit-exactly)
is checked on everything that is NOT random plus the distribution:
  * per-row record counts exactly equal (min(q, |distinct row|), hg2v_sample.py:80-83)
    and the record kind blocks in the reference's order;
  * every (row, col) pair is a member of the row of A*A^T / A^T*A / A /
    A*A^T*A / ... and distinct within its row;
  * neighbour draws come from the right rows (nn_k in N(e), ne_k in E(v));
  * HOBE probabilities of every record equal the oracle's for that pair
    (bit-exact given the same coordinates);
  * uniformity of the chosen subset (chi-square over seeds).
"""

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.stats

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["expand", "union"])
def mode(request, monkeypatch):
  """expand: every row's 2-hop expansion is materialised (default for these
  small graphs); union: 2-hop rows with more than 1 path are union-sampled
  by Karp-Luby rejection (the path large power-law rows take)."""
  if request.param == "union":
    monkeypatch.setenv("HGX_SAMPLE_REJECT_W", "1")
  else:
    monkeypatch.setenv("HGX_SAMPLE_REJECT_W", "0")
  return request.param


@pytest.fixture(scope="module")
def ctx():
  from hypergraphembedding_amd import _hgx
  c = _hgx.Context(0)
  yield c
  c.close()


def _blocks(idx, tgt, K):
  """Split model-input records into kind blocks by which fields are set."""
  ln, le, rn, re = idx[:, 0], idx[:, 1], idx[:, 2], idx[:, 3]
  nn = (ln > 0) & (rn > 0)
  ee = (le > 0) & (re > 0)
  ne = (ln > 0) & (re > 0) & (rn == 0)
  return nn, ee, ne


def _pairs_valid(pat, rows, cols):
  pat = sp.csr_matrix(pat)
  return bool(np.all(np.asarray(pat[rows, cols]).ravel() != 0))


def _row_counts(rows, n):
  return np.bincount(rows, minlength=n)


def _check_distinct(rows, cols):
  key = rows.astype(np.int64) * (1 << 32) + cols
  assert np.unique(key).size == key.size


def test_fobe_tiny_counts_validity(ctx, tiny_inc, mode):
  inc = tiny_inc
  S, K = 200, 5
  ctx.upload(inc)
  nq = np.full(inc.N, S, np.int32)
  eq = np.full(inc.E, S, np.int32)
  n = ctx.sample_fobe(7, K, nq, eq)
  idx, tgt = ctx.records_get()
  assert n == idx.shape[0] == 724792  # == reference (golden fobe_tiny n)
  ridx, rtgt = O.fobe_sample(O.Rng(3), inc, nq, eq, K)
  a, at = inc.to_scipy()
  a = a.astype(np.int32)
  at = at.astype(np.int32)
  gnn, gee, gne = _blocks(idx, tgt, K)
  onn, oee, one = _blocks(ridx, rtgt, K)
  # same block layout: nn, then ee, then ne (node rows, then edge rows)
  assert np.array_equal(gnn, onn) and np.array_equal(gee, oee)
  assert np.array_equal(gne, one)
  # nn: counts per row and membership in A*A^T
  r, c = idx[gnn, 0] - 1, idx[gnn, 2] - 1
  assert np.array_equal(_row_counts(r, inc.N), _row_counts(ridx[onn, 0] - 1, inc.N))
  assert _pairs_valid(a @ at, r, c)
  _check_distinct(r, c)
  r, c = idx[gee, 1] - 1, idx[gee, 3] - 1
  assert np.array_equal(_row_counts(r, inc.E), _row_counts(ridx[oee, 1] - 1, inc.E))
  assert _pairs_valid(at @ a, r, c)
  _check_distinct(r, c)
  # ne: node side = min(S, deg(v)) incidences of v, then edge side =
  # min(S, |e|) incidences of e (swapped); youtube_tiny has edges > S
  v, e = idx[gne, 0] - 1, idx[gne, 3] - 1
  assert _pairs_valid(a, v, e)
  n_node = int(np.minimum(inc.node_degree(), S).sum())
  assert np.array_equal(_row_counts(v[:n_node], inc.N), np.minimum(inc.node_degree(), S))
  assert np.array_equal(_row_counts(e[n_node:], inc.E), np.minimum(inc.edge_size(), S))
  ov, oe = ridx[one, 0] - 1, ridx[one, 3] - 1
  assert np.array_equal(_row_counts(ov[:n_node], inc.N), _row_counts(v[:n_node], inc.N))
  assert np.array_equal(_row_counts(oe[n_node:], inc.E), _row_counts(e[n_node:], inc.E))
  _check_distinct(v[:n_node], e[:n_node])
  _check_distinct(e[n_node:], v[n_node:])
  # neighbours: nn_k in N(e) (+1), ne_k in E(v) (+1)
  nbn = idx[gne, 4:4 + K] - 1
  nbe = idx[gne, 4 + K:] - 1
  assert _pairs_valid(at, np.repeat(e, K), nbn.ravel())
  assert _pairs_valid(a, np.repeat(v, K), nbe.ravel())
  union_rows, _ = ctx.sample_stats()
  assert (union_rows > 0) == (mode == "union")
  # targets: 1 on the record's own head, 0 elsewhere (unweighted FOBE)
  assert np.all(tgt[gnn, 0] == 1) and np.all(tgt[gee, 1] == 1)
  assert np.all(tgt[gne, 2] == 1)
  assert np.all(tgt.sum(1) == 1)


def test_fobe_weighted_negatives_counts(ctx, small_inc):
  z = golden("fobe_small_ns.npz")
  S, neg, K = int(z["S"]), int(z["neg"]), int(z["K"])
  nq = np.array([int(float(w) * S) for w in z["node_weight"]], np.int32)
  eq = np.array([int(float(w) * S) for w in z["edge_weight"]], np.int32)
  nnq = np.array([int(float(w) * neg) for w in z["node_weight"]], np.int32)
  neq = np.array([int(float(w) * neg) for w in z["edge_weight"]], np.int32)
  ctx.upload(small_inc)
  n = ctx.sample_fobe(11, K, nq, eq, nnq, neq)
  idx, tgt = ctx.records_get()
  ref_idx, ref_tgt = z["idx"], z["tgt"]
  assert n == ref_idx.shape[0]
  # positives then negatives with the same per-kind sizes as the reference
  pos = tgt.sum(1) > 0
  assert np.array_equal(pos, ref_tgt.sum(1) > 0)
  for col in range(4):
    assert np.array_equal(idx[:, col] > 0, ref_idx[:, col] > 0), col
  # negatives are uniform over all columns -> just in range
  assert idx[:, [0, 2]].max() <= small_inc.N and idx[:, [1, 3]].max() <= small_inc.E


def test_hobe_small_counts_and_probs(ctx, small_inc):
  z = golden("hobe_small.npz")
  S, K = int(z["S"]), int(z["K"])
  ctx.upload(small_inc)
  ctx.alg_set(z["alg_x"], z["alg_y"])  # the reference's alg coords
  n = ctx.sample_hobe(5, K, S)
  idx, tgt = ctx.records_get()
  ref_idx, ref_tgt = z["idx"], z["tgt"]
  assert n == ref_idx.shape[0]
  gnn, gee, gne = _blocks(idx, tgt, K)
  onn, oee, one = _blocks(ref_idx, ref_tgt, K)
  assert gnn.sum() == onn.sum() and gee.sum() == oee.sum() and gne.sum() == one.sum()
  a, at = small_inc.to_scipy()
  a = a.astype(np.int32)
  at = at.astype(np.int32)
  r, c = idx[gnn, 0] - 1, idx[gnn, 2] - 1
  assert np.array_equal(_row_counts(r, small_inc.N), _row_counts(ref_idx[onn, 0] - 1, small_inc.N))
  assert _pairs_valid(a @ at, r, c)
  _check_distinct(r, c)
  p = O.hobe_probs(O.HOBE_NN, r, c, small_inc, z["alg_x"], z["alg_y"])
  assert np.array_equal(tgt[gnn, 0], p)
  r, c = idx[gee, 1] - 1, idx[gee, 3] - 1
  assert _pairs_valid(at @ a, r, c)
  _check_distinct(r, c)
  p = O.hobe_probs(O.HOBE_EE, r, c, small_inc, z["alg_x"], z["alg_y"])
  assert np.array_equal(tgt[gee, 1], p)
  v, e = idx[gne, 0] - 1, idx[gne, 3] - 1
  assert _pairs_valid(a @ at @ a, v, e)
  p = O.hobe_probs(O.HOBE_NE, v, e, small_inc, z["alg_x"], z["alg_y"])
  assert np.array_equal(tgt[gne, 2], p)
  assert _pairs_valid(at, np.repeat(e, K), (idx[gne, 4:4 + K] - 1).ravel())
  assert _pairs_valid(a, np.repeat(v, K), (idx[gne, 4 + K:] - 1).ravel())
  # node-side block (rows of A*A^T*A) then edge-side block (rows of
  # A^T*A*A^T, swapped): exact per-row counts min(S, |row|)
  n3 = np.diff((a @ at @ a).tocsr().indptr)
  e3 = np.diff((at @ a @ at).tocsr().indptr)
  n_node = int(np.minimum(n3, S).sum())
  assert n_node + int(np.minimum(e3, S).sum()) == gne.sum()
  assert np.array_equal(_row_counts(v[:n_node], small_inc.N), np.minimum(n3, S))
  assert np.array_equal(_row_counts(e[n_node:], small_inc.E), np.minimum(e3, S))
  _check_distinct(v[:n_node], e[:n_node])
  _check_distinct(e[n_node:], v[n_node:])


def test_sampler_uniformity_chi_square(ctx, small_inc, mode):
  """Inclusion frequency of every column of a row is q/|row| over seeds."""
  ctx.upload(small_inc)
  a, at = small_inc.to_scipy()
  nn = (a.astype(np.int32) @ at.astype(np.int32)).tocsr()
  sizes = np.diff(nn.indptr)
  row = int(np.argmax(sizes))
  q = max(2, sizes[row] // 3)
  nq = np.zeros(small_inc.N, np.int32)
  nq[row] = q
  eq = np.zeros(small_inc.E, np.int32)
  counts = {}
  trials = 300
  for seed in range(trials):
    ctx.sample_fobe(1000 + seed, 2, nq, eq)
    idx, _ = ctx.records_get()
    cols = idx[(idx[:, 0] == row + 1) & (idx[:, 2] > 0), 2] - 1
    assert cols.size == q
    for c in cols:
      counts[c] = counts.get(c, 0) + 1
  cols = np.sort(nn[row].indices)
  obs = np.array([counts.get(c, 0) for c in cols])
  assert set(counts) <= set(cols.tolist())
  exp = np.full(cols.size, trials * q / cols.size)
  chi = scipy.stats.chisquare(obs, exp)
  assert chi.pvalue > 1e-4, (chi, obs)


def test_sampler_deterministic_for_seed(ctx, small_inc, mode):
  ctx.upload(small_inc)
  nq = np.full(small_inc.N, 5, np.int32)
  eq = np.full(small_inc.E, 5, np.int32)
  ctx.sample_fobe(3, 2, nq, eq)
  a = ctx.records_get()
  ctx.sample_fobe(3, 2, nq, eq)
  b = ctx.records_get()
  ctx.sample_fobe(4, 2, nq, eq)
  c = ctx.records_get()
  assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
  assert not np.array_equal(a[0], c[0])


def test_fobe_powerlaw_union_rows(ctx, monkeypatch):
  """Power-law edges make 2-hop rows far too large to expand: those rows are
  union-sampled; exact per-row counts min(S, |union|) and pair validity are
  checked on sampled rows, with unions computed from the CSR."""
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  monkeypatch.setenv("HGX_SAMPLE_REJECT_W", "4096")
  inc = powerlaw_hypergraph(N=20_000, E=10_000, seed=4)
  S, K = 200, 5
  ctx.upload(inc)
  nq = np.full(inc.N, S, np.int32)
  eq = np.full(inc.E, S, np.int32)
  ctx.sample_fobe(21, K, nq, eq)
  union_rows, fallbacks = ctx.sample_stats()
  assert union_rows > 1000
  idx, tgt = ctx.records_get()
  gnn, gee, _ = _blocks(idx, tgt, K)
  rs = np.random.RandomState(1)
  for kind, rp1, c1, rp2, c2, nrow, lcol, rcol, sel in (
      ("nn", inc.rp_n, inc.col_n, inc.rp_e, inc.col_e, inc.N, 0, 2, gnn),
      ("ee", inc.rp_e, inc.col_e, inc.rp_n, inc.col_n, inc.E, 1, 3, gee)):
    left = idx[sel, lcol] - 1
    right = idx[sel, rcol] - 1
    cnt = np.bincount(left, minlength=nrow)
    for r in rs.choice(nrow, 80, replace=False):
      mids = c1[rp1[r]:rp1[r + 1]]
      union = np.unique(np.concatenate([c2[rp2[m]:rp2[m + 1]] for m in mids]))
      assert cnt[r] == min(S, union.size), (kind, r)
      got = right[left == r]
      assert np.unique(got).size == got.size and np.isin(got, union).all()
