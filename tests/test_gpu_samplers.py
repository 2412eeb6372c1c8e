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


@pytest.fixture(scope="module")
def ctx():
  from hypergraphembedding_amd import _hgx
  c = _hgx.Context(0)
  yield c
  c.close()


@pytest.fixture(params=["expand", "paths", "uniform"])
def mode3(request, ctx):
  """Row sampling of the 2/3-hop patterns: expand every row; or sample every
  row with more than one path by rejection, 3-hop rows proposing uniform
  paths (Karp-Luby) or uniform columns (membership probe)."""
  if request.param == "expand":
    ctx.set_tuning("sample_reject_w", 0)
  else:
    ctx.set_tuning("sample_reject_w", 1)
    ctx.set_tuning("sample_mode3", 1 if request.param == "paths" else 2)
  yield request.param
  ctx.set_tuning("sample_reject_w", 32768)
  ctx.set_tuning("sample_mode3", 0)


@pytest.fixture(params=["expand", "union"])
def mode(request, ctx):
  """expand: every row's 2/3-hop expansion is materialised (default for
  these small graphs); union: rows with more than 1 path are sampled by
  rejection from the union (the path large power-law rows take)."""
  ctx.set_tuning("sample_reject_w", 1 if request.param == "union" else 0)
  yield request.param
  ctx.set_tuning("sample_reject_w", 32768)


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


def test_hobe_small_counts_and_probs(ctx, small_inc, mode3):
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


def test_fobe_powerlaw_union_rows(ctx):
  """Power-law edges make 2-hop rows far too large to expand: those rows are
  union-sampled; exact per-row counts min(S, |union|) and pair validity are
  checked on sampled rows, with unions computed from the CSR."""
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  inc = powerlaw_hypergraph(N=20_000, E=10_000, seed=4)
  S, K = 200, 5
  ctx.upload(inc)
  nq = np.full(inc.N, S, np.int32)
  eq = np.full(inc.E, S, np.int32)
  try:
    ctx.set_tuning("sample_reject_w", 4096)
    ctx.sample_fobe(21, K, nq, eq)
  finally:
    ctx.set_tuning("sample_reject_w", 32768)
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


def _hop3_row(inc, side, r):
  """Row r of A A^T A (side 'node') or A^T A A^T (side 'edge') as a sorted
  array, from the CSR."""
  if side == "node":
    l1, l2, l3 = (inc.rp_n, inc.col_n), (inc.rp_e, inc.col_e), (inc.rp_n, inc.col_n)
  else:
    l1, l2, l3 = (inc.rp_e, inc.col_e), (inc.rp_n, inc.col_n), (inc.rp_e, inc.col_e)
  m1 = l1[1][l1[0][r]:l1[0][r + 1]]
  m2 = np.unique(np.concatenate([l2[1][l2[0][m]:l2[0][m + 1]] for m in m1]))
  return np.unique(np.concatenate([l3[1][l3[0][m]:l3[0][m + 1]] for m in m2]))


@pytest.mark.parametrize("side", ["node", "edge"])
def test_hobe_3hop_uniformity_chi_square(ctx, small_inc, mode3, side):
  """Inclusion frequency of every column of a 3-hop row (A A^T A node rows,
  A^T A A^T edge rows) is q/|row| over seeds, in every sampling mode."""
  inc = small_inc
  z = golden("hobe_small.npz")
  ctx.upload(inc)
  ctx.alg_set(z["alg_x"], z["alg_y"])
  nrow = inc.N if side == "node" else inc.E
  rs = np.random.RandomState(5)
  rows = rs.choice(nrow, 40, replace=False)
  sizes = np.array([_hop3_row(inc, side, r).size for r in rows])
  r = int(rows[np.argmax(sizes)])
  full = _hop3_row(inc, side, r)
  q = max(2, full.size // 3)
  nq = np.zeros(inc.N, np.int32)
  eq = np.zeros(inc.E, np.int32)
  (nq if side == "node" else eq)[r] = q
  counts = np.zeros(full.size, np.int64)
  trials = 150
  for seed in range(trials):
    ctx.sample_hobe(3000 + seed, 2, q, node_q=nq, edge_q=eq)
    idx, _ = ctx.records_get()
    ne = (idx[:, 0] > 0) & (idx[:, 3] > 0) & (idx[:, 2] == 0)
    if side == "node":
      cols = idx[ne & (idx[:, 0] == r + 1), 3] - 1
    else:
      cols = idx[ne & (idx[:, 3] == r + 1), 0] - 1
    assert cols.size == q and np.unique(cols).size == q
    pos = np.searchsorted(full, cols)
    assert np.all(full[np.minimum(pos, full.size - 1)] == cols)
    counts[pos] += 1
  exp = np.full(full.size, trials * q / full.size)
  chi = scipy.stats.chisquare(counts, exp)
  assert chi.pvalue > 1e-4, (mode3, side, chi)


def test_neighbor_draws_uniform_chi_square(ctx, small_inc):
  """_sample_neighbors (hg2v_sample.py:49-51): K draws WITH replacement,
  uniform over N(e) (nn_k) and over E(v) (ne_k): chi-square over seeds."""
  inc = small_inc
  ctx.upload(inc)
  K = 5
  e = int(np.argmax(inc.edge_size()))
  v = int(np.argmax(np.diff(inc.rp_n)))
  members = inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]
  edges_v = inc.col_n[inc.rp_n[v]:inc.rp_n[v + 1]]
  assert members.size >= 8 and edges_v.size >= 4
  nq = np.zeros(inc.N, np.int32)
  eq = np.zeros(inc.E, np.int32)
  nq[v] = edges_v.size  # ne records (v, e') for every e' in E(v)
  eq[e] = members.size  # ne records (u, e) for every u in e
  cn = np.zeros(members.size, np.int64)
  ce = np.zeros(edges_v.size, np.int64)
  for seed in range(60):
    ctx.sample_fobe(500 + seed, K, nq, eq)
    idx, _ = ctx.records_get()
    ne = (idx[:, 0] > 0) & (idx[:, 3] > 0) & (idx[:, 2] == 0)
    nn_k = idx[ne & (idx[:, 3] == e + 1), 4:4 + K].ravel() - 1
    ne_k = idx[ne & (idx[:, 0] == v + 1), 4 + K:].ravel() - 1
    assert np.isin(nn_k, members).all() and np.isin(ne_k, edges_v).all()
    cn += np.bincount(np.searchsorted(members, nn_k), minlength=members.size)
    ce += np.bincount(np.searchsorted(edges_v, ne_k), minlength=edges_v.size)
  for obs in (cn, ce):
    chi = scipy.stats.chisquare(obs, np.full(obs.size, obs.sum() / obs.size))
    assert chi.pvalue > 1e-4, (chi, obs)


def test_neighbors_isolated_endpoint_raises(ctx):
  """np.random.choice on an empty row raises ValueError in the reference
  (hg2v_sample.py:49-51): a node-edge negative whose node has no edges."""
  from hypergraphembedding_amd.hypergraph_util import Incidence
  # node 2 has no edges
  inc = Incidence(3, 2, [0, 2, 3, 3], [0, 1, 1])
  ctx.upload(inc)
  z3, z2 = np.zeros(3, np.int32), np.zeros(2, np.int32)
  with pytest.raises(ValueError):
    ctx.sample_fobe(1, 2, z3, z2, np.array([0, 0, 3], np.int32), z2)
  # without the isolated endpoint the same call succeeds
  ctx.sample_fobe(1, 2, z3, z2, np.array([3, 3, 0], np.int32), z2)


def test_hobe_powerlaw_probs_bit_exact_and_counts(ctx):
  """HOBE on a 20k/10k power-law graph (edges up to ~15k members), the C4
  shape scaled down: large 2/3-hop rows are rejection-sampled (3-hop rows by
  uniform columns or paths), never expanded. Exact per-row counts
  min(S, |row|) and pair validity on sampled rows (row sets from the CSR),
  and the nn / ee / ne probability of every record of those rows (plus every
  nn record) bit-exact vs the oracle's restatement of
  _same_type_dist_calc / DiffTypeDistanceSample."""
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  inc = powerlaw_hypergraph(N=20_000, E=10_000, seed=4)
  S, K = 200, 5
  ctx.upload(inc)
  r = O.Rng(5)
  ctx.alg_set(r.random((inc.N, 10)), r.random((inc.E, 10)))
  ctx.alg_run(20)
  xg, yg = ctx.alg_get()
  rs = np.random.RandomState(3)
  big = np.argsort(-inc.edge_size())[:8]
  for side in ("node", "edge"):
    nrow = inc.N if side == "node" else inc.E
    nq = np.full(inc.N, S if side == "node" else 0, np.int32)
    eq = np.full(inc.E, S if side == "edge" else 0, np.int32)
    ctx.sample_hobe(77, K, S, node_q=nq, edge_q=eq)
    rej, _ = ctx.sample_stats()
    assert rej > nrow // 2, (side, rej)
    if side == "node":
      assert ctx.sample_uniform_rows() > 1000
    idx, tgt = ctx.records_get()
    nn, ee, ne = _blocks(idx, tgt, K)
    if side == "node":
      a, b = idx[nn, 0] - 1, idx[nn, 2] - 1
      p = O.hobe_probs(O.HOBE_NN, a, b, inc, xg, yg)
      assert np.array_equal(tgt[nn, 0], p)
      left, right = idx[ne, 0] - 1, idx[ne, 3] - 1
    else:
      left, right = idx[ne, 3] - 1, idx[ne, 0] - 1
      le, re = idx[ee, 1] - 1, idx[ee, 3] - 1
    cnt = np.bincount(left, minlength=nrow)
    rows = rs.choice(nrow, 60, replace=False)
    if side == "edge":
      rows = np.unique(np.concatenate([rows, big]))
    for row in rows:
      full = _hop3_row(inc, side, row)
      assert cnt[row] == min(S, full.size), (side, row)
      got = right[left == row]
      assert np.unique(got).size == got.size and np.isin(got, full).all()
    sel = np.isin(left, rows)
    v, e = (left[sel], right[sel]) if side == "node" else (right[sel], left[sel])
    p = O.hobe_probs(O.HOBE_NE, v, e, inc, xg, yg)
    assert np.array_equal(tgt[ne][sel, 2], p), side
    if side == "edge":
      se = np.isin(le, rows)
      p = O.hobe_probs(O.HOBE_EE, le[se], re[se], inc, xg, yg)
      assert np.array_equal(tgt[ee][se, 1], p)
      cnt_ee = np.bincount(le, minlength=inc.E)
      for row in rows[:20]:
        two = _two_hop_row(inc, row)
        assert cnt_ee[row] == min(S, two.size)
        got = re[le == row]
        assert np.unique(got).size == got.size and np.isin(got, two).all()


def _two_hop_row(inc, e):
  mids = inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]
  return np.unique(np.concatenate([inc.col_n[inc.rp_n[m]:inc.rp_n[m + 1]] for m in mids]))


def test_hobe_probs_api_powerlaw_vs_oracle(ctx):
  """hgx_hobe_probs on explicit pairs of a power-law graph, including the
  largest edges paired with each other and with themselves."""
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  inc = powerlaw_hypergraph(N=20_000, E=10_000, seed=6)
  ctx.upload(inc)
  r = O.Rng(8)
  x, y = r.random((inc.N, 10)).astype(np.float32), r.random((inc.E, 10)).astype(np.float32)
  ctx.alg_set(x, y)
  rs = np.random.RandomState(0)
  big = np.argsort(-inc.edge_size())[:12]
  ea = np.concatenate([np.repeat(big, 12), rs.randint(0, inc.E, 3000)])
  eb = np.concatenate([np.tile(big, 12), rs.randint(0, inc.E, 3000)])
  assert np.array_equal(ctx.hobe_probs(1, ea, eb), O.hobe_probs(O.HOBE_EE, ea, eb, inc, x, y))
  va = rs.randint(0, inc.N, 4000)
  vb = np.concatenate([np.repeat(big, 100), rs.randint(0, inc.E, 2800)])
  assert np.array_equal(ctx.hobe_probs(2, va, vb), O.hobe_probs(O.HOBE_NE, va, vb, inc, x, y))
  na, nb = rs.randint(0, inc.N, 5000), rs.randint(0, inc.N, 5000)
  assert np.array_equal(ctx.hobe_probs(0, na, nb), O.hobe_probs(O.HOBE_NN, na, nb, inc, x, y))
