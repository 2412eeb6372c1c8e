"""Per-incidence and pair weights (reference:
hypergraph_embedding/hg2v_weighting.py).

UniformWeight (195-198) and WeightByNeighborhood (137-167) are computed on
the device (libhgx ``hgx_incidence_weights``, bit-exact with the reference's
double math rounded to float32 by DictToSparseRow) and returned as the same
scipy CSR pair as the reference (node2weight nodes x edges, edge2weight
edges x nodes, indexed by the hypergraph's own ids).

The distance weights run on the device too (csrc/hgx_weights.hip), with the
reference embedding's rows resident as the context's coordinates:
  * WeightByDistance (67-103): first order, per incidence;
  * WeightBySameTypeDistance (34-64): second order, every pair of the
    A A^T / A^T A pattern (diagonal included);
  * ComputeSpans (236-293) and WeightByAlgebraicSpan (170-192);
  * WeightByDistanceCluster (106-134): WeightByDistance's matrix, then the
    reference's own sklearn NMF on the host.
`norm` is np.linalg.norm (optionally functools.partial(np.linalg.norm,
ord=2 / np.inf)): the device restates numpy's float32 / float64 arithmetic
for it bit for bit; other callables raise ValueError. Zeros are not stored,
as the reference's lil_matrix does not store them.

The small dict helpers (ZeroOneScaleValues 301-317, OneMinusValues
325-326, AlphaScaleValues 329-333, DictToSparseRow 336-341) are host-side,
as in the reference.
"""

import functools

import numpy as np
import scipy.sparse

from . import _hgx
from .hypergraph_util import Incidence
from .runtime import scratch_context


def _to_csr(inc, node_major, edge_major):
  """Weights keyed by the hypergraph's own ids, shaped like the reference's
  ToCsrMatrix / ToEdgeCsrMatrix ((max id + 1) rows and columns)."""
  nrow = int(inc.node_ids.max()) + 1 if inc.N else 0
  ncol = int(inc.edge_ids.max()) + 1 if inc.E else 0
  rows = np.repeat(inc.node_ids, np.diff(inc.rp_n))
  cols = inc.edge_ids[inc.col_n]
  n2w = scipy.sparse.csr_matrix((node_major, (rows, cols)), shape=(nrow, ncol),
                                dtype=np.float32)
  rows = np.repeat(inc.edge_ids, np.diff(inc.rp_e))
  cols = inc.node_ids[inc.col_e]
  e2w = scipy.sparse.csr_matrix((edge_major, (rows, cols)), shape=(ncol, nrow),
                                dtype=np.float32)
  return n2w, e2w


def _weights(hypergraph, which, alpha):
  inc = Incidence.from_hypergraph(hypergraph)
  with scratch_context() as ctx:  # the reference functions have no side effects
    ctx.upload(inc)
    n, e = ctx.incidence_weights(which, alpha)
  return _to_csr(inc, n, e)


def UniformWeight(hypergraph):
  return _weights(hypergraph, _hgx.WEIGHT_UNIFORM, 0.0)


def WeightByNeighborhood(hypergraph, alpha):
  assert 0 <= alpha <= 1
  return _weights(hypergraph, _hgx.WEIGHT_NEIGHBORHOOD, float(alpha))


def _norm_kind(norm):
  """np.linalg.norm (ord None / 2) -> NORM_L2, ord inf -> NORM_INF."""
  ord_ = None
  if isinstance(norm, functools.partial) and norm.func is np.linalg.norm \
      and not norm.args and set(norm.keywords) <= {"ord"}:
    ord_ = norm.keywords.get("ord")
  elif norm is not np.linalg.norm:
    raise ValueError(f"norm {norm!r} is not supported on the device: pass "
                     "np.linalg.norm (ord None, 2 or np.inf)")
  if ord_ is None or ord_ == 2:
    return _hgx.NORM_L2
  if ord_ == np.inf:
    return _hgx.NORM_INF
  raise ValueError(f"np.linalg.norm ord={ord_!r} is not supported on the device")


def _rows_of(side_map, ids):
  """float32 rows of an embedding map (HypergraphEmbedding.node / .edge, or
  a ShardedEmbedding's) for the given original ids."""
  from .proto_native import _MapView
  if isinstance(side_map, _MapView):
    j = np.searchsorted(side_map._sorted, ids)
    assert np.all(j < side_map._sorted.size) and \
        np.array_equal(side_map._sorted[np.minimum(j, side_map._sorted.size - 1)], ids), \
        "embedding lacks ids of the hypergraph"
    return np.ascontiguousarray(side_map._tab[side_map._order[j]], np.float32)
  return np.array([side_map[int(i)].values for i in ids], np.float32)


def _with_embedding(hypergraph, ref_embedding, ctx):
  """Upload the hypergraph and the embedding's rows (as the alg coordinates)
  to the private context `ctx`; returns the compressed incidence."""
  inc = Incidence.from_hypergraph(hypergraph)
  X = _rows_of(ref_embedding.node, inc.node_ids)
  Y = _rows_of(ref_embedding.edge, inc.edge_ids)
  assert X.shape[1] == Y.shape[1] and X.shape[1] > 0
  ctx.upload(inc)
  ctx.alg_set(X, Y)
  return inc


def _nonzero(m):
  m.eliminate_zeros()  # lil_matrix never stores a zero
  return m


def WeightByDistance(hypergraph, alpha, ref_embedding, norm, disable_pbar=False):
  """hg2v_weighting.py:67-103: (node2edge_dist, its transpose), float32 CSR
  of (max node id + 1) x (max edge id + 1)."""
  del disable_pbar
  assert 0 <= alpha <= 1
  kind = _norm_kind(norm)
  with scratch_context() as ctx:
    inc = _with_embedding(hypergraph, ref_embedding, ctx)
    n, e = ctx.weight_distance(kind, float(alpha))
  return tuple(_nonzero(m) for m in _to_csr(inc, n, e))


def _pattern_csr(ids, rp, col, val):
  """Compressed-id CSR -> the reference's (max id + 1)^2 matrix."""
  nrow = int(ids.max()) + 1 if ids.size else 0
  indptr = np.zeros(nrow + 1, np.int64)
  indptr[ids + 1] = np.diff(rp)
  indptr = np.cumsum(indptr)
  m = scipy.sparse.csr_matrix((val, ids[col].astype(np.int32), indptr),
                              shape=(nrow, nrow), dtype=np.float32)
  return _nonzero(m)


def WeightBySameTypeDistance(hypergraph, alpha, ref_embedding, norm,
                             disable_pbar=False):
  """hg2v_weighting.py:34-64: (node2node_dist, edge2edge_dist) over the
  A A^T and A^T A patterns (diagonal included)."""
  del disable_pbar
  assert 0 <= alpha <= 1
  kind = _norm_kind(norm)
  out = []
  with scratch_context() as ctx:
    inc = _with_embedding(hypergraph, ref_embedding, ctx)
    for side, ids in ((0, inc.node_ids), (1, inc.edge_ids)):
      rp, col, val = ctx.weight_same_type(side, kind, float(alpha))
      out.append(_pattern_csr(ids, rp, col, val))
  return tuple(out)


def WeightByDistanceCluster(hypergraph, alpha, ref_embedding, norm, dim):
  """hg2v_weighting.py:106-134: WeightByDistance's node x edge matrix
  factored by sklearn NMF(dim) on the host (as the reference does)."""
  from sklearn.decomposition import NMF
  node2edge, _ = WeightByDistance(hypergraph, alpha, ref_embedding, norm)
  nmf_model = NMF(dim)
  W = nmf_model.fit_transform(node2edge)
  H = nmf_model.components_
  return scipy.sparse.csr_matrix(W), scipy.sparse.csr_matrix(H.T)


def _spans_on_device(hypergraph, embedding, alpha):
  """(node spans, edge spans, span weights per incidence node-major and
  edge-major) of the given embedding, or (as the reference's default) of a
  5-d, 10-iteration alg-dist of the hypergraph (hg2v_weighting.py:256-262)
  relaxed on the device; on a private context."""
  with scratch_context() as ctx:
    if embedding is not None:
      assert set(hypergraph.node) == set(embedding.node)
      assert set(hypergraph.edge) == set(embedding.edge)
      inc = _with_embedding(hypergraph, embedding, ctx)
    else:
      from .algebraic_distance import AlgebraicDistance
      inc = Incidence.from_hypergraph(hypergraph)
      AlgebraicDistance(inc, 5, 10, ctx=ctx)
    return (inc,) + ctx.weight_span(float(alpha))


def ComputeSpans(hypergraph, embedding=None, run_in_parallel=True,
                 disable_pbar=False):
  """hg2v_weighting.py:236-293: (node2span, edge2span) dicts keyed by the
  hypergraph's ids (float32 spans, as np.subtract of the embedding's float
  fields computes them)."""
  del run_in_parallel, disable_pbar
  inc, sn, se, _, _ = _spans_on_device(hypergraph, embedding, 0.0)
  return (dict(zip(inc.node_ids.tolist(), sn.tolist())),
          dict(zip(inc.edge_ids.tolist(), se.tolist())))


def WeightByAlgebraicSpan(hypergraph, alpha, embedding=None):
  """hg2v_weighting.py:170-192 (node2weight = A x the edges' scaled spans,
  edge2weight = A^T x the nodes'). `embedding` (not in the reference's
  signature) fixes ComputeSpans' embedding instead of its random alg-dist."""
  assert 0 <= alpha <= 1
  inc, _, _, n, e = _spans_on_device(hypergraph, embedding, alpha)
  return tuple(_nonzero(m) for m in _to_csr(inc, n, e))


def ZeroOneScaleValues(idx2value, disable_pbar=False):
  del disable_pbar
  if len(idx2value) == 0:
    return {}
  lo = min(idx2value.values())
  hi = max(idx2value.values())
  if hi - lo == 0:
    return {idx: 1 for idx in idx2value}
  return {idx: (v - lo) / (hi - lo) for idx, v in idx2value.items()}


def OneMinusValues(data):
  return {k: 1 - v for k, v in data.items()}


def AlphaScaleValues(data, alpha):
  assert 0 <= alpha <= 1
  return {k: (alpha + (1 - alpha) * v) for k, v in data.items()}


def DictToSparseRow(idx2val):
  num_cols = max(idx2val)
  row = scipy.sparse.lil_matrix((1, num_cols + 1), dtype=np.float32)
  for idx, val in idx2val.items():
    row[0, idx] = val
  return scipy.sparse.csr_matrix(row)


__all__ = ["UniformWeight", "WeightByNeighborhood", "WeightByDistance",
           "WeightBySameTypeDistance", "WeightByDistanceCluster",
           "WeightByAlgebraicSpan", "ComputeSpans", "ZeroOneScaleValues",
           "OneMinusValues", "AlphaScaleValues", "DictToSparseRow"]
