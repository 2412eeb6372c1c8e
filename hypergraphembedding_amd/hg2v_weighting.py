"""Per-incidence weights (reference: hypergraph_embedding/hg2v_weighting.py).

UniformWeight (195-198) and WeightByNeighborhood (137-167) are computed on
the device (libhgx ``hgx_incidence_weights``, bit-exact with the reference's
double math rounded to float32 by DictToSparseRow) and returned as the same
scipy CSR pair as the reference (node2weight nodes x edges, edge2weight
edges x nodes, indexed by the hypergraph's own ids). The small dict helpers
(ZeroOneScaleValues 301-317, OneMinusValues 325-326, AlphaScaleValues
329-333, DictToSparseRow 336-341) are host-side, as in the reference.
"""

import numpy as np
import scipy.sparse

from . import _hgx
from .hypergraph_util import Incidence
from .runtime import get_context


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
  ctx = get_context()
  ctx.upload(inc)
  n, e = ctx.incidence_weights(which, alpha)
  return _to_csr(inc, n, e)


def UniformWeight(hypergraph):
  return _weights(hypergraph, _hgx.WEIGHT_UNIFORM, 0.0)


def WeightByNeighborhood(hypergraph, alpha):
  assert 0 <= alpha <= 1
  return _weights(hypergraph, _hgx.WEIGHT_NEIGHBORHOOD, float(alpha))


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


__all__ = ["UniformWeight", "WeightByNeighborhood", "ZeroOneScaleValues",
           "OneMinusValues", "AlphaScaleValues", "DictToSparseRow"]
