"""Hypergraph proto <-> CSR incidence helpers.

Mirrors the hot-path subset of reference ``hypergraph_embedding/hypergraph_util.py``
(AddNodeToEdge 13-44, RemoveNodeFromEdge 47-58, CreateRandomHyperGraph 61-75,
FromSparseMatrix 78-88, IsEmpty 91-93, ToCsrMatrix 96-114, ToEdgeCsrMatrix
117-135, ToCscMatrix 138-156, Relabel 198-220, CompressRange 223-244,
RemoveNode 288-294, RemoveEdge 297-303) with the same names and semantics.

New here: :class:`Incidence`, the device-ready form of a hypergraph. It is the
compressed (0..n-1, sorted-id) incidence matrix in BOTH orientations as int32
CSR with sorted columns -- exactly ``ToCsrMatrix(CompressRange(hg)[0])`` and
``ToEdgeCsrMatrix(...)`` -- plus the inverse id maps and the per-row weights.
It is built with numpy instead of the reference's per-incidence
``AddNodeToEdge`` loop (hypergraph_util.py:28-31 is O(nnz*deg)).
"""

from random import random

import numpy as np
import scipy as sp
import scipy.sparse

from .proto import Hypergraph


def AddNodeToEdge(hypergraph, node_idx, edge_idx, node_name=None,
                  edge_name=None):
  """Connect node -> edge in both maps (hypergraph_util.py:13-44)."""
  assert node_idx >= 0
  assert edge_idx >= 0
  node = hypergraph.node[node_idx]
  edge = hypergraph.edge[edge_idx]
  if edge_idx not in node.edges:
    node.edges.append(edge_idx)
  if node_idx not in edge.nodes:
    edge.nodes.append(node_idx)
  if node_name is not None:
    node.name = node_name
  if edge_name is not None:
    edge.name = edge_name
  return hypergraph


def RemoveNodeFromEdge(hypergraph, node_idx, edge_idx):
  """hypergraph_util.py:47-58."""
  assert node_idx in hypergraph.node
  assert edge_idx in hypergraph.node[node_idx].edges
  assert edge_idx in hypergraph.edge
  assert node_idx in hypergraph.edge[edge_idx].nodes
  hypergraph.node[node_idx].edges.remove(edge_idx)
  hypergraph.edge[edge_idx].nodes.remove(node_idx)
  if len(hypergraph.node[node_idx].edges) == 0:
    hypergraph.node.pop(node_idx)
  if len(hypergraph.edge[edge_idx].nodes) == 0:
    hypergraph.edge.pop(edge_idx)


def RemoveNode(hypergraph, node_idx):
  """hypergraph_util.py:288-294."""
  assert node_idx in hypergraph.node
  for edge_idx in list(hypergraph.node[node_idx].edges):
    RemoveNodeFromEdge(hypergraph, node_idx, edge_idx)


def RemoveEdge(hypergraph, edge_idx):
  """hypergraph_util.py:297-303."""
  assert edge_idx in hypergraph.edge
  for node_idx in list(hypergraph.edge[edge_idx].nodes):
    RemoveNodeFromEdge(hypergraph, node_idx, edge_idx)


def CreateRandomHyperGraph(num_nodes, num_edges, probability):
  """hypergraph_util.py:61-75 (uses Python's ``random`` like the reference)."""
  assert 0 <= probability <= 1
  assert num_edges >= 0
  assert num_nodes >= 0
  result = Hypergraph()
  for i in range(num_nodes):
    for j in range(num_edges):
      if random() < probability:
        AddNodeToEdge(result, i, j)
  return result


def FromSparseMatrix(sparse_matrix):
  """Rows = nodes, cols = edges (hypergraph_util.py:78-88)."""
  res = Hypergraph()
  rows, cols = sparse_matrix.nonzero()
  for r, c in zip(rows, cols):
    AddNodeToEdge(res, int(r), int(c))
  return res


def IsEmpty(hypergraph):
  """hypergraph_util.py:91-93."""
  return len(hypergraph.node) == 0 or len(hypergraph.edge) == 0


def _coo(hypergraph, edge_major):
  rows, cols = [], []
  if edge_major:
    for edge_idx, edge in hypergraph.edge.items():
      rows.extend([edge_idx] * len(edge.nodes))
      cols.extend(edge.nodes)
  else:
    for node_idx, node in hypergraph.node.items():
      rows.extend([node_idx] * len(node.edges))
      cols.extend(node.edges)
  return rows, cols


def ToCsrMatrix(hypergraph):
  """Bool CSR, row i = node i, col j = edge j (hypergraph_util.py:96-114)."""
  if IsEmpty(hypergraph):
    return sp.sparse.csr_matrix([])
  rows, cols = _coo(hypergraph, edge_major=False)
  return sp.sparse.csr_matrix(([1] * len(rows), (rows, cols)), dtype=bool)


def ToEdgeCsrMatrix(hypergraph):
  """Bool CSR, row j = edge j, col i = node i (hypergraph_util.py:117-135)."""
  if IsEmpty(hypergraph):
    return sp.sparse.csr_matrix([])
  rows, cols = _coo(hypergraph, edge_major=True)
  return sp.sparse.csr_matrix(([1] * len(rows), (rows, cols)), dtype=bool)


def ToCscMatrix(hypergraph):
  """hypergraph_util.py:138-156."""
  if IsEmpty(hypergraph):
    return sp.sparse.csc_matrix([])
  rows, cols = _coo(hypergraph, edge_major=False)
  return sp.sparse.csc_matrix(([1] * len(rows), (rows, cols)), dtype=bool)


def Relabel(original_hg, node_map, edge_map):
  """hypergraph_util.py:198-220: relabel through the maps, keep weights."""
  relabed_hg = Hypergraph()
  if original_hg.HasField("name"):
    relabed_hg.name = original_hg.name
  for node_idx, node in original_hg.node.items():
    for edge_idx in node.edges:
      assert node_idx in node_map
      assert edge_idx in edge_map
      AddNodeToEdge(relabed_hg, node_map[node_idx], edge_map[edge_idx])
  for node_idx, node in original_hg.node.items():
    relabed_hg.node[node_map[node_idx]].weight = node.weight
  for edge_idx, edge in original_hg.edge.items():
    relabed_hg.edge[edge_map[edge_idx]].weight = edge.weight
  return relabed_hg


def CompressRange(original_hg):
  """Sorted ids -> 0..n-1; returns (compressed, inv_node_map, inv_edge_map)
  (hypergraph_util.py:223-244)."""
  node_indices = sorted(original_hg.node)
  edge_indices = sorted(original_hg.edge)
  node_map = {n: i for i, n in enumerate(node_indices)}
  edge_map = {e: i for i, e in enumerate(edge_indices)}
  compressed_hg = Relabel(original_hg, node_map, edge_map)
  inv_node_map = {y: x for x, y in node_map.items()}
  inv_edge_map = {y: x for x, y in edge_map.items()}
  return compressed_hg, inv_node_map, inv_edge_map


################################################################################
# Device-ready incidence (new)                                                 #
################################################################################


def _csr_from_pairs(nrow, rows, cols):
  """Sorted, de-duplicated int32 CSR from (row, col) int64 arrays."""
  if rows.size:
    key = rows.astype(np.int64) * (int(cols.max()) + 1) + cols
    key = np.unique(key)
    ncol_span = int(cols.max()) + 1
    rows = (key // ncol_span).astype(np.int64)
    cols = (key % ncol_span).astype(np.int32)
  rp = np.zeros(nrow + 1, dtype=np.int64)
  np.add.at(rp, rows + 1, 1)
  rp = np.cumsum(rp)
  if rp[-1] >= 2**31:
    raise ValueError("incidence count exceeds int32 CSR range")
  return rp.astype(np.int32), cols.astype(np.int32)


class Incidence:
  """Compressed incidence matrix in both orientations (int32 CSR, sorted cols).

  rp_n/col_n  = ToCsrMatrix(CompressRange(hg)[0])      (N x E)
  rp_e/col_e  = ToEdgeCsrMatrix(CompressRange(hg)[0])  (E x N)
  node_ids/edge_ids = inverse maps (compressed index -> original id)
  node_weight/edge_weight = float32 proto weights in compressed order.
  """

  def __init__(self, N, E, rp_n, col_n, rp_e=None, col_e=None, node_ids=None,
               edge_ids=None, node_weight=None, edge_weight=None):
    self.N = int(N)
    self.E = int(E)
    self.rp_n = np.ascontiguousarray(rp_n, dtype=np.int32)
    self.col_n = np.ascontiguousarray(col_n, dtype=np.int32)
    if rp_e is None:
      rp_e, col_e = self._transpose()
    self.rp_e = np.ascontiguousarray(rp_e, dtype=np.int32)
    self.col_e = np.ascontiguousarray(col_e, dtype=np.int32)
    self.node_ids = (np.arange(self.N, dtype=np.int64)
                     if node_ids is None else np.asarray(node_ids, np.int64))
    self.edge_ids = (np.arange(self.E, dtype=np.int64)
                     if edge_ids is None else np.asarray(edge_ids, np.int64))
    self.node_weight = (np.ones(self.N, np.float32) if node_weight is None
                        else np.asarray(node_weight, np.float32))
    self.edge_weight = (np.ones(self.E, np.float32) if edge_weight is None
                        else np.asarray(edge_weight, np.float32))
    assert self.rp_n.shape == (self.N + 1,)
    assert self.rp_e.shape == (self.E + 1,)

  @property
  def nnz(self):
    return int(self.rp_n[-1])

  def _transpose(self):
    rows = np.repeat(np.arange(self.N, dtype=np.int64), np.diff(self.rp_n))
    order = np.lexsort((rows, self.col_n))  # stable: by col, then row
    col_e = rows[order].astype(np.int32)
    rp_e = np.zeros(self.E + 1, dtype=np.int64)
    np.add.at(rp_e, self.col_n.astype(np.int64) + 1, 1)
    return np.cumsum(rp_e).astype(np.int32), col_e

  def node_degree(self):
    return np.diff(self.rp_n)

  def edge_size(self):
    return np.diff(self.rp_e)

  def to_scipy(self):
    a = sp.sparse.csr_matrix(
        (np.ones(self.nnz, dtype=bool), self.col_n, self.rp_n),
        shape=(self.N, self.E))
    at = sp.sparse.csr_matrix(
        (np.ones(self.nnz, dtype=bool), self.col_e, self.rp_e),
        shape=(self.E, self.N))
    return a, at

  @staticmethod
  def from_hypergraph(hypergraph):
    """CompressRange + ToCsrMatrix + ToEdgeCsrMatrix in one vectorised pass.

    Follows Relabel (hypergraph_util.py:208-212): the incidence set is the
    union of every node's ``edges`` list; edge keys that no node references
    stay as empty rows, as do nodes without edges.
    """
    node_ids = np.array(sorted(hypergraph.node), dtype=np.int64)
    edge_ids = np.array(sorted(hypergraph.edge), dtype=np.int64)
    N, E = node_ids.size, edge_ids.size
    rows, cols = [], []
    for node_idx, node in hypergraph.node.items():
      rows.append(np.full(len(node.edges), node_idx, dtype=np.int64))
      cols.append(np.fromiter(node.edges, dtype=np.int64, count=len(node.edges)))
    rows = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    cols = np.concatenate(cols) if cols else np.zeros(0, np.int64)
    r = np.searchsorted(node_ids, rows)
    c = np.searchsorted(edge_ids, cols)
    assert np.all(c < E) and np.all(edge_ids[c] == cols), \
        "node lists an edge id missing from hypergraph.edge"
    rp_n, col_n = _csr_from_pairs(N, r, c)
    node_weight = np.array([hypergraph.node[int(i)].weight for i in node_ids],
                           dtype=np.float32)
    edge_weight = np.array([hypergraph.edge[int(i)].weight for i in edge_ids],
                           dtype=np.float32)
    return Incidence(N, E, rp_n, col_n, node_ids=node_ids, edge_ids=edge_ids,
                     node_weight=node_weight, edge_weight=edge_weight)

  @staticmethod
  def from_scipy(node2edge):
    """From an N x E sparse matrix (rows = nodes), no id remapping."""
    a = sp.sparse.csr_matrix(node2edge, dtype=bool)
    a.sum_duplicates()
    a.sort_indices()
    return Incidence(a.shape[0], a.shape[1], a.indptr, a.indices)
