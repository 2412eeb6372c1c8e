"""Embedding combiners (reference: hypergraph_embedding/combine_embeddings_util.py).

``CombineEmbeddingsViaConcatenation`` (27-41) and
``CombineEmbeddingsViaNodeEdgeClassifier`` (80-174), the N_E_SUPERVISED /
N_E_SEMI_SUPERVISED strategies of ``CombineEmbeddings`` -- the C5 ensemble's
default. The combiner trains on the MI355X dense-MLP engine
(csrc/hgx_mlp.hip): the concatenated node and edge embeddings are uploaded
once as two tables, samples are (node row, edge row, label) triples, and
the first layer gathers its input rows and applies Dropout(0.5) itself, so
the reference's per-sample Python lists of concatenated vectors
(6 x nnz x 2 x input_size floats) never exist.

Samples (_sample_hypergraph, 46-67): every (node, edge) incidence in node map
order labelled 1, then ``SampleMissingConnections(hypergraph, 5 *
num_pos)`` labelled 0 (Python-``random``-exact, evaluation_util.py).
Model: per side Dropout(0.5) -> Dense((in + d) // 2, relu) ->
Dense(d, sigmoid) ["JointNode"/"JointEdge"]; Concatenate -> Dense(d, relu)
-> Dense(1, sigmoid); with the auto-encoder, per side joint ->
Dense(h, relu) -> Dense(in, relu) reproducing the input, loss weights
[4, 1, 1]. MSE, Adagrad, batch 256, 100 epochs, EarlyStopping(loss).
The embedding is JointNode / JointEdge of every node / edge (no dropout).

Scale (C5: 10M x 5M, 2e8 incidences, 1.2e9 samples per epoch). The
`hypergraph` may be an :class:`Incidence` (proto_native.read_incidence; the
only practical C4 input) and the embeddings ShardedEmbeddings (what the
embedders return past protobuf's 2 GiB limit). Then nothing is per id or
per incidence in Python: the tables are the embeddings' rows gathered by
id and concatenated with one np.concatenate, the positives are the CSR
itself (row i's edges in column order: the order of the equivalent proto
with ascending ids), the negatives come from SampleMissingConnections'
native restatement fed the CSR arrays, and the result is built from the
joint tables by proto_native (a ShardedEmbedding past the limit).
"""

import logging
import random

import numpy as np

from . import _hgx
from .dense_mlp import NE_SEMI_SUPERVISED, NE_SUPERVISED, DenseModel
from .evaluation_util import _missing_positions
from .hypergraph_util import Incidence
from .proto import HypergraphEmbedding

log = logging.getLogger()


def _concatenated_table(indices, half_embeddings):
  """_concatenate_embeddings (combine_embeddings_util.py:15-24) as one
  (len(indices) x sum(dims)) float32 table in `indices` order."""
  indices = list(indices)
  rows = [[v for emb in half_embeddings for v in emb[idx].values]
          for idx in indices]
  return indices, np.asarray(rows, np.float32).reshape(len(indices), -1)


def _tables_of(inc, embeddings):
  """Node / edge tables (compressed order) of the embeddings, concatenated
  side by side (_concatenate_embeddings, combine_embeddings_util.py:15-24)."""
  from .hg2v_weighting import _rows_of
  nt = np.concatenate([_rows_of(e.node, inc.node_ids) for e in embeddings], 1)
  et = np.concatenate([_rows_of(e.edge, inc.edge_ids) for e in embeddings], 1)
  return nt, et


def CombineEmbeddingsViaConcatenation(hypergraph, embeddings):
  """combine_embeddings_util.py:27-41."""
  if isinstance(hypergraph, Incidence):
    from .algebraic_distance import coords_to_embedding
    nt, et = _tables_of(hypergraph, embeddings)
    return coords_to_embedding(hypergraph, nt, et, nt.shape[1], "")
  emb = HypergraphEmbedding()
  emb.dim = sum(e.dim for e in embeddings)
  nodes, nt = _concatenated_table(hypergraph.node, [e.node for e in embeddings])
  edges, et = _concatenated_table(hypergraph.edge, [e.edge for e in embeddings])
  for i, node_idx in enumerate(nodes):
    emb.node[node_idx].values.extend(nt[i].tolist())
  for i, edge_idx in enumerate(edges):
    emb.edge[edge_idx].values.extend(et[i].tolist())
  return emb


def combine_node_edge_classifier(node_tab, edge_tab, node_row, edge_row, label,
                                 desired_dim, with_auto_encoder, epochs=100,
                                 perms=None, ctx=None):
  """Array-level combiner: tables (rows x input_size), samples as table rows
  + labels. Returns (node joint rows, edge joint rows, epoch losses, engine
  stats of the fit)."""
  in_dim = node_tab.shape[1]
  assert desired_dim > 0
  kind = NE_SEMI_SUPERVISED if with_auto_encoder else NE_SUPERVISED
  model = DenseModel(kind, in_dim, desired_dim, ctx=ctx)
  model.set_tables(node_tab, edge_tab)
  losses = model.fit(node_row, edge_row, label, epochs=epochs, min_delta=0.0,
                     perms=perms)
  st = model.stats()
  jn = model.predict_joint(1, np.arange(node_tab.shape[0], dtype=np.int32))
  je = model.predict_joint(2, np.arange(edge_tab.shape[0], dtype=np.int32))
  model.close()
  return jn, je, losses, st


def incidence_samples(inc, max_positives=None, rs=None):
  """_sample_hypergraph (combine_embeddings_util.py:46-67) on the CSR: every
  incidence (row order, columns ascending) labelled 1, then
  SampleMissingConnections' 5 x num_pos draws (Python-`random`-exact,
  fed the CSR arrays) labelled 0. max_positives (not in the reference: a
  bounded slice for tests and benches) keeps a seeded random subset of the
  incidences, in CSR order. Returns (node_row, edge_row, label)."""
  pos_n = np.repeat(np.arange(inc.N, dtype=np.int32), np.diff(inc.rp_n))
  pos_e = np.ascontiguousarray(inc.col_n, np.int32)
  if max_positives is not None and max_positives < pos_n.size:
    rs = rs or np.random.mtrand._rand
    pick = np.sort(rs.choice(pos_n.size, max_positives, replace=False))
    pos_n, pos_e = pos_n[pick], pos_e[pick]
  num_pos = pos_n.size
  assert 5 * num_pos < inc.N * inc.E
  npos, epos = _hgx.pyrandom_sample_missing(
      random._inst, inc.N, inc.E, np.asarray(inc.rp_n, np.int64), inc.col_n,
      5 * num_pos)
  if len(npos) < 5 * num_pos:
    log.critical("SampleMissingConnections failed to find %i samples",
                 5 * num_pos)
  node_row = np.concatenate([pos_n, npos.astype(np.int32)])
  edge_row = np.concatenate([pos_e, epos.astype(np.int32)])
  label = np.concatenate([np.ones(num_pos, np.float32),
                          np.zeros(len(npos), np.float32)])
  return node_row, edge_row, label


def proto_samples(hypergraph, nodes, edges):
  """_sample_hypergraph (combine_embeddings_util.py:46-67) on a Hypergraph
  message: every (node, edge) in node map order labelled 1, then the
  SampleMissingConnections(hypergraph, 5 * num_pos) draws in insertion order
  labelled 0 (the set's iteration order only permutes samples that fit
  shuffles anyway), as rows of the `nodes` / `edges` tables."""
  nrow = {n: i for i, n in enumerate(nodes)}
  erow = {e: i for i, e in enumerate(edges)}
  pos_n, pos_e = [], []
  for node_idx, node in hypergraph.node.items():
    for edge_idx in node.edges:
      pos_n.append(nrow[node_idx])
      pos_e.append(erow[edge_idx])
  num_pos = len(pos_n)
  mnodes, medges, npos, epos = _missing_positions(hypergraph, 5 * num_pos)
  if len(npos) < 5 * num_pos:
    log.critical("SampleMissingConnections failed to find %i samples",
                 5 * num_pos)
  node_row = np.concatenate([np.asarray(pos_n, np.int32),
                             np.array([nrow[mnodes[p]] for p in npos], np.int32)])
  edge_row = np.concatenate([np.asarray(pos_e, np.int32),
                             np.array([erow[medges[q]] for q in epos], np.int32)])
  label = np.concatenate([np.ones(num_pos, np.float32),
                          np.zeros(len(npos), np.float32)])
  return node_row, edge_row, label


# seconds of the last CombineEmbeddingsViaNodeEdgeClassifier on an
# Incidence: host preparation (tables + samples), device fit, joint rows
last_timings = {}


def CombineEmbeddingsViaNodeEdgeClassifier(hypergraph, embeddings, desired_dim,
                                           with_auto_encoder, disable_pbar,
                                           epochs=100, max_positives=None):
  """combine_embeddings_util.py:80-174 on the MI355X dense-MLP engine.
  `epochs` (the reference's fixed 100) and `max_positives`
  (incidence_samples) are extensions for bounded runs."""
  del disable_pbar
  assert desired_dim > 0
  if isinstance(hypergraph, Incidence):
    import time
    from .algebraic_distance import coords_to_embedding
    inc = hypergraph
    t0 = time.perf_counter()
    nt, et = _tables_of(inc, embeddings)
    node_row, edge_row, label = incidence_samples(inc, max_positives)
    t1 = time.perf_counter()
    jn, je, _, _ = combine_node_edge_classifier(
        nt, et, node_row, edge_row, label, desired_dim, with_auto_encoder,
        epochs=epochs)
    del nt, et
    t2 = time.perf_counter()
    out = coords_to_embedding(inc, jn, je, desired_dim, "")
    last_timings.update(prep_s=t1 - t0, fit_and_joint_s=t2 - t1,
                        output_s=time.perf_counter() - t2,
                        samples=int(label.size))
    return out
  nodes, nt = _concatenated_table(hypergraph.node, [e.node for e in embeddings])
  edges, et = _concatenated_table(hypergraph.edge, [e.edge for e in embeddings])
  node_row, edge_row, label = proto_samples(hypergraph, nodes, edges)
  jn, je, _, _ = combine_node_edge_classifier(nt, et, node_row, edge_row, label,
                                              desired_dim, with_auto_encoder,
                                              epochs=epochs)
  embedding = HypergraphEmbedding()
  embedding.dim = desired_dim
  for i, node_idx in enumerate(nodes):
    embedding.node[node_idx].values.extend(jn[i].tolist())
  for i, edge_idx in enumerate(edges):
    embedding.edge[edge_idx].values.extend(je[i].tolist())
  return embedding
