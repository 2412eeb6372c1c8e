"""Embedding entry points (reference: hypergraph_embedding/embedding.py).

Registry and signatures kept for the FOBE/HOBE path: ``Embed(args, hg)``
(81-107), ``EMBEDDING_OPTIONS`` (423-444) with "ALG_DIST",
"HG2V_BOOLEAN", "HG2V_ALG_DIST", "HG2V_BOOLEAN_NS", "HG2V_ADJ_JAC",
"HG2V_NEIGH_JAC", ``EmbedHg2vBoolean`` (308-329), ``EmbedHg2vAdjJaccard``
(330-355), ``EmbedHg2vNeighborhoodWeightedJaccard`` (358-386),
``EmbedHg2vAlgDist`` (389-416), ``CombineEmbeddings`` (51-78).

``_hypergraph2vec_skeleton`` (269-305) runs entirely on one device context:
incidence upload -> sampler -> records stay in HBM -> tables initialised on
device -> Keras-semantics fit -> rows idx+1 copied into the proto.
The reference's other methods (SVD, NMF, node2vec, auto-encoder) are
outside this hot path: their keys raise like the reference's
``method_not_supported`` (419-420).
"""

import logging

import numpy as np

from . import _hgx
from .algebraic_distance import EmbedAlgebraicDistance, coords_to_embedding
from .combine_embeddings_util import (CombineEmbeddingsViaConcatenation,
                                      CombineEmbeddingsViaNodeEdgeClassifier)
from .hg2v_model import Hg2vModel
from .hg2v_sample import _quotas, sample_fobe, sample_hobe, sample_jaccard
from .hypergraph_util import Incidence
from .proto import HypergraphEmbedding
from .runtime import get_context, numpy_seed

log = logging.getLogger()

COMBINATION_OPTIONS = [
    "N_E_SUPERVISED",  # default @ 0 (reference)
    "N_E_SEMI_SUPERVISED",
    "CONCATENATE",
]


def CombineEmbeddings(args, hypergraph, embeddings, disable_pbar=False):
  """embedding.py:51-78: CONCATENATE, or the node/edge-classifier MLP
  combiners (N_E_SUPERVISED, N_E_SEMI_SUPERVISED) on the MI355X dense-MLP
  engine (combine_embeddings_util.py)."""
  assert len(embeddings) >= 1
  if len(embeddings) == 1:
    return embeddings[0]
  strategy = args.embedding_combination_strategy
  if strategy == "CONCATENATE":
    comb = CombineEmbeddingsViaConcatenation(hypergraph, embeddings)
    args.embedding_dimension = comb.dim
  elif strategy in ("N_E_SUPERVISED", "N_E_SEMI_SUPERVISED"):
    comb = CombineEmbeddingsViaNodeEdgeClassifier(
        hypergraph, embeddings, args.embedding_dimension,
        with_auto_encoder=strategy == "N_E_SEMI_SUPERVISED",
        disable_pbar=disable_pbar)
  else:
    raise ValueError("Args contains an illegal embedding-combination-strategy")
  comb.method_name = "_".join(args.embedding_method)
  return comb


def Embed(args, hypergraph, shortcut_embeddings=None):
  """embedding.py:81-107."""
  assert min(len(hypergraph.node), len(hypergraph.edge)) > \
      args.embedding_dimension
  assert len(args.embedding_method) >= 1
  embeddings = []
  for method in args.embedding_method:
    if shortcut_embeddings is not None and method in shortcut_embeddings:
      embeddings.append(shortcut_embeddings[method])
      continue
    log.info("Embedding using method %s with %i dim", method,
             args.embedding_dimension)
    if getattr(args, "embedding_debug_summary", None):
      embeddings.append(EMBEDDING_OPTIONS[method](
          hypergraph, args.embedding_dimension,
          debug_summary_path=args.embedding_debug_summary))
    else:
      embeddings.append(EMBEDDING_OPTIONS[method](hypergraph,
                                                  args.embedding_dimension))
  embedding = CombineEmbeddings(args, hypergraph, embeddings)
  log.info("Embedding contains %i node and %i edge vectors",
           len(embedding.node), len(embedding.edge))
  return embedding


def _plot_distributions(path, records):
  """PlotDistributions (hg2v_sample.py:805-853): histograms of the three
  target kinds of the record stream."""
  import matplotlib
  matplotlib.use("Agg")
  import matplotlib.pyplot as plt
  idx, tgt = records.arrays()
  nn = (idx[:, 0] > 0) & (idx[:, 2] > 0)
  ee = (idx[:, 1] > 0) & (idx[:, 3] > 0)
  ne = ~(nn | ee)
  fig, axes = plt.subplots(3, 1, figsize=(8.5, 11))
  for ax, sel, col, title in ((axes[0], nn, 0, "Node-Node"),
                              (axes[1], ee, 1, "Edge-Edge"),
                              (axes[2], ne, 2, "Node-Edge")):
    ax.set_title(f"{title} Probability Distribution")
    ax.hist(tgt[sel, col])
    ax.set_yscale("log")
  fig.tight_layout()
  fig.savefig(str(path))


# Records resident at once before the skeleton streams the record stream in
# row-range chunks (68 B per record at K = 5: 2^30 records = 73 GB of HBM).
RECORDS_BUDGET = 1 << 30


def _row_chunks(inc, bound_per_row, budget):
  """Split node rows and edge rows into n contiguous ranges so that each
  chunk's record upper bound (bound_per_row per node row and per edge row)
  stays within `budget`."""
  total = bound_per_row * (inc.N + inc.E)
  n = max(1, -(-total // budget))
  nodes = [(inc.N * c // n, inc.N * (c + 1) // n) for c in range(n)]
  edges = [(inc.E * c // n, inc.E * (c + 1) // n) for c in range(n)]
  return list(zip(nodes, edges))


def _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors, sampler_fn,
                             loss, act, fit_batch_size, fit_epochs,
                             debug_summary_path, disable_pbar, ctx=None,
                             chunk_sampler_fn=None, bound_per_row=0,
                             records_budget=None):
  """embedding.py:269-305, device-resident end to end. `hypergraph` is the
  reference's Hypergraph message or an already compressed Incidence (e.g.
  proto_native.read_incidence of a file too large for Python protobuf)."""
  del disable_pbar
  ctx = ctx or get_context()
  if isinstance(hypergraph, Incidence):
    inc = hypergraph
  else:
    inc = Incidence.from_hypergraph(hypergraph)  # CompressRange + CSR
  budget = RECORDS_BUDGET if records_budget is None else records_budget
  if callable(bound_per_row):  # a bound that depends on the incidence
    bound_per_row = bound_per_row(inc)
  if chunk_sampler_fn is not None and bound_per_row * (inc.N + inc.E) > budget:
    # the stream does not fit: sample and train row-range chunks in turn
    chunks = _row_chunks(inc, bound_per_row, budget)
    seed = numpy_seed()
    prep = chunk_sampler_fn(inc, ctx)
    model = Hg2vModel(inc.N + 1, inc.E + 1, dimension, num_neighbors, loss,
                      act, ctx=ctx)
    model.fit_streaming(lambda c: prep(seed, *chunks[c]), len(chunks),
                        batch_size=fit_batch_size, epochs=fit_epochs)
    node_w, edge_w = model.get_weights()
    return coords_to_embedding(inc, node_w[1:], edge_w[1:], dimension, "")
  records = sampler_fn(inc, ctx)
  if debug_summary_path is not None:
    _plot_distributions(debug_summary_path, records)
  model = Hg2vModel(inc.N + 1, inc.E + 1, dimension, num_neighbors, loss, act,
                    ctx=ctx)  # rows = max compressed idx + 2
  model.fit(batch_size=fit_batch_size, epochs=fit_epochs)
  node_w, edge_w = model.get_weights()
  return coords_to_embedding(inc, node_w[1:], edge_w[1:], dimension, "")


def EmbedHg2vBoolean(hypergraph, dimension, num_neighbors=5, num_samples=200,
                     batch_size=256, epochs=10, neg_samples=0,
                     debug_summary_path=None, disable_pbar=False,
                     records_budget=None):
  """FOBE: BooleanSamples + BooleanModel (embedding.py:308-329). A stream of
  more than `records_budget` records is sampled and trained in row-range
  chunks (Hg2vModel.fit_streaming)."""
  sampler_fn = lambda inc, ctx: sample_fobe(inc, num_neighbors, num_samples,
                                            neg_samples, ctx=ctx)

  def chunk_sampler_fn(inc, ctx):
    ctx.upload(inc)
    q = [_quotas(w, n) for w in (inc.node_weight, inc.edge_weight)
         for n in (num_samples, neg_samples)]

    def chunk(seed, nodes, edges):
      nq, gnq, eq, geq = (np.zeros_like(x) for x in q)
      nq[nodes[0]:nodes[1]] = q[0][nodes[0]:nodes[1]]
      gnq[nodes[0]:nodes[1]] = q[1][nodes[0]:nodes[1]]
      eq[edges[0]:edges[1]] = q[2][edges[0]:edges[1]]
      geq[edges[0]:edges[1]] = q[3][edges[0]:edges[1]]
      neg = neg_samples > 0
      return ctx.sample_fobe(seed, num_neighbors, nq, eq, gnq if neg else None,
                             geq if neg else None)
    return chunk

  # per row at most q nn (or ee) and q node-edge records, q = int(w * S)
  # (hg2v_sample.py:138-194), plus 3 negative blocks of int(w * neg_samples),
  # w the largest node / edge weight of the compressed incidence (any float
  # in the proto, default 1)
  def bound_per_row(inc):
    wmax = float(max(np.max(inc.node_weight, initial=0.0),
                     np.max(inc.edge_weight, initial=0.0), 0.0))
    return int(wmax * 2 * num_samples) + int(wmax * 3 * neg_samples) + 2

  emb = _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                 sampler_fn, _hgx.LOSS_KLD, _hgx.ACT_SIGMOID,
                                 batch_size, epochs, debug_summary_path,
                                 disable_pbar, chunk_sampler_fn=chunk_sampler_fn,
                                 bound_per_row=bound_per_row,
                                 records_budget=records_budget)
  emb.method_name = "HG2V_BOOLEAN"
  return emb


def EmbedHg2vAlgDist(hypergraph, dimension, alpha=0, num_neighbors=5,
                     num_samples=200, batch_size=256, epochs=10,
                     debug_summary_path=None, disable_pbar=False,
                     records_budget=None):
  """HOBE: alg-dist (k=10, 20 iterations) + AlgebraicDistanceSamples +
  UnweightedFloatModel (embedding.py:389-416). `alpha` is accepted and, as
  in the reference, not used (_alpha_scale is called with alpha=0).
  A stream of more than `records_budget` records (RECORDS_BUDGET) is
  sampled and trained in row-range chunks (Hg2vModel.fit_streaming)."""
  del alpha

  def alg_dist(inc, ctx):
    x0 = np.random.random((inc.N, 10))  # algebraic_distance.py:140-141
    y0 = np.random.random((inc.E, 10))
    ctx.upload(inc)
    ctx.alg_set(x0, y0)
    ctx.alg_run(20)  # coords stay resident for the HOBE probabilities

  def sampler_fn(inc, ctx):
    alg_dist(inc, ctx)
    return sample_hobe(inc, num_neighbors, num_samples, ctx=ctx)

  def chunk_sampler_fn(inc, ctx):
    alg_dist(inc, ctx)

    def chunk(seed, nodes, edges):
      nq = np.zeros(inc.N, np.int32)
      eq = np.zeros(inc.E, np.int32)
      nq[nodes[0]:nodes[1]] = num_samples
      eq[edges[0]:edges[1]] = num_samples
      return ctx.sample_hobe(seed, num_neighbors, num_samples, node_q=nq,
                             edge_q=eq)
    return chunk

  # per row at most S nn (or ee) and S node-edge records (hg2v_sample.py:659-703)
  emb = _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                 sampler_fn, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                                 batch_size, epochs, debug_summary_path,
                                 disable_pbar, chunk_sampler_fn=chunk_sampler_fn,
                                 bound_per_row=2 * num_samples,
                                 records_budget=records_budget)
  emb.method_name = "HG2V_ALG_DIST"
  return emb


def _jaccard_embed(hypergraph, dimension, which, alpha, num_neighbors,
                   num_samples, batch_size, epochs, debug_summary_path,
                   disable_pbar):
  """embedding.py:330-386: WeightedJaccardSamples over UniformWeight or
  WeightByNeighborhood features, UnweightedFloatModel (relu, MSE)."""

  def sampler_fn(inc, ctx):
    ctx.upload(inc)
    fn, fe = ctx.incidence_weights(which, float(alpha))
    return sample_jaccard(inc, fn, fe, num_neighbors, num_samples, ctx=ctx)

  return _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                  sampler_fn, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                                  batch_size, epochs, debug_summary_path,
                                  disable_pbar)


def EmbedHg2vAdjJaccard(hypergraph, dimension, num_neighbors=5,
                        num_samples=200, batch_size=256, epochs=10,
                        debug_summary_path=None, disable_pbar=False):
  """embedding.py:330-355 (UniformWeight features)."""
  emb = _jaccard_embed(hypergraph, dimension, _hgx.WEIGHT_UNIFORM, 0.0,
                       num_neighbors, num_samples, batch_size, epochs,
                       debug_summary_path, disable_pbar)
  emb.method_name = "HG2V_ADJ_JAC"
  return emb


def EmbedHg2vNeighborhoodWeightedJaccard(hypergraph, dimension, alpha=0,
                                         num_neighbors=5, num_samples=200,
                                         batch_size=256, epochs=10,
                                         debug_summary_path=None,
                                         disable_pbar=False):
  """embedding.py:358-386 (WeightByNeighborhood(alpha) features)."""
  assert 0 <= alpha <= 1
  emb = _jaccard_embed(hypergraph, dimension, _hgx.WEIGHT_NEIGHBORHOOD, alpha,
                       num_neighbors, num_samples, batch_size, epochs,
                       debug_summary_path, disable_pbar)
  emb.method_name = "HG2V_NEIGH_JAC"
  return emb


def method_not_supported(hypergraph, dim, **kwargs):
  raise RuntimeError(
      "Method not supported. Try making the embedding on your own.")


EMBEDDING_OPTIONS = {
    "ALG_DIST": EmbedAlgebraicDistance,
    "HG2V_BOOLEAN": EmbedHg2vBoolean,
    "HG2V_ALG_DIST": EmbedHg2vAlgDist,
    "HG2V_BOOLEAN_NS": lambda h, d, **kw: EmbedHg2vBoolean(h, d, neg_samples=500,
                                                           **kw),
    # outside the FOBE/HOBE hot path (SURVEY §2 "OUT OF SCOPE")
    "SVD": method_not_supported,
    "RANDOM": method_not_supported,
    "NMF": method_not_supported,
    "AUTO_ENCODER": method_not_supported,
    "N2V3_BIPARTIDE": method_not_supported,
    "N2V3_CLIQUE": method_not_supported,
    "N2V5_BIPARTIDE": method_not_supported,
    "N2V5_CLIQUE": method_not_supported,
    "N2V7_BIPARTIDE": method_not_supported,
    "N2V7_CLIQUE": method_not_supported,
    "HG2V_ADJ_JAC": EmbedHg2vAdjJaccard,
    "HG2V_NEIGH_JAC": EmbedHg2vNeighborhoodWeightedJaccard,
    "metapath2vec++": method_not_supported,
    "deepwalk": method_not_supported,
    "LINE": method_not_supported,
    "BiNE": method_not_supported,
}

DEBUG_SUMMARY_OPTIONS = {"HG2V_BOOLEAN", "HG2V_ALG_DIST", "HG2V_ADJ_JAC",
                         "HG2V_NEIGH_JAC"}

__all__ = ["Embed", "EMBEDDING_OPTIONS", "DEBUG_SUMMARY_OPTIONS",
           "COMBINATION_OPTIONS", "CombineEmbeddings", "EmbedHg2vBoolean",
           "EmbedHg2vAlgDist", "EmbedAlgebraicDistance", "EmbedHg2vAdjJaccard",
           "EmbedHg2vNeighborhoodWeightedJaccard",
           "CombineEmbeddingsViaConcatenation", "method_not_supported"]
