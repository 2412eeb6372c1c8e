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
from .hg2v_sample import (_quotas, row_class_quota, sample_fobe, sample_hobe,
                          sample_jaccard)
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
  engine (combine_embeddings_util.py). `hypergraph` may be an Incidence
  and the embeddings ShardedEmbeddings (C5 scale); the optional
  `args.combination_kwargs` dict (not in the reference) reaches the
  classifier combiner (epochs, max_positives)."""
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
        disable_pbar=disable_pbar,
        **(getattr(args, "combination_kwargs", None) or {}))
  else:
    raise ValueError("Args contains an illegal embedding-combination-strategy")
  comb.method_name = "_".join(args.embedding_method)
  return comb


def Embed(args, hypergraph, shortcut_embeddings=None):
  """embedding.py:81-107. `hypergraph` is the reference's Hypergraph
  message or an Incidence (proto_native.read_incidence: C4/C5 inputs Python
  protobuf cannot hold). The optional `args.embedding_kwargs` dict (not in
  the reference) maps a method name to extra keyword arguments of its
  embedder (e.g. epochs, records_budget, row quotas for bounded runs)."""
  if isinstance(hypergraph, Incidence):
    n_nodes, n_edges = hypergraph.N, hypergraph.E
  else:
    n_nodes, n_edges = len(hypergraph.node), len(hypergraph.edge)
  assert min(n_nodes, n_edges) > args.embedding_dimension
  assert len(args.embedding_method) >= 1
  extra = getattr(args, "embedding_kwargs", None) or {}
  embeddings = []
  for method in args.embedding_method:
    if shortcut_embeddings is not None and method in shortcut_embeddings:
      embeddings.append(shortcut_embeddings[method])
      continue
    log.info("Embedding using method %s with %i dim", method,
             args.embedding_dimension)
    kw = dict(extra.get(method, {}))
    if getattr(args, "embedding_debug_summary", None):
      kw["debug_summary_path"] = args.embedding_debug_summary
    embeddings.append(EMBEDDING_OPTIONS[method](hypergraph,
                                                args.embedding_dimension, **kw))
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
# row chunks (68 B per record at K = 5: 2^30 records = 73 GB of HBM).
RECORDS_BUDGET = 1 << 30


# CUs of the sampling context when a streamed epoch samples chunk c + 1
# beside chunk c's training (0: sample and train in turn on one context).
# 192 of MI355X's 256: the trainer keeps 64 CUs (one per workgroup of a
# batch step). Full C4 HOBE epoch (profiles/r04/c4_epoch/): 350 s in turn,
# 261 s at 192 / 262 s at 160 / 286 s at 128 sampler CUs, the batch step
# 9.28 -> 9.42 us, tables bit-identical.
STREAM_OVERLAP_CUS = 192


class _SideSampler:
  """The second context of an overlapped streamed epoch and its sampler."""

  def __init__(self, ctx, sample):
    self.ctx, self.sample = ctx, sample


def _bound(inc, per_row, row_quota, per_quota):
  """Record bound per row: `per_row`, or with row quotas (node, edge) their
  total times `per_quota` spread over the rows (the streaming decision and
  the chunk count only use bound x rows)."""
  if row_quota is None:
    return per_row
  tot = per_quota * (int(np.sum(row_quota[0], dtype=np.int64)) +
                     int(np.sum(row_quota[1], dtype=np.int64)))
  return max(1, -(-tot // max(inc.N + inc.E, 1)))


def _row_chunks(inc, bound_per_row, budget):
  """Split the rows into n strided classes (offset c, stride n: node rows
  and edge rows r = c mod n) so that each chunk's record upper bound
  (bound_per_row per node row and per edge row) stays within `budget`.
  Strided, not contiguous: every chunk is a uniform slice of the id space,
  so hub rows (low ids in the power-law generator; sorted or community
  ordered ids in real data) spread over all chunks, chunks cost the same to
  sample, and each chunk's shuffle window mixes the whole graph."""
  total = bound_per_row * (inc.N + inc.E)
  n = max(1, -(-total // budget))
  return [(c, n) for c in range(n)]


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
    # the stream does not fit: sample and train strided row chunks in turn
    chunks = _row_chunks(inc, bound_per_row, budget)
    seed = numpy_seed()
    cus = STREAM_OVERLAP_CUS
    side = None
    if cus:
      # chunk c + 1 sampled on a second context (its stream on `cus` CUs)
      # while chunk c trains on this one (the other CUs); the host hands
      # the chunks over (Hg2vModel.fit_streaming `side`)
      side_ctx = _hgx.Context(ctx.device)
      side_ctx.set_tuning("stream_cus", cus)
      ctx.set_tuning("stream_cus", -cus)
      prep = chunk_sampler_fn(inc, side_ctx)
      side = _SideSampler(side_ctx, lambda c: prep(seed, *chunks[c]))
    else:
      prep = chunk_sampler_fn(inc, ctx)
    try:
      model = Hg2vModel(inc.N + 1, inc.E + 1, dimension, num_neighbors, loss,
                        act, ctx=ctx)
      model.fit_streaming(lambda c: prep(seed, *chunks[c]), len(chunks),
                          batch_size=fit_batch_size, epochs=fit_epochs,
                          side=side)
      node_w, edge_w = model.get_weights()
    finally:
      if side is not None:
        ctx.set_tuning("stream_cus", 0)
        side.ctx.close()
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
                     records_budget=None, row_quota=None):
  """FOBE: BooleanSamples + BooleanModel (embedding.py:308-329). A stream of
  more than `records_budget` records is sampled and trained in strided row
  chunks (Hg2vModel.fit_streaming). row_quota = (node quotas, edge quotas)
  (not in the reference) replaces int(weight * S) per row: bounded runs."""
  sampler_fn = lambda inc, ctx: sample_fobe(inc, num_neighbors, num_samples,
                                            neg_samples, ctx=ctx,
                                            row_quota=row_quota)

  def chunk_sampler_fn(inc, ctx):
    ctx.upload(inc)
    if row_quota is not None:
      q = [np.asarray(row_quota[0], np.int32), _quotas(inc.node_weight, neg_samples),
           np.asarray(row_quota[1], np.int32), _quotas(inc.edge_weight, neg_samples)]
    else:
      q = [_quotas(w, n) for w in (inc.node_weight, inc.edge_weight)
           for n in (num_samples, neg_samples)]

    def chunk(seed, offset, stride):
      nq, gnq, eq, geq = (row_class_quota(x, offset, stride) for x in q)
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
    neg = int(wmax * 3 * neg_samples)
    return _bound(inc, int(wmax * 2 * num_samples) + 2, row_quota, 2) + neg

  emb = _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                 sampler_fn, _hgx.LOSS_KLD, _hgx.ACT_SIGMOID,
                                 batch_size, epochs, debug_summary_path,
                                 disable_pbar, chunk_sampler_fn=chunk_sampler_fn,
                                 bound_per_row=bound_per_row,
                                 records_budget=records_budget)
  emb.method_name = "HG2V_BOOLEAN"
  return emb


def _dist_backend_device(group):
  import torch.distributed as dist
  return "cpu" if dist.get_backend(group) == "gloo" else None


def _all_gather_rows(part, r0, r1, n_rows, group, device):
  """Every rank's row range [r0, r1) of an (n_rows x k) float32 table,
  assembled on every rank (one all-gather of padded row blocks)."""
  import torch
  import torch.distributed as dist
  world = dist.get_world_size(group)
  k = part.shape[1]
  dev = torch.device("cpu") if device == "cpu" else torch.device(
      "cuda", torch.cuda.current_device())
  lim = torch.tensor([r0, r1], dtype=torch.int64, device=dev)
  lims = [torch.zeros_like(lim) for _ in range(world)]
  dist.all_gather(lims, lim, group=group)
  lims = [tuple(int(v) for v in t.cpu()) for t in lims]
  m = max(b - a for a, b in lims)
  buf = torch.zeros((max(m, 1), k), dtype=torch.float32, device=dev)
  buf[:r1 - r0] = torch.from_numpy(np.ascontiguousarray(part, np.float32))
  outs = [torch.empty_like(buf) for _ in range(world)]
  dist.all_gather(outs, buf, group=group)
  full = np.zeros((n_rows, k), np.float32)
  for (a, b), t in zip(lims, outs):
    full[a:b] = t[:b - a].cpu().numpy()
  return full


def _broadcast_seeds(n, group, device):
  """n 62-bit seeds drawn from rank 0's numpy RandomState, on every rank."""
  import torch
  import torch.distributed as dist
  dev = torch.device("cpu") if device == "cpu" else torch.device(
      "cuda", torch.cuda.current_device())
  t = torch.tensor([numpy_seed() for _ in range(n)], dtype=torch.int64,
                   device=dev)
  dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None
                 else 0, group=group)
  return [int(v) for v in t.cpu()]


def hobe_sharded(inc, dimension, num_neighbors=5, num_samples=200,
                 batch_size=256, epochs=10, group=None, records_budget=None,
                 edge_ranges=1, alg_coords=None, ctx=None, stats=None):
  """The HOBE pipeline over the ranks of a torch.distributed group, one GPU
  per rank (EmbedHg2vAlgDist(..., group=) calls it):
    1. alg-dist node-row sharded (algebraic_distance.alg_dist_sharded: the
       edge-side partials all-reduced every iteration), from rank 0's
       np.random draws (algebraic_distance.py:140-141), then one all-gather
       of the node coordinates (N x 10 floats: 400 MB at C4) so every rank
       holds the HOBE weights' inputs;
    2. the stream in strided row chunks (_row_chunks), each sampled by the
       ranks on strided shares of its rows and all-gathered in row order
       (hg2v_sample.sharded_chunk_fn);
    3. training as replicas (batch-256 Adagrad does not
       partition): every rank trains the same model on the same chunks in
       the same order (seeds broadcast from rank 0), Hg2vModel.fit_streaming
       -- or, when the stream is one chunk, it is sampled once and fit() runs
       the epochs on it, as the single-process path does.
  `alg_coords` = (x, y) skips step 1 (tests: the sharded relaxation sums
  partials in another order than one GPU, within 1e-4; steps 2-3 are then
  bit-identical to the single-process call). Returns (node_tab, edge_tab)
  without the padding row, identical on every rank."""
  import torch.distributed as dist
  from .algebraic_distance import _init_coords, alg_dist_sharded
  from .hg2v_sample import sharded_chunk_fn
  ctx = ctx or get_context()
  dev = _dist_backend_device(group)
  world = dist.get_world_size(group)
  ctx.upload(inc)
  if alg_coords is None:
    x0 = y0 = None
    if dist.get_rank(group) == 0:
      x0, y0 = _init_coords(inc, 10)
    import torch
    tdev = torch.device("cpu") if dev == "cpu" else torch.device(
        "cuda", torch.cuda.current_device())
    bx = torch.from_numpy(np.ascontiguousarray(x0, np.float32)) \
        if x0 is not None else torch.empty((inc.N, 10), dtype=torch.float32)
    by = torch.from_numpy(np.ascontiguousarray(y0, np.float32)) \
        if y0 is not None else torch.empty((inc.E, 10), dtype=torch.float32)
    bx, by = bx.to(tdev), by.to(tdev)
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(bx, src=src, group=group)
    dist.broadcast(by, src=src, group=group)
    x0, y0 = bx.cpu().numpy(), by.cpu().numpy()
    (r0, r1, xo), y, ms = alg_dist_sharded(ctx, inc, x0, y0, 20, group=group,
                                           edge_ranges=edge_ranges,
                                           stats=stats)
    x = _all_gather_rows(xo, r0, r1, inc.N, group, dev)
    if stats is not None:
      stats["alg_ms"] = ms
  else:
    x, y = alg_coords
  ctx.alg_set(x, y)
  sample_seed, model_seed, fit_seed = _broadcast_seeds(3, group, dev)
  budget = (RECORDS_BUDGET // 2 if world > 1 else RECORDS_BUDGET) \
      if records_budget is None else records_budget
  chunks = _row_chunks(inc, 2 * num_samples, budget)
  fn = sharded_chunk_fn(inc, num_neighbors, num_samples, chunks, ctx=ctx,
                        seed=sample_seed, kind="hobe", group=group, device=dev)
  model = Hg2vModel(inc.N + 1, inc.E + 1, dimension, num_neighbors,
                    _hgx.LOSS_MSE, _hgx.ACT_RELU, ctx=ctx, seed=model_seed)
  if len(chunks) == 1:
    fn(0)
    model.fit(batch_size=batch_size, epochs=epochs, shuffle_seed=fit_seed)
  else:
    model.fit_streaming(fn, len(chunks), batch_size=batch_size, epochs=epochs,
                        seed=fit_seed % (2**32))
  node_w, edge_w = model.get_weights()
  return node_w[1:], edge_w[1:]


def EmbedHg2vAlgDist(hypergraph, dimension, alpha=0, num_neighbors=5,
                     num_samples=200, batch_size=256, epochs=10,
                     debug_summary_path=None, disable_pbar=False,
                     records_budget=None, group=None, edge_ranges=1,
                     row_quota=None):
  """HOBE: alg-dist (k=10, 20 iterations) + AlgebraicDistanceSamples +
  UnweightedFloatModel (embedding.py:389-416). `alpha` is accepted and, as
  in the reference, not used (_alpha_scale is called with alpha=0).
  A stream of more than `records_budget` records (RECORDS_BUDGET) is
  sampled and trained in strided row chunks (Hg2vModel.fit_streaming).
  `group` (a torch.distributed process group, e.g. group.WORLD under
  torch.distributed.run, one GPU per rank): the multi-GPU pipeline
  (hobe_sharded); every rank returns the same embedding. row_quota =
  (node quotas, edge quotas) (not in the reference) replaces S on every
  row: bounded runs (rows with quota 0 are not sampled)."""
  del alpha
  if group is not None:
    assert row_quota is None, "row_quota is a single-process option"
    inc = (hypergraph if isinstance(hypergraph, Incidence)
           else Incidence.from_hypergraph(hypergraph))
    nt, et = hobe_sharded(inc, dimension, num_neighbors, num_samples,
                          batch_size, epochs, group=group,
                          records_budget=records_budget,
                          edge_ranges=edge_ranges)
    emb = coords_to_embedding(inc, nt, et, dimension, "")
    emb.method_name = "HG2V_ALG_DIST"
    return emb

  def alg_dist(inc, ctx):
    x0 = np.random.random((inc.N, 10))  # algebraic_distance.py:140-141
    y0 = np.random.random((inc.E, 10))
    ctx.upload(inc)
    ctx.alg_set(x0, y0)
    ctx.alg_run(20)  # coords stay resident for the HOBE probabilities

  def sampler_fn(inc, ctx):
    alg_dist(inc, ctx)
    return sample_hobe(inc, num_neighbors, num_samples, ctx=ctx,
                       row_quota=row_quota)

  def chunk_sampler_fn(inc, ctx):
    alg_dist(inc, ctx)
    full = (row_quota if row_quota is not None else
            (np.full(inc.N, num_samples, np.int32),
             np.full(inc.E, num_samples, np.int32)))

    def chunk(seed, offset, stride):
      nq = row_class_quota(full[0], offset, stride)
      eq = row_class_quota(full[1], offset, stride)
      return ctx.sample_hobe(seed, num_neighbors, num_samples, node_q=nq,
                             edge_q=eq)
    return chunk

  # per row at most S nn (or ee) and S node-edge records (hg2v_sample.py:659-703)
  emb = _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                 sampler_fn, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                                 batch_size, epochs, debug_summary_path,
                                 disable_pbar, chunk_sampler_fn=chunk_sampler_fn,
                                 bound_per_row=lambda inc: _bound(
                                     inc, 2 * num_samples, row_quota, 2),
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
