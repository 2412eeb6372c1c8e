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
from .runtime import check_rng, get_context, numpy_seed, numpy_state_seed

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


# Records resident at once (68 B per record at K = 5: 2^30 records = 73
# GB of HBM). A stream whose record bound exceeds it is sampled once into
# the compact record store (12 B per record) in strided row chunks of at
# most this many records, and every epoch streams through the store in
# chunks of at most this many records (Hg2vModel.fit_store).
RECORDS_BUDGET = 1 << 30
# Records per sampled row class and per loaded chunk of a streamed epoch:
# C4 (5.9e9 records) then holds the 71 GB store, one 36.5 GB chunk of
# trainer records, 19 GB of load scratch and 31 GB of d = 256 tables and
# Adagrad state -- ~170 GB of the 288 GB HBM.
STORE_CHUNK = 1 << 29


def _row_chunks(bound_n, bound_e, budget):
  """Split the rows into n strided classes (offset c, stride n: node rows
  and edge rows r = c mod n) so that every class's record bound -- the sum
  of its rows' bounds bound_n[r] / bound_e[r] -- stays within `budget`
  (the sampler holds one class's records at a time). Strided, not
  contiguous: hub rows (low ids in the power-law generator; sorted or
  community ordered ids in real data) spread over all classes, so classes
  cost the same to sample."""
  bn = np.asarray(bound_n, np.int64)
  be = np.asarray(bound_e, np.int64)
  total = int(bn.sum() + be.sum())
  n = max(1, -(-total // budget))
  top = max(bn.size, be.size, 1)
  while n < top:
    cls = (np.bincount(np.arange(bn.size) % n, weights=bn, minlength=n) +
           np.bincount(np.arange(be.size) % n, weights=be, minlength=n))
    if cls.max() <= budget:
      break
    n = min(top, n + max(1, n // 8))
  return [(c, n) for c in range(n)]


def fill_store(ctx, inc, chunk_fn, bound_n, bound_e, budget):
  """Sample the stream once into ctx's record store: strided row classes
  (_row_chunks) sampled in turn by chunk_fn(offset, stride) (the records of
  that class now on ctx), each packed into the store (hgx_store_append).
  Returns the records stored."""
  bn = np.asarray(bound_n, np.int64)
  be = np.asarray(bound_e, np.int64)
  chunks = _row_chunks(bn, be, budget)
  ctx.store_reset(int(bn.sum() + be.sum()))
  for off, stride in chunks:
    m = chunk_fn(off, stride)
    check_class_bound(m, bn, be, off, stride)
    ctx.store_append()
  return ctx.store_info()[0]


def check_class_bound(m, bn, be, off, stride):
  """A row class must not sample more records than its rows' bounds (the
  store and the chunk plan are sized by them): a real exception, not an
  assert, so python -O keeps it."""
  cap = int(bn[off::stride].sum() + be[off::stride].sum())
  if m is not None and m > cap:
    raise RuntimeError("row class %d/%d sampled %d records, above its bound "
                       "%d" % (off, stride, m, cap))


def _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors, sampler_fn,
                             loss, act, fit_batch_size, fit_epochs,
                             debug_summary_path, disable_pbar, ctx=None,
                             chunk_sampler_fn=None, row_bounds=None,
                             records_budget=None, rng=None):
  """embedding.py:269-305, device-resident end to end. `hypergraph` is the
  reference's Hypergraph message or an already compressed Incidence (e.g.
  proto_native.read_incidence of a file too large for Python protobuf).
  A stream whose record bound (row_bounds(inc): per node row, per edge
  row) exceeds the budget is sampled once into the compact record store
  and trained from it with Keras' global shuffle (Hg2vModel.fit_store).
  rng="mt19937" (the stream stays resident): the sampler draws numpy's
  stream, the tables are initialised from a seed derived from numpy's
  state without drawing from it (Keras' init comes from TF), and every
  epoch's order is Keras' np.random.shuffle -- numpy's global stream
  advances exactly as the reference's does."""
  del disable_pbar
  ctx = ctx or get_context()
  if isinstance(hypergraph, Incidence):
    inc = hypergraph
  else:
    inc = Incidence.from_hypergraph(hypergraph)  # CompressRange + CSR
  budget = RECORDS_BUDGET if records_budget is None else records_budget
  if chunk_sampler_fn is not None and rng is None:
    bn, be = row_bounds(inc)
    if int(np.sum(bn, dtype=np.int64) + np.sum(be, dtype=np.int64)) > budget:
      seed = numpy_seed()
      sample = chunk_sampler_fn(inc, ctx)
      chunk = min(budget, STORE_CHUNK)
      try:
        fill_store(ctx, inc, lambda off, stride: sample(seed, off, stride),
                   bn, be, chunk)
        model = Hg2vModel(inc.N + 1, inc.E + 1, dimension, num_neighbors,
                          loss, act, ctx=ctx)
        model.fit_store(chunk, batch_size=fit_batch_size, epochs=fit_epochs)
        node_w, edge_w = model.get_weights()
      finally:
        # the store (~71 GB at C4), its load scratch and the last chunk's
        # records go back to the device, also when sampling or fit raises
        ctx.store_release()
      return coords_to_embedding(inc, node_w[1:], edge_w[1:], dimension, "")
  records = sampler_fn(inc, ctx)
  if debug_summary_path is not None:
    _plot_distributions(debug_summary_path, records)
  model = Hg2vModel(inc.N + 1, inc.E + 1, dimension, num_neighbors, loss, act,
                    ctx=ctx, seed=numpy_state_seed() if rng else None)
  # (rows = max compressed idx + 2)
  model.fit(batch_size=fit_batch_size, epochs=fit_epochs, rng=rng)
  node_w, edge_w = model.get_weights()
  return coords_to_embedding(inc, node_w[1:], edge_w[1:], dimension, "")


def EmbedHg2vBoolean(hypergraph, dimension, num_neighbors=5, num_samples=200,
                     batch_size=256, epochs=10, neg_samples=0,
                     debug_summary_path=None, disable_pbar=False,
                     records_budget=None, row_quota=None, rng=None):
  """FOBE: BooleanSamples + BooleanModel (embedding.py:308-329). A stream of
  more than `records_budget` records is sampled once into the compact
  record store and every epoch trains it in Keras' global shuffle order
  (Hg2vModel.fit_store). row_quota = (node quotas, edge quotas) (not in
  the reference) replaces int(weight * S) per row: bounded runs.
  rng="mt19937": after np.random.seed(s) the records and every epoch's
  order are the reference's bit for bit (_hypergraph2vec_skeleton)."""
  if check_rng(rng) and row_quota is not None:
    raise ValueError("row_quota is not a reference option: not with "
                     "rng='mt19937'")
  sampler_fn = lambda inc, ctx: sample_fobe(inc, num_neighbors, num_samples,
                                            neg_samples, ctx=ctx,
                                            row_quota=row_quota, rng=rng)

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

  # per node row at most q nn and q node-edge records, per edge row q ee and
  # q node-edge records, q = int(w * S) (hg2v_sample.py:138-194); negatives
  # (:198-240): g nn + g node-edge per node row, 2 g ee + g node-edge per
  # edge row, g = int(w * neg_samples)
  def row_bounds(inc):
    if row_quota is not None:
      qn, qe = (np.asarray(q, np.int64) for q in row_quota)
    else:
      qn = _quotas(inc.node_weight, num_samples).astype(np.int64)
      qe = _quotas(inc.edge_weight, num_samples).astype(np.int64)
    bn, be = 2 * qn, 2 * qe
    if neg_samples > 0:
      bn = bn + 2 * _quotas(inc.node_weight, neg_samples).astype(np.int64)
      be = be + 3 * _quotas(inc.edge_weight, neg_samples).astype(np.int64)
    return bn, be

  emb = _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                 sampler_fn, _hgx.LOSS_KLD, _hgx.ACT_SIGMOID,
                                 batch_size, epochs, debug_summary_path,
                                 disable_pbar, chunk_sampler_fn=chunk_sampler_fn,
                                 row_bounds=row_bounds,
                                 records_budget=records_budget, rng=rng)
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
    2. sampling row-sharded: a stream within the budget is sampled on the
       ranks' strided row shares and all-gathered in row order
       (hg2v_sample.sample_sharded); a larger one is sampled once into
       every rank's record store, strided row class by class, each class's
       12-byte entries all-gathered while the next class samples
       (hg2v_sample.sharded_store_fill);
    3. training as replicas (batch-256 Adagrad does not
       partition): every rank trains the same model on the same epochs
       (seeds broadcast from rank 0): fit() on the resident stream, or
       Hg2vModel.fit_store's global-shuffle epochs over the store.
  `alg_coords` = (x, y) skips step 1 (tests: the sharded relaxation sums
  partials in another order than one GPU, within 1e-4; steps 2-3 are then
  bit-identical to the single-process call). `stats` (a dict) receives the
  stage times. Returns (node_tab, edge_tab) without the padding row,
  identical on every rank."""
  import time
  import torch.distributed as dist
  from .algebraic_distance import _init_coords, alg_dist_sharded
  from .hg2v_sample import sample_sharded, sharded_store_fill
  ctx = ctx or get_context()
  dev = _dist_backend_device(group)
  world = dist.get_world_size(group)
  st = stats if stats is not None else {}
  ctx.upload(inc)
  t0 = time.perf_counter()
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
    st["alg_ms"] = ms
  else:
    x, y = alg_coords
  ctx.alg_set(x, y)
  st["alg_s"] = time.perf_counter() - t0
  sample_seed, model_seed, fit_seed = _broadcast_seeds(3, group, dev)
  # resident at world > 1 only up to half the single-GPU budget: the
  # row-sharded sampler holds its gather buffers, the gathered stream and
  # the context's copy at once (~2.5x the stream); larger streams take the
  # store path, whose per-rank peak is the single-GPU one
  if records_budget is not None:
    budget = records_budget
  else:
    budget = RECORDS_BUDGET if world == 1 else RECORDS_BUDGET // 2
  bn = np.full(inc.N, 2 * num_samples, np.int64)
  be = np.full(inc.E, 2 * num_samples, np.int64)
  model = Hg2vModel(inc.N + 1, inc.E + 1, dimension, num_neighbors,
                    _hgx.LOSS_MSE, _hgx.ACT_RELU, ctx=ctx, seed=model_seed)
  t0 = time.perf_counter()
  if int(bn.sum() + be.sum()) <= budget:
    n, _ = sample_sharded(inc, num_neighbors, num_samples, ctx=ctx,
                          seed=sample_seed, kind="hobe", group=group,
                          device=dev)
    st["sampling_s"] = time.perf_counter() - t0
    st["records"] = n
    t0 = time.perf_counter()
    model.fit(batch_size=batch_size, epochs=epochs, shuffle_seed=fit_seed)
  else:
    chunk = min(budget, STORE_CHUNK)
    chunks = _row_chunks(bn, be, chunk)
    try:
      n = sharded_store_fill(inc, num_neighbors, num_samples, chunks, ctx=ctx,
                             seed=sample_seed, kind="hobe", group=group,
                             device=dev, capacity=int(bn.sum() + be.sum()),
                             row_bounds=(bn, be))
      st["sampling_s"] = time.perf_counter() - t0
      st["records"] = n
      st["sampling_chunks"] = len(chunks)
      t0 = time.perf_counter()
      model.fit_store(chunk, batch_size=batch_size, epochs=epochs,
                      seed=fit_seed % (2**32))
    finally:
      ctx.store_release()
  st["train_s"] = time.perf_counter() - t0
  node_w, edge_w = model.get_weights()
  return node_w[1:], edge_w[1:]


def EmbedHg2vAlgDist(hypergraph, dimension, alpha=0, num_neighbors=5,
                     num_samples=200, batch_size=256, epochs=10,
                     debug_summary_path=None, disable_pbar=False,
                     records_budget=None, group=None, edge_ranges=1,
                     row_quota=None, rng=None):
  """HOBE: alg-dist (k=10, 20 iterations) + AlgebraicDistanceSamples +
  UnweightedFloatModel (embedding.py:389-416). `alpha` is accepted and, as
  in the reference, not used (_alpha_scale is called with alpha=0).
  A stream of more than `records_budget` records (RECORDS_BUDGET) is
  sampled once into the compact record store and every epoch trains it in
  Keras' global shuffle order (Hg2vModel.fit_store).
  `group` (a torch.distributed process group, e.g. group.WORLD under
  torch.distributed.run, one GPU per rank): the multi-GPU pipeline
  (hobe_sharded); every rank returns the same embedding. row_quota =
  (node quotas, edge quotas) (not in the reference) replaces S on every
  row: bounded runs (rows with quota 0 are not sampled). rng="mt19937":
  after np.random.seed(s) the alg-dist init, the HOBE pairs and
  (run_in_parallel=False) neighbours and every epoch's order come from
  numpy's stream as in the reference (the probabilities from this
  device's alg-dist coordinates, within 1e-4 of the reference's)."""
  del alpha
  if check_rng(rng) and (group is not None or row_quota is not None):
    raise ValueError("rng='mt19937' is the single-process reference "
                     "stream: no group, no row_quota")
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
                       row_quota=row_quota, rng=rng)

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

  # per row at most q nn (or ee) and q node-edge records, q = S or the row's
  # quota (hg2v_sample.py:659-703)
  def row_bounds(inc):
    if row_quota is not None:
      return (2 * np.asarray(row_quota[0], np.int64),
              2 * np.asarray(row_quota[1], np.int64))
    return (np.full(inc.N, 2 * num_samples, np.int64),
            np.full(inc.E, 2 * num_samples, np.int64))

  emb = _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                 sampler_fn, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                                 batch_size, epochs, debug_summary_path,
                                 disable_pbar, chunk_sampler_fn=chunk_sampler_fn,
                                 row_bounds=row_bounds,
                                 records_budget=records_budget, rng=rng)
  emb.method_name = "HG2V_ALG_DIST"
  return emb


def _jaccard_embed(hypergraph, dimension, which, alpha, num_neighbors,
                   num_samples, batch_size, epochs, debug_summary_path,
                   disable_pbar, rng=None):
  """embedding.py:330-386: WeightedJaccardSamples over UniformWeight or
  WeightByNeighborhood features, UnweightedFloatModel (relu, MSE).
  rng="mt19937": numpy's stream for the samples and the epoch orders."""
  check_rng(rng)

  def sampler_fn(inc, ctx):
    ctx.upload(inc)
    fn, fe = ctx.incidence_weights(which, float(alpha))
    return sample_jaccard(inc, fn, fe, num_neighbors, num_samples, ctx=ctx,
                          rng=rng)

  return _hypergraph2vec_skeleton(hypergraph, dimension, num_neighbors,
                                  sampler_fn, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                                  batch_size, epochs, debug_summary_path,
                                  disable_pbar, rng=rng)


def EmbedHg2vAdjJaccard(hypergraph, dimension, num_neighbors=5,
                        num_samples=200, batch_size=256, epochs=10,
                        debug_summary_path=None, disable_pbar=False, rng=None):
  """embedding.py:330-355 (UniformWeight features)."""
  emb = _jaccard_embed(hypergraph, dimension, _hgx.WEIGHT_UNIFORM, 0.0,
                       num_neighbors, num_samples, batch_size, epochs,
                       debug_summary_path, disable_pbar, rng=rng)
  emb.method_name = "HG2V_ADJ_JAC"
  return emb


def EmbedHg2vNeighborhoodWeightedJaccard(hypergraph, dimension, alpha=0,
                                         num_neighbors=5, num_samples=200,
                                         batch_size=256, epochs=10,
                                         debug_summary_path=None,
                                         disable_pbar=False, rng=None):
  """embedding.py:358-386 (WeightByNeighborhood(alpha) features)."""
  assert 0 <= alpha <= 1
  emb = _jaccard_embed(hypergraph, dimension, _hgx.WEIGHT_NEIGHBORHOOD, alpha,
                       num_neighbors, num_samples, batch_size, epochs,
                       debug_summary_path, disable_pbar, rng=rng)
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
