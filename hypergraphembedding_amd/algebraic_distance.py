"""Algebraic distance (reference: hypergraph_embedding/algebraic_distance.py).

``EmbedAlgebraicDistance`` keeps the reference signature and result
(algebraic_distance.py:126-175): CompressRange, uniform [0,1) init from
numpy's global RNG (nodes then edges, :140-141), ``iterations`` rounds of
node half / edge half / joint min-max rescale on the GPU (libhgx
``hgx_alg_*``), a ``HypergraphEmbedding`` keyed by the original ids with
method_name "AlgebraicDistance" (:166-174).

``alg_dist_sharded`` is the multi-GPU form: node rows split
across ranks by incidence count, edge coords replicated, per iteration one
SUM all-reduce of the E x KS edge partials and one MAX all-reduce of the
min/max words, both through torch.distributed (RCCL on GPUs, gloo in tests).
"""

import numpy as np

from . import _hgx
from .hypergraph_util import Incidence
from .proto import HypergraphEmbedding
from .runtime import get_context


def _init_coords(inc, dimension):
  # same draw order as algebraic_distance.py:140-141
  x = np.random.random((inc.N, dimension))
  y = np.random.random((inc.E, dimension))
  return x, y


def AlgebraicDistance(inc, dimension, iterations=20, init=None, ctx=None):
  """Relax on the device; returns (node_coords, edge_coords) float32 and the
  context, whose device copy stays resident for HOBE sampling."""
  ctx = ctx or get_context()
  x0, y0 = init if init is not None else _init_coords(inc, dimension)
  ctx.upload(inc)
  x, y = ctx.alg_dist(x0, y0, iterations)
  return x, y, ctx


def EmbedAlgebraicDistance(hypergraph, dimension, iterations=20,
                           run_in_parallel=True, disable_pbar=False):
  """Drop-in for algebraic_distance.py:126-175 (run_in_parallel and
  disable_pbar are accepted for signature compatibility)."""
  del run_in_parallel, disable_pbar
  inc = Incidence.from_hypergraph(hypergraph)
  x, y, _ = AlgebraicDistance(inc, dimension, iterations)
  return coords_to_embedding(inc, x, y, dimension, "AlgebraicDistance")


def coords_to_embedding(inc, x, y, dimension, method_name):
  """HypergraphEmbedding keyed by the original ids (KerasModelToEmbedding,
  hg2v_model.py:31-48 / algebraic_distance.py:166-174): serialized by the
  native writer and parsed once, instead of filling the maps field by field
  in Python (same message; map entries in ascending id order). A message
  beyond protobuf's 2 GiB limit (C4 at d=256: ~10 GB) cannot exist as one
  HypergraphEmbedding: a proto_native.ShardedEmbedding (the same message
  surface, written as shards of complete messages) is returned instead."""
  from . import _hgx
  from .proto_native import PROTO_LIMIT, ShardedEmbedding, message_bytes
  x = np.ascontiguousarray(x, np.float32).reshape(inc.N, dimension)
  y = np.ascontiguousarray(y, np.float32).reshape(inc.E, dimension)
  if message_bytes(inc.node_ids, inc.edge_ids, dimension,
                   method_name) > PROTO_LIMIT:
    return ShardedEmbedding(inc.node_ids, x, inc.edge_ids, y, dimension,
                            method_name)
  emb = HypergraphEmbedding()
  emb.ParseFromString(_hgx.write_embedding_bytes(inc.node_ids, x, inc.edge_ids,
                                                 y, method_name).tobytes())
  emb.dim = dimension
  emb.method_name = method_name
  return emb


def shard_rows(rp, world, rank):
  """Contiguous node-row range of `rank`, balanced by incidence count."""
  nnz = int(rp[-1])
  lo = int(np.searchsorted(rp, nnz * rank / world, side="left"))
  hi = int(np.searchsorted(rp, nnz * (rank + 1) / world, side="left"))
  if rank == world - 1:
    hi = len(rp) - 1
  return min(lo, len(rp) - 1), min(hi, len(rp) - 1)


def alg_dist_sharded(ctx, inc, x0, y0, iterations, group=None, device=None,
                     compact=True, stats=None, edge_ranges=1):
  """Node-row-sharded relaxation; the caller's process group does the
  exchange. Every rank must call it with the same inputs. Returns the node
  rows this rank owns (row0, row1, x_own) and all edge coords, already
  rescaled, plus the time in ms of the iteration loop.

  Per iteration (algebraic_distance.py:54-123 split by node rows): the node
  half of the own rows, the edge partial sums [sum w, sum w x] over the own
  rows, a SUM all-reduce of those partials, the edge finish, a MAX
  all-reduce of the min/max words. With `compact` only the edges whose
  incidences sit on two or more ranks are exchanged, as k + 1 floats
  (hgx_alg_shard_wire); an edge private to one rank is finished there and
  gathered once after the last iteration. With `edge_ranges` > 1 the edge
  partials are computed range by range (hgx_alg_shard_ranges: the same split
  on every rank) and each range's exchange is issued asynchronously as soon
  as its partials are queued, so the all-reduce of range r overlaps the
  partials of range r + 1; edge_final waits for all of them. `stats` (a
  dict) receives the exchanged bytes per iteration.

  `ctx` is a libhgx Context (exchange buffers on its GPU, RCCL) or any
  object with the same alg_shard_* protocol; with device=cpu the exchange
  buffers are host tensors and the collectives run over gloo (the CPU tests
  drive this function with a numpy restatement of the shard kernels).
  """
  import time
  import contextlib
  import torch
  import torch.distributed as dist
  world = dist.get_world_size(group)
  rank = dist.get_rank(group)
  r0, r1 = shard_rows(inc.rp_n, world, rank)
  dev = torch.device("cuda", ctx.device) if device is None else device
  on_gpu = dev.type == "cuda"
  ctx.upload(inc)
  ctx.alg_set(x0, y0)
  k = x0.shape[1]
  # the library picks the row width KS (round_up(k + 1, 4), widened to 16
  # floats on large graphs, or the alg_ks tuning, at most 20 on the narrow
  # path): size the exchange buffers for the widest, trim after begin
  ks_max = ((k + 1) + 3) // 4 * 4
  ks_max = max(ks_max, 20) if ks_max <= 20 else ks_max
  part = torch.zeros(inc.E * ks_max, dtype=torch.float32, device=dev)
  mm = torch.zeros(iterations * 2 * ks_max * 64, dtype=torch.int32, device=dev)
  slot = None
  if compact:
    # ranks holding incidences of each edge (one int32 all-reduce, once)
    touched = np.zeros(inc.E, np.int32)
    touched[inc.col_n[inc.rp_n[r0]:inc.rp_n[r1]]] = 1
    cnt = torch.from_numpy(touched.copy()).to(dev)  # never alias `touched`
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
    cnt = cnt.cpu().numpy()
    shared = cnt >= 2
    n_shared = int(shared.sum())
    slot = np.where(shared, np.cumsum(shared) - 1,
                    np.where(touched == 1, -1, -2)).astype(np.int32)
    wire = torch.zeros(max(n_shared, 1) * (k + 1), dtype=torch.float32,
                       device=dev)[:n_shared * (k + 1)]
    exch = wire
  stream = None
  if on_gpu:
    # kernels and collectives share one (non-default) torch stream: stream
    # order is the only synchronisation needed between the phases
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    ctx.set_stream(stream.cuda_stream)
  try:
    ks = ctx.alg_shard_begin(r0, r1, part.data_ptr(), mm.data_ptr(),
                             iterations)
    assert ks <= ks_max
    M = 2 * ks * 64  # HGX_MM_REPLICAS
    part, mm = part[:inc.E * ks], mm[:iterations * M]
    if not compact:
      exch = part
    if compact:
      ctx.alg_shard_wire(wire.data_ptr() if n_shared else None, n_shared, slot)
    segs = [exch]
    if edge_ranges > 1:
      b = ctx.alg_shard_ranges(edge_ranges).astype(np.int64)
      if compact:
        # wire rows are the shared edges in id order
        first = np.concatenate([[0], np.cumsum(slot >= 0)])[b] * (k + 1)
      else:
        first = b * ks
      segs = [exch[int(first[r]):int(first[r + 1])] for r in range(edge_ranges)]
    if on_gpu:
      start = torch.cuda.Event(enable_timing=True)
      end = torch.cuda.Event(enable_timing=True)
      start.record(stream)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream) if on_gpu else contextlib.nullcontext():
      for it in range(iterations):
        ctx.alg_shard_node(it)
        if edge_ranges > 1:
          works = []
          for r, seg in enumerate(segs):
            ctx.alg_shard_edge_partial_range(it, r)
            if seg.numel():
              works.append(dist.all_reduce(seg, op=dist.ReduceOp.SUM,
                                           group=group, async_op=True))
          for w in works:
            w.wait()
        else:
          ctx.alg_shard_edge_partial(it)
          if exch.numel():
            dist.all_reduce(exch, op=dist.ReduceOp.SUM, group=group)
        ctx.alg_shard_edge_final(it)
        dist.all_reduce(mm[it * M:(it + 1) * M], op=dist.ReduceOp.MAX,
                        group=group)
      if on_gpu:
        end.record(stream)
    ctx.alg_shard_end()
    if on_gpu:
      torch.cuda.synchronize(dev)
  finally:
    if on_gpu:
      ctx.set_stream(None)
  ms = start.elapsed_time(end) if on_gpu else (time.perf_counter() - t0) * 1e3
  x, y = ctx.alg_get()
  if compact and (slot == -2).any():
    # other ranks' private edges: each has exactly one owner
    priv = torch.from_numpy(np.where((slot == -1)[:, None], y, 0).astype(np.float32))
    priv = priv.to(dev)
    dist.all_reduce(priv, op=dist.ReduceOp.SUM, group=group)
    y = np.where((slot == -2)[:, None], priv.cpu().numpy(), y).astype(np.float32)
  if stats is not None:
    mm_bytes = M * 4
    stats.update(
        exchange="compact" if compact else "dense",
        edge_ranges=int(edge_ranges),
        shared_edges=int(n_shared) if compact else inc.E,
        partial_bytes_per_iter=int(exch.numel()) * 4,
        dense_partial_bytes_per_iter=inc.E * ks * 4,
        minmax_bytes_per_iter=mm_bytes,
        # ring all-reduce: each rank sends and receives 2 (G-1)/G of a buffer
        ring_bytes_per_rank_per_iter=int(2 * (world - 1) / world *
                                         (int(exch.numel()) * 4 + mm_bytes)))
  return (r0, r1, x[r0:r1].copy()), y, ms


__all__ = ["EmbedAlgebraicDistance", "AlgebraicDistance", "alg_dist_sharded",
           "coords_to_embedding", "shard_rows"]
