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
  in Python (same message; map entries in ascending id order)."""
  from . import _hgx
  x = np.ascontiguousarray(x, np.float32).reshape(inc.N, dimension)
  y = np.ascontiguousarray(y, np.float32).reshape(inc.E, dimension)
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


def alg_dist_sharded(ctx, inc, x0, y0, iterations, group=None, device=None):
  """Node-row-sharded relaxation; the caller's process group does the
  exchange. Every rank must call it with the same inputs. Returns the node
  rows this rank owns (row0, row1, x_own) and all edge coords, already
  rescaled, plus the time in ms of the iteration loop.

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
  ks = ((k + 1) + 3) // 4 * 4
  M = 2 * ks * 64  # HGX_MM_REPLICAS
  part = torch.zeros(inc.E * ks, dtype=torch.float32, device=dev)
  mm = torch.zeros(iterations * M, dtype=torch.int32, device=dev)
  stream = None
  if on_gpu:
    # kernels and collectives share one (non-default) torch stream: stream
    # order is the only synchronisation needed between the phases
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    ctx.set_stream(stream.cuda_stream)
  try:
    ks_lib = ctx.alg_shard_begin(r0, r1, part.data_ptr(), mm.data_ptr(),
                                 iterations)
    assert ks_lib == ks
    if on_gpu:
      start = torch.cuda.Event(enable_timing=True)
      end = torch.cuda.Event(enable_timing=True)
      start.record(stream)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream) if on_gpu else contextlib.nullcontext():
      for it in range(iterations):
        ctx.alg_shard_node(it)
        ctx.alg_shard_edge_partial(it)
        dist.all_reduce(part, op=dist.ReduceOp.SUM, group=group)
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
  return (r0, r1, x[r0:r1].copy()), y, ms


__all__ = ["EmbedAlgebraicDistance", "AlgebraicDistance", "alg_dist_sharded",
           "coords_to_embedding", "shard_rows"]
