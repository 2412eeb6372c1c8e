"""FOBE / HOBE samplers (reference: hypergraph_embedding/hg2v_sample.py).

Same names and record semantics as the reference; the sampling runs on the
GPU (libhgx ``hgx_sample_fobe`` / ``hgx_sample_hobe``), records stay in HBM
in SamplesToModelInput layout for the trainer. The list-returning functions
(``BooleanSamples``, ``AlgebraicDistanceSamples``) materialise
``SimilarityRecord`` tuples only for API compatibility; the embedding
pipeline (embedding.py) never leaves the device.

Distribution parity: per row the reference draws min(q, |row|) distinct
columns uniformly (np.random.choice(replace=False), :77-85) and K
neighbours with replacement (:49-51). The device draws the same
distribution from a counter-based generator keyed by a seed taken from
numpy's global RNG, so np.random.seed(s) still makes runs reproducible.

rng="mt19937": the samplers draw from numpy's global RandomState itself
(hgx_sample_fobe_mt / hgx_sample_hobe_mt): after np.random.seed(s) the
records are the reference's bit for bit and numpy's state is left where the
reference leaves it (HOBE: run_in_parallel=False semantics).
"""

from collections import namedtuple

import numpy as np
import scipy.sparse as sp

from . import _hgx
from .hypergraph_util import Incidence
from .runtime import check_rng, get_context, numpy_seed

SimilarityRecord = namedtuple(
    "SimilarityRecord",
    ("left_node_idx", "left_edge_idx", "right_node_idx", "right_edge_idx",
     "left_weight", "right_weight", "neighbor_node_indices",
     "neighbor_node_weights", "neighbor_edge_indices", "neighbor_edge_weights",
     "node_node_prob", "edge_edge_prob", "node_edge_prob"))
SimilarityRecord.__new__.__defaults__ = (None,) * len(SimilarityRecord._fields)


def _quotas(weights, num_samples):
  # int(weight * num_samples) with the float32 proto weight (:138-146)
  return np.array([int(float(w) * num_samples) for w in weights], np.int32)


class DeviceRecords:
  """Handle to the record stream resident on a context (n x (4+2K) int32
  ids, +1 shifted, and n x 3 float32 targets)."""

  def __init__(self, ctx, inc, n, K):
    self.ctx, self.inc, self.n, self.K = ctx, inc, n, K

  def arrays(self):
    return self.ctx.records_get()

  def to_similarity_records(self):
    idx, tgt = self.arrays()
    return records_from_arrays(idx, tgt, self.K)


def records_from_arrays(idx, tgt, K):
  """Inverse of SamplesToModelInput(weighted=False) for our own streams."""
  out = []
  for r, t in zip(idx.tolist(), tgt.tolist()):
    ln, le, rn, re = (x - 1 if x > 0 else None for x in r[:4])
    nn = [x - 1 for x in r[4:4 + K]] if ln is not None and re is not None and rn is None else None
    ne = [x - 1 for x in r[4 + K:]] if nn is not None else None
    out.append(SimilarityRecord(
        left_node_idx=ln, left_edge_idx=le, right_node_idx=rn,
        right_edge_idx=re, neighbor_node_indices=nn, neighbor_edge_indices=ne,
        node_node_prob=t[0] if ln is not None and rn is not None else None,
        edge_edge_prob=t[1] if le is not None and re is not None else None,
        node_edge_prob=t[2] if nn is not None else None))
  return out


def sample_fobe(inc, num_neighbors, num_samples, neg_samples=0, ctx=None,
                seed=None, row_quota=None, rng=None):
  """BooleanSamples on the device; returns DeviceRecords. row_quota =
  (node quotas, edge quotas) replaces int(weight * S) per row (bounded
  runs; rows with quota 0 are not sampled). rng="mt19937": numpy's global
  stream, the reference's records bit for bit (seed unused)."""
  assert num_neighbors >= 1
  check_rng(rng)
  ctx = ctx or get_context()
  ctx.upload(inc)
  if row_quota is not None:
    nq, eq = (np.asarray(q, np.int32) for q in row_quota)
  else:
    nq = _quotas(inc.node_weight, num_samples)
    eq = _quotas(inc.edge_weight, num_samples)
  nnq = neq = None
  if neg_samples > 0:
    nnq = _quotas(inc.node_weight, neg_samples)
    neq = _quotas(inc.edge_weight, neg_samples)
  if rng == "mt19937":
    n = ctx.sample_fobe_mt(num_neighbors, nq, eq, nnq, neq)
  else:
    n = ctx.sample_fobe(numpy_seed() if seed is None else seed,
                        num_neighbors, nq, eq, nnq, neq)
  return DeviceRecords(ctx, inc, n, num_neighbors)


def sample_hobe(inc, num_neighbors, num_samples, ctx=None, seed=None,
                alg_coords=None, row_quota=None, rng=None):
  """AlgebraicDistanceSamples on the device (alg coords must be resident on
  ctx, e.g. from algebraic_distance.AlgebraicDistance, or given). row_quota
  = (node quotas, edge quotas) instead of S on every row (bounded runs).
  rng="mt19937": numpy's global stream, the reference's pairs and
  (run_in_parallel=False) neighbours bit for bit."""
  assert num_neighbors >= 0
  assert num_samples >= 0
  check_rng(rng)
  ctx = ctx or get_context()
  if alg_coords is not None:
    ctx.upload(inc)
    ctx.alg_set(*alg_coords)
  if rng == "mt19937":
    if row_quota is not None:
      raise ValueError("row_quota is not a reference option: not with "
                       "rng='mt19937'")
    n = ctx.sample_hobe_mt(num_neighbors, num_samples)
    return DeviceRecords(ctx, inc, n, num_neighbors)
  seed = numpy_seed() if seed is None else seed
  if row_quota is not None:
    n = ctx.sample_hobe(seed, num_neighbors, num_samples,
                        node_q=row_quota[0], edge_q=row_quota[1])
  else:
    n = ctx.sample_hobe(seed, num_neighbors, num_samples)
  return DeviceRecords(ctx, inc, n, num_neighbors)


def shard_range(n, world, rank):
  """Contiguous rows [lo, hi) of `rank` out of n rows split over `world`."""
  return n * rank // world, n * (rank + 1) // world


def row_class_quota(quota, offset, stride):
  """`quota` on the rows r = offset (mod stride), 0 elsewhere: one row class
  of a strided split (record-store fill chunks, sample_sharded ranks). A class
  is a uniform slice of the id space, so hub rows (the power-law generator
  numbers edges by popularity; real ids are often sorted or community
  ordered) spread over every chunk and rank instead of filling the first."""
  quota = np.asarray(quota, np.int32)
  out = np.zeros_like(quota)
  out[offset::stride] = quota[offset::stride]
  return out


# record column holding the row a record was sampled from, per kind block:
# nn (ln), ee (le), ne of node rows (ln), ne of edge rows (re, swapped);
# FOBE's negatives nn, ee, ee (the reference's repeated block), ne, ne
_ROW_COL = {"hobe": (0, 1, 0, 3), "fobe": (0, 1, 0, 3, 0, 1, 1, 0, 3)}


def sample_sharded(inc, num_neighbors, num_samples, ctx=None, seed=0,
                   kind="hobe", node_quota=None, edge_quota=None, group=None,
                   gather=True, device=None, rows=None):
  """Row-sharded sampling over the ranks of a torch.distributed group
  (sampling shards by row with no data-path collective).

  `rows` = (offset, stride) restricts the call to one row class of a
  strided split (store-fill chunk `offset` of `stride`; default: every
  row): node rows and edge rows r = offset (mod stride). Rank g samples the
  rows r = offset + g * stride (mod stride * world) of that class -- a
  strided share, so the hub rows spread over the ranks -- (kind "hobe":
  AlgebraicDistanceSamples, quota S per row unless quotas are given; kind
  "fobe": BooleanSamples with the given per-row quotas); the other rows'
  quotas are 0. Every draw, including the K neighbour draws of node-edge
  records, is keyed by (seed, pattern or block, row, rank in the row), so
  with the same seed on every rank the ranks' rows are exactly the rows a
  single process would draw. A count all-gather gives every rank the
  kind-block sizes of every rank. With `gather`, the per-rank streams are
  then all-gathered and, kind block by kind block, merged back into row
  order (a stable sort by each record's source row: within a row the
  owning rank's order stays): the reference's record order (nn, ee, ne node
  rows, ne edge rows, ...) of the class, the stream every training replica
  needs, identical to a single-process call on the same rows.

  Collectives: RCCL on device buffers for a GPU device (the records never
  leave HBM), gloo through host arrays otherwise. Returns
  (records now on ctx, sizes[world][blocks]).
  """
  import torch
  import torch.distributed as dist
  ctx = ctx or get_context()
  world, rank = dist.get_world_size(group), dist.get_rank(group)
  K = num_neighbors
  offset, stride = rows if rows is not None else (0, 1)
  assert 0 <= offset < stride
  if node_quota is None:  # HOBE: S per row (hg2v_sample.py:659-703)
    assert kind == "hobe"
    node_quota = np.full(inc.N, num_samples, np.int32)
    edge_quota = np.full(inc.E, num_samples, np.int32)
  mine = (offset + rank * stride, stride * world)
  nq = row_class_quota(node_quota, *mine)
  eq = row_class_quota(edge_quota, *mine)
  if kind == "hobe":
    ctx.sample_hobe(seed, K, num_samples, node_q=nq, edge_q=eq)
  else:
    ctx.sample_fobe(seed, K, nq, eq)
  bounds = ctx.records_blocks()
  sizes = np.diff(bounds)
  gpu = device is None or torch.device(device).type == "cuda"
  dev = torch.device("cuda", ctx.device) if device is None else torch.device(device)
  t = torch.tensor(sizes, dtype=torch.int64, device=dev)
  got = [torch.zeros_like(t) for _ in range(world)]
  dist.all_gather(got, t, group=group)
  allsz = np.stack([g.cpu().numpy() for g in got])  # [world][blocks]
  if not gather:
    return int(sizes.sum()), allsz
  R = 4 + 2 * K
  n_loc = allsz.sum(1)
  maxn = int(n_loc.max())
  total = int(allsz.sum())
  blk_tot = allsz.sum(0)
  gbounds = np.concatenate([[0], np.cumsum(blk_tot)]).astype(np.int64)
  # destination of (rank r, block j): block start + ranks before r
  dst = gbounds[:-1][None, :] + np.concatenate(
      [np.zeros((1, allsz.shape[1]), np.int64), np.cumsum(allsz, 0)[:-1]], 0)
  src = np.concatenate([np.zeros((world, 1), np.int64),
                        np.cumsum(allsz, 1)[:, :-1]], 1)
  # rows past a rank's count are never read: no fill is needed
  li = torch.empty((max(maxn, 1), R), dtype=torch.int32, device=dev)
  lt = torch.empty((max(maxn, 1), 3), dtype=torch.float32, device=dev)
  nl_ = int(n_loc[rank])
  if gpu:
    if nl_:
      # the export runs on the context's stream: torch's stream (which owns
      # li / lt and may still be using their memory) must be done first;
      # records_export returns after its copies completed
      torch.cuda.current_stream(dev).synchronize()
      ctx.records_export(li.data_ptr(), lt.data_ptr())
  else:
    hi, ht = ctx.records_get()
    li[:nl_] = torch.from_numpy(hi)
    lt[:nl_] = torch.from_numpy(ht)
  gi = [torch.empty_like(li) for _ in range(world)]
  gt = [torch.empty_like(lt) for _ in range(world)]
  dist.all_gather(gi, li, group=group)
  dist.all_gather(gt, lt, group=group)
  fi = torch.empty((max(total, 1), R), dtype=torch.int32, device=dev)
  ft = torch.empty((max(total, 1), 3), dtype=torch.float32, device=dev)
  for r in range(world):
    for j in range(allsz.shape[1]):
      c = int(allsz[r, j])
      if c:
        d, s0 = int(dst[r, j]), int(src[r, j])
        fi[d:d + c] = gi[r][s0:s0 + c]
        ft[d:d + c] = gt[r][s0:s0 + c]
  del gi, gt, li, lt
  if world > 1:
    # the ranks' rows interleave: restore row order inside every block
    # (FOBE: 4 blocks, or 9 with negatives)
    cols = _ROW_COL[kind][:allsz.shape[1]]
    assert len(cols) == allsz.shape[1], (kind, allsz.shape)
    for j, col in enumerate(cols):
      b0, b1 = int(gbounds[j]), int(gbounds[j + 1])
      if b1 - b0 > 1:
        perm = torch.sort(fi[b0:b1, col], stable=True).indices
        fi[b0:b1] = fi[b0:b1][perm]
        ft[b0:b1] = ft[b0:b1][perm]
        del perm
  if gpu:
    torch.cuda.synchronize(dev)
    # the gather buffers go back to the device before the context grows its
    # record buffer (hipMalloc) for the chunk: per rank the peak is the
    # import copy plus fi (SURVEY §8e budget)
    torch.cuda.empty_cache()
    ctx.records_import(total, K, fi.data_ptr(), ft.data_ptr(), gbounds)
    del fi, ft
    torch.cuda.empty_cache()
  else:
    ctx.records_set(fi[:total].numpy(), ft[:total].numpy())
  return total, allsz


def sharded_store_fill(inc, num_neighbors, num_samples, chunks, ctx=None,
                       seed=0, kind="hobe", node_quota=None, edge_quota=None,
                       group=None, device=None, capacity=0,
                       neg_node_quota=None, neg_edge_quota=None,
                       row_bounds=None):
  """Sample a record stream too large for HBM once into every rank's record
  store (hgx_store_*), the sampling row-sharded over the ranks of a
  torch.distributed group. For each strided row class
  chunks[c] = (offset, stride) (embedding._row_chunks) rank g samples the
  rows r = offset + g * stride (mod stride * world) of the class and packs
  them into its store; the class's new entries (12 B per record) are then
  all-gathered asynchronously -- RCCL on device buffers for a GPU device,
  gloo through host arrays otherwise -- while the next class is sampled,
  and every rank appends the other ranks' entries. Every draw is keyed by
  (seed, block, row, column or rank in row), so every rank ends with
  exactly the records a single process samples, in another order -- which
  the store's epoch order does not see (it is keyed by record identity):
  Hg2vModel.fit_store then trains the same epochs on every rank. Returns
  the records in the store. FOBE takes its negative quotas
  (neg_node_quota / neg_edge_quota, both or neither), sharded like the
  positive ones. row_bounds = (per node row, per edge row) record bounds:
  each rank's share of a class is checked against them (RuntimeError)."""
  import torch
  import torch.distributed as dist
  K = num_neighbors
  if (neg_node_quota is None) != (neg_edge_quota is None):
    raise ValueError("give both negative quotas or neither")
  if neg_node_quota is not None and kind != "fobe":
    raise ValueError("negative quotas are a FOBE (BooleanSamples) option")
  if node_quota is None:  # HOBE: S per row (hg2v_sample.py:659-703)
    if kind != "hobe":
      raise ValueError("FOBE sharded sampling needs its row quotas")
    node_quota = np.full(inc.N, num_samples, np.int32)
    edge_quota = np.full(inc.E, num_samples, np.int32)
  ctx = ctx or get_context()
  world, rank = dist.get_world_size(group), dist.get_rank(group)
  gpu = device is None or torch.device(device).type == "cuda"
  dev = torch.device("cuda", ctx.device) if device is None else torch.device(device)
  ctx.store_reset(capacity)
  pending = None  # (handle, recv buffers, per-rank counts) of the last class

  def finish(p):
    work, recv, cnt, _send = p
    work.wait()
    if gpu:
      torch.cuda.current_stream(dev).synchronize()
    for r in range(world):
      if r == rank or cnt[r] == 0:
        continue
      if gpu:
        ctx.store_write(None, fam, K, seed, n=int(cnt[r]),
                        src_ptr=recv[r].data_ptr())
      else:
        ctx.store_write(recv[r][:int(cnt[r])].numpy().view(np.uint32), fam, K,
                        seed)

  fam = _hgx.STORE_HOBE if kind == "hobe" else _hgx.STORE_FOBE
  for off, stride in chunks:
    mine = (off + rank * stride, stride * world)
    nq = row_class_quota(node_quota, *mine)
    eq = row_class_quota(edge_quota, *mine)
    before = ctx.store_info()[0]
    if kind == "hobe":
      got_n = ctx.sample_hobe(seed, K, num_samples, node_q=nq, edge_q=eq)
    elif neg_node_quota is not None:
      got_n = ctx.sample_fobe(seed, K, nq, eq,
                              row_class_quota(neg_node_quota, *mine),
                              row_class_quota(neg_edge_quota, *mine))
    else:
      got_n = ctx.sample_fobe(seed, K, nq, eq)
    if row_bounds is not None:
      cap = int(np.asarray(row_bounds[0], np.int64)[mine[0]::mine[1]].sum() +
                np.asarray(row_bounds[1], np.int64)[mine[0]::mine[1]].sum())
      if got_n > cap:
        raise RuntimeError("rank %d's share of row class %d/%d sampled %d "
                           "records, above its bound %d" %
                           (rank, off, stride, got_n, cap))
    ctx.store_append()
    new = ctx.store_info()[0] - before
    t = torch.tensor([new], dtype=torch.int64, device=dev)
    got = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(got, t, group=group)
    cnt = [int(g.item()) for g in got]
    if pending is not None:  # the previous class's exchange is done by now
      finish(pending)
      pending = None
    m = max(cnt)
    if m == 0:
      continue
    send = torch.zeros((m, 3), dtype=torch.int32, device=dev)
    if new:
      if gpu:
        torch.cuda.current_stream(dev).synchronize()
        ctx.store_read(before, new, dst_ptr=send.data_ptr())
      else:
        send[:new] = torch.from_numpy(ctx.store_read(before, new).view(np.int32))
    recv = [torch.empty_like(send) for _ in range(world)]
    work = dist.all_gather(recv, send, group=group, async_op=True)
    pending = (work, recv, cnt, send)  # buffers live until the gather ends
  if pending is not None:
    finish(pending)
  if gpu:
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
  n = ctx.store_info()[0]
  tot = torch.tensor([n], dtype=torch.int64, device=dev)
  dist.all_reduce(tot, op=dist.ReduceOp.MAX, group=group)
  assert int(tot.item()) == n, "ranks hold stores of different sizes"
  return n


def BooleanSamples(hypergraph, num_neighbors, num_samples, neg_samples=0,
                   disable_pbar=False):
  """hg2v_sample.py:125-242 (expects a compressed hypergraph, as the
  skeleton passes; ids are the compressed ones)."""
  del disable_pbar
  inc = Incidence.from_hypergraph(hypergraph)
  return sample_fobe(inc, num_neighbors, num_samples,
                     neg_samples).to_similarity_records()


def AlgebraicDistanceSamples(hypergraph, algebraic_embedding, num_neighbors,
                             num_samples, run_in_parallel=True,
                             disable_pbar=False):
  """hg2v_sample.py:632-717: probabilities from the (float32) alg coords of
  `algebraic_embedding`, keyed like the compressed hypergraph."""
  del run_in_parallel, disable_pbar
  inc = Incidence.from_hypergraph(hypergraph)
  x = np.array([algebraic_embedding.node[int(i)].values for i in inc.node_ids],
               np.float32)
  y = np.array([algebraic_embedding.edge[int(i)].values for i in inc.edge_ids],
               np.float32)
  return sample_hobe(inc, num_neighbors, num_samples,
                     alg_coords=(x, y)).to_similarity_records()


def _incidence_values(inc, m, node_major):
  """Values of feature matrix m (node2features N x E, or edge2features
  E x N) at the incidences of inc, in A's (node_major) or A^T's CSR order.
  m must not have nonzeros outside the incidence pattern."""
  m = sp.csr_matrix(m, dtype=np.float32)
  if node_major:
    rows = np.repeat(np.arange(inc.N), np.diff(inc.rp_n))
    cols = inc.col_n
    shape = (inc.N, inc.E)
  else:
    rows = np.repeat(np.arange(inc.E), np.diff(inc.rp_e))
    cols = inc.col_e
    shape = (inc.E, inc.N)
  assert m.shape[0] >= shape[0] and m.shape[1] >= shape[1]
  vals = np.asarray(m[rows, cols], dtype=np.float32).ravel()
  outside = float(np.abs(m).sum()) - float(np.abs(vals).sum())
  assert abs(outside) <= 1e-6 * max(1.0, float(np.abs(vals).sum())), \
      "feature matrix has entries outside the incidence pattern"
  return vals


def sample_jaccard(inc, node_features, edge_features, num_neighbors,
                   num_samples, ctx=None, seed=None, rng=None):
  """WeightedJaccardSamples on the device (features as per-incidence values,
  node-major / edge-major); returns DeviceRecords. rng="mt19937": numpy's
  global stream (run_in_parallel=False semantics), the reference's records
  bit for bit."""
  assert num_neighbors >= 1
  assert num_samples >= 0
  check_rng(rng)
  ctx = ctx or get_context()
  ctx.upload(inc)
  ctx.features_set(node_features, edge_features)
  nq = _quotas(inc.node_weight, num_samples)
  eq = _quotas(inc.edge_weight, num_samples)
  if rng == "mt19937":
    n = ctx.sample_jaccard_mt(num_neighbors, nq, eq)
  else:
    n = ctx.sample_jaccard(numpy_seed() if seed is None else seed,
                           num_neighbors, nq, eq)
  return DeviceRecords(ctx, inc, n, num_neighbors)


def WeightedJaccardSamples(hypergraph, node2features, edge2features,
                           num_neighbors, num_samples, run_in_parallel=True,
                           disable_pbar=False):
  """hg2v_sample.py:395-510 (node2features N x E, edge2features E x N on
  the compressed hypergraph's incidence pattern, e.g. UniformWeight /
  WeightByNeighborhood)."""
  del run_in_parallel, disable_pbar
  inc = Incidence.from_hypergraph(hypergraph)
  fn = _incidence_values(inc, node2features, True)
  fe = _incidence_values(inc, edge2features, False)
  return sample_jaccard(inc, fn, fe, num_neighbors,
                        num_samples).to_similarity_records()


def _same_type_dist_calc(indices, inc, alg_x, alg_y, is_edge, ctx=None):
  """hg2v_sample.py:527-543 for one pair (device computed, bit-exact)."""
  ctx = ctx or get_context()
  ctx.upload(inc)
  ctx.alg_set(alg_x, alg_y)
  kind = _hgx.HOBE_EE if is_edge else _hgx.HOBE_NN
  return float(ctx.hobe_probs(kind, [indices[0]], [indices[1]])[0])


################################################################################
# Samples to model input (hg2v_sample.py:725-797), host side                   #
################################################################################


def _inc_or_zero(x):
  return 0 if x is None else x + 1


def _val_or_zero(x):
  return 0 if x is None else x


def _pad_or_val(arr, idx):
  if arr is None or idx >= len(arr):
    return 0
  return arr[idx]


def _pad_or_inc(arr, idx):
  if arr is None or idx >= len(arr):
    return 0
  return arr[idx] + 1


def SamplesToModelInput(similarity_records, num_neighbors, weighted=True):
  """Records -> (features, targets) lists, exactly as hg2v_sample.py:751-797."""
  K = num_neighbors
  ln, le, rn, re, lw, rw = [], [], [], [], [], []
  nn = [[] for _ in range(K)]
  nnw = [[] for _ in range(K)]
  ne = [[] for _ in range(K)]
  new = [[] for _ in range(K)]
  p_nn, p_ee, p_ne = [], [], []
  for r in similarity_records:
    ln.append(_inc_or_zero(r.left_node_idx))
    rn.append(_inc_or_zero(r.right_node_idx))
    le.append(_inc_or_zero(r.left_edge_idx))
    re.append(_inc_or_zero(r.right_edge_idx))
    lw.append(_val_or_zero(r.left_weight))
    rw.append(_val_or_zero(r.right_weight))
    for i in range(K):
      nn[i].append(_pad_or_inc(r.neighbor_node_indices, i))
      ne[i].append(_pad_or_inc(r.neighbor_edge_indices, i))
      if weighted:
        nnw[i].append(_pad_or_val(r.neighbor_node_weights, i))
        new[i].append(_pad_or_val(r.neighbor_edge_weights, i))
    p_nn.append(_val_or_zero(r.node_node_prob))
    p_ee.append(_val_or_zero(r.edge_edge_prob))
    p_ne.append(_val_or_zero(r.node_edge_prob))
  features = [ln, le, rn, re]
  if weighted:
    features += [lw, rw]
  features += nn
  if weighted:
    features += nnw
  features += ne
  if weighted:
    features += new
  return features, [p_nn, p_ee, p_ne]


def ModelInputToArrays(features, targets):
  """(features, targets) of SamplesToModelInput(weighted=False) -> the
  (n, 4+2K) int32 / (n, 3) float32 arrays hgx_records_set takes."""
  idx = np.ascontiguousarray(np.array(features, dtype=np.int64).T,
                             dtype=np.int32)
  tgt = np.ascontiguousarray(np.array(targets, dtype=np.float64).T,
                             dtype=np.float32)
  return idx, tgt


__all__ = ["SimilarityRecord", "BooleanSamples", "AlgebraicDistanceSamples",
           "WeightedJaccardSamples", "sample_jaccard",
           "SamplesToModelInput", "ModelInputToArrays", "DeviceRecords",
           "sample_sharded", "sharded_store_fill", "shard_range",
           "row_class_quota",
           "sample_fobe", "sample_hobe", "records_from_arrays"]
