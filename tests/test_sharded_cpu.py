"""Multi-rank alg-dist driver on CPU: world_size 2 and 3 over gloo.

The driver (algebraic_distance.alg_dist_sharded) is the one bench.py runs
over RCCL; here each rank's kernels are the numpy restatement in
shard_emu.py, so the test covers the decomposition (row shards, SUM of the
edge partials, MAX of the order-preserving min/max words) against the
reference's float64 golden vectors.
"""

import os
import socket
import sys

import numpy as np
import pytest

from conftest import golden, golden_incidence
from hypergraphembedding_amd.algebraic_distance import shard_rows


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _worker(rank, world, port, out_path, iters, compact=True, graph="tiny",
            edge_ranges=1):
  import torch
  import torch.distributed as dist
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  sys.path[:0] = [root, os.path.join(root, "oracle"),
                  os.path.join(root, "tests")]
  import oracle as O
  from conftest import golden_incidence as gi
  from shard_emu import ShardEmu
  from hypergraphembedding_amd.algebraic_distance import alg_dist_sharded
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  inc = gi("csr_tiny.npz") if graph == "tiny" else _local_graph()
  r = O.Rng(0)
  x0, y0 = r.random((inc.N, 10)), r.random((inc.E, 10))
  st = {}
  (r0, r1, xo), y, _ = alg_dist_sharded(ShardEmu(), inc, x0, y0, iters,
                                        device=torch.device("cpu"),
                                        compact=compact, stats=st,
                                        edge_ranges=edge_ranges)
  np.savez(out_path + f".{rank}.npz", r0=r0, r1=r1, x=xo, y=y,
           wire=st["partial_bytes_per_iter"],
           dense=st["dense_partial_bytes_per_iter"])
  dist.barrier()
  dist.destroy_process_group()


def _local_graph():
  """Two communities of 60 nodes / 20 edges each (node ids ordered by
  community) joined by 3 bridge edges: most edges sit on one rank."""
  from hypergraphembedding_amd.hypergraph_util import Incidence
  rs = np.random.RandomState(7)
  rows, cols = [], []
  for c in range(2):
    for v in range(60):
      for e in rs.choice(20, 3, replace=False):
        rows.append(60 * c + v)
        cols.append(20 * c + e)
  for b in range(3):
    for v in (b, 60 + b):
      rows.append(v)
      cols.append(40 + b)
  a = np.unique(np.array(rows) * 64 + np.array(cols))
  rows, cols = a // 64, a % 64
  rp = np.searchsorted(rows, np.arange(121))
  return Incidence(120, 43, rp, cols)


@pytest.mark.parametrize("world,compact,ranges", [(2, True, 1), (3, True, 1),
                                                  (2, False, 1), (3, True, 4),
                                                  (2, False, 3)])
def test_sharded_driver_gloo(tmp_path, world, compact, ranges):
  """ranges > 1: the exchange pipelined over edge ranges (async all-reduce of
  range r while range r + 1's partials are computed)."""
  import torch.multiprocessing as mp
  iters = 20
  out = str(tmp_path / "shard")
  mp.start_processes(_worker, args=(world, _free_port(), out, iters, compact,
                                    "tiny", ranges),
                     nprocs=world, join=True, start_method="spawn")
  inc = golden_incidence("csr_tiny.npz")
  z = golden("algdist_tiny.npz")
  x = np.full((inc.N, 10), np.nan, np.float32)
  ys = []
  for r in range(world):
    d = np.load(out + f".{r}.npz")
    x[int(d["r0"]):int(d["r1"])] = d["x"]
    ys.append(d["y"])
  assert not np.isnan(x).any()  # the shards tile the node rows
  for y in ys[1:]:
    assert np.array_equal(y, ys[0])  # edge coords replicated identically
  assert np.abs(x - z["x_20"]).max() <= 1e-4
  assert np.abs(ys[0] - z["y_20"]).max() <= 1e-4


@pytest.mark.parametrize("world", [1, 2, 3, 8, 64])
def test_shard_rows_tile_and_balance(world, small_inc):
  rp = small_inc.rp_n
  spans = [shard_rows(rp, world, r) for r in range(world)]
  assert spans[0][0] == 0 and spans[-1][1] == small_inc.N
  for (a, b), (c, d) in zip(spans, spans[1:]):
    assert b == c and a <= b
  loads = [int(rp[b] - rp[a]) for a, b in spans]
  assert sum(loads) == small_inc.nnz
  max_deg = int(np.diff(rp).max())
  assert max(loads) <= small_inc.nnz / world + max_deg + 1


def test_order_words_roundtrip():
  from shard_emu import f2ord, ord2f
  v = np.array([-np.inf, -3.5, -1e-30, -0.0, 0.0, 1e-30, 0.25, 7.0, np.inf],
               np.float32)
  w = f2ord(v)
  assert np.all(np.diff(w.astype(np.int64)) >= 0)  # order preserving
  assert np.array_equal(ord2f(w), v)
  assert np.all(np.diff((~w).astype(np.int64)) <= 0)  # ~ reverses order


def test_sharded_compact_exchange_local_edges(tmp_path):
  """A graph whose edges mostly sit on one rank: only the bridge edges go on
  the wire (k + 1 floats each), and the result still equals the oracle."""
  import torch.multiprocessing as mp
  sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(
      os.path.abspath(__file__))), "oracle"))
  import oracle as O
  world, iters = 2, 15
  out = str(tmp_path / "local")
  mp.start_processes(_worker, args=(world, _free_port(), out, iters, True,
                                    "local"),
                     nprocs=world, join=True, start_method="spawn")
  inc = _local_graph()
  r = O.Rng(0)
  x0, y0 = r.random((inc.N, 10)), r.random((inc.E, 10))
  xr, yr = O.algdist(inc, x0, y0, iters)
  x = np.zeros((inc.N, 10), np.float32)
  for rk in range(world):
    d = np.load(out + f".{rk}.npz")
    x[int(d["r0"]):int(d["r1"])] = d["x"]
    assert np.abs(d["y"] - yr).max() <= 1e-4  # every rank has every edge
    assert int(d["wire"]) == 3 * 11 * 4  # the 3 bridge edges, k + 1 floats
    assert int(d["dense"]) == inc.E * 12 * 4
  assert np.abs(x - xr).max() <= 1e-4


# ---- row-sharded sampling into the record store (sharded_store_fill) --------
def _chunks(inc, n):
  from hypergraphembedding_amd.embedding import _row_chunks
  per_row = 12
  budget = -(-per_row * (inc.N + inc.E) // n)
  return _row_chunks(np.full(inc.N, per_row), np.full(inc.E, per_row), budget)


def _store_worker(rank, world, port, out_path, n_chunks):
  import torch.distributed as dist
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  sys.path[:0] = [root, os.path.join(root, "oracle"),
                  os.path.join(root, "tests")]
  from conftest import golden_incidence as gi
  from shard_emu import SampleEmu
  from test_sharded_cpu import _chunks
  from hypergraphembedding_amd.hg2v_sample import sharded_store_fill
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  inc = gi("csr_small.npz")
  emu = SampleEmu()
  emu.upload(inc)
  n = sharded_store_fill(inc, 3, 6, _chunks(inc, n_chunks), ctx=emu, seed=77,
                         kind="hobe", device="cpu")
  assert n == emu.store_info()[0]
  np.savez(out_path + f".{rank}.npz", store=emu.store_read())
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_store_fill_equals_single_process(tmp_path, world):
  """Strided row classes sampled over gloo ranks (each rank a strided share
  of each class's rows), each class's store entries all-gathered while the
  next class samples: every rank's record store holds exactly the entries
  a single process stores for the whole stream (as a multiset: the store's
  epoch order is keyed by record identity, not position)."""
  import torch.multiprocessing as mp
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from shard_emu import SampleEmu
  out = str(tmp_path / "store")
  mp.start_processes(_store_worker, args=(world, _free_port(), out, 3),
                     nprocs=world, join=True, start_method="spawn")
  inc = golden_incidence("csr_small.npz")
  assert len(_chunks(inc, 3)) >= 3
  emu = SampleEmu()
  emu.upload(inc)
  emu.sample_hobe(77, 3, 6)
  emu.store_reset()
  emu.store_append()
  ref = emu.store_read()
  key = lambda e: np.sort(e[:, 0].astype(np.uint64) << np.uint64(32) |
                          e[:, 1].astype(np.uint64))
  for r in range(world):
    st = np.load(out + f".{r}.npz")["store"]
    assert st.shape == ref.shape
    assert np.array_equal(key(st), key(ref))
    o1 = np.lexsort(st.T[::-1])
    o2 = np.lexsort(ref.T[::-1])
    assert np.array_equal(st[o1], ref[o2])


def test_row_chunks_respect_per_row_bounds():
  """the strided classes are sized from the rows' actual
  bounds: a class holding the heavy-quota rows stays within the budget."""
  from hypergraphembedding_amd.embedding import _row_chunks
  bn = np.full(1000, 2, np.int64)
  bn[::50] = 400  # 20 heavy rows, all in class 0 of a stride of 2, 5, 10, 25, 50
  be = np.full(300, 2, np.int64)
  budget = 1000
  chunks = _row_chunks(bn, be, budget)
  n = chunks[0][1]
  cls = (np.bincount(np.arange(bn.size) % n, weights=bn, minlength=n) +
         np.bincount(np.arange(be.size) % n, weights=be, minlength=n))
  assert cls.max() <= budget
  assert [c for c, _ in chunks] == list(range(n))
  assert n > -(-int(bn.sum() + be.sum()) // budget)  # the even split was not


def test_fill_store_checks_each_class_against_its_bound():
  """fill_store samples every strided class once, appends it, and refuses a
  class whose sampled count exceeds the class's record bound (the sampler
  holds one class at a time; the trainer's loads are sized from it)."""
  from hypergraphembedding_amd.embedding import fill_store

  class FakeStore:
    def __init__(self):
      self.n, self.appends, self.cap = 0, 0, None

    def store_reset(self, cap):
      self.n, self.cap = 0, cap

    def store_append(self):
      self.appends += 1

    def store_info(self):
      return (self.n, 1, 5, 0)

  bn = np.full(100, 4, np.int64)
  be = np.full(40, 4, np.int64)
  ctx = FakeStore()
  seen = []

  def ok(off, stride):
    seen.append((off, stride))
    m = int(bn[off::stride].sum() + be[off::stride].sum())
    ctx.n += m
    return m

  assert fill_store(ctx, None, ok, bn, be, 100) == int(bn.sum() + be.sum())
  assert ctx.cap == int(bn.sum() + be.sum())
  assert ctx.appends == len(seen) and sorted(o for o, _ in seen) == list(range(seen[0][1]))

  def too_many(off, stride):
    return int(bn[off::stride].sum() + be[off::stride].sum()) + 1

  with pytest.raises(RuntimeError, match="above its bound"):
    fill_store(FakeStore(), None, too_many, bn, be, 100)


def test_sharded_store_fill_argument_checks():
  """FOBE needs its quotas; negative quotas come in pairs and only for FOBE
  (checked before any collective)."""
  from hypergraphembedding_amd.hg2v_sample import sharded_store_fill
  q = np.ones(4, np.int32)
  with pytest.raises(ValueError, match="needs its row quotas"):
    sharded_store_fill(None, 2, 3, [(0, 1)], kind="fobe")
  with pytest.raises(ValueError, match="both negative quotas"):
    sharded_store_fill(None, 2, 3, [(0, 1)], kind="fobe", node_quota=q,
                       edge_quota=q, neg_node_quota=q)
  with pytest.raises(ValueError, match="FOBE"):
    sharded_store_fill(None, 2, 3, [(0, 1)], kind="hobe", neg_node_quota=q,
                       neg_edge_quota=q)
