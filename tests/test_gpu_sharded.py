"""Node-row-sharded alg-dist on one GPU with two processes (gloo), checked
against the single-process device result and the float64 oracle.

The driver's 8-GPU scaling run uses the same code path with the nccl (=RCCL)
backend; only one GPU is available to the test, so both ranks share cuda:0.
"""

import os
import socket

import numpy as np
import pytest

import oracle as O
from conftest import golden, golden_incidence

pytestmark = pytest.mark.gpu


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _graph(name):
  if name == "tiny":
    from conftest import golden_incidence as gi
    return gi("csr_tiny.npz")
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  return powerlaw_hypergraph(N=20_000, E=10_000, seed=5)  # long edge rows


def _worker(rank, world, port, out_path, iters, graph="tiny", edge_ranges=1,
            ks=0):
  import torch
  import torch.distributed as dist
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
  from test_gpu_sharded import _graph
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.algebraic_distance import alg_dist_sharded
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  torch.cuda.set_device(0)
  inc = _graph(graph)
  r = O.Rng(0)
  x0, y0 = r.random((inc.N, 10)), r.random((inc.E, 10))
  ctx = _hgx.Context(0)
  ctx.set_tuning("alg_ks", ks)  # 16: the 64-B rows large graphs get
  (r0, r1, xo), y, ms = alg_dist_sharded(ctx, inc, x0, y0, iters,
                                         edge_ranges=edge_ranges)
  np.savez(out_path + f".{rank}.npz", r0=r0, r1=r1, x=xo, y=y)
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_algdist_matches_reference(tmp_path, world):
  import torch.multiprocessing as mp
  iters = 20
  out = str(tmp_path / "shard")
  mp.start_processes(_worker, args=(world, _free_port(), out, iters),
                     nprocs=world, join=True, start_method="spawn")
  inc = golden_incidence("csr_tiny.npz")
  z = golden("algdist_tiny.npz")
  x = np.zeros((inc.N, 10), np.float32)
  ys = []
  for r in range(world):
    d = np.load(out + f".{r}.npz")
    x[int(d["r0"]):int(d["r1"])] = d["x"]
    ys.append(d["y"])
  for y in ys[1:]:
    assert np.array_equal(y, ys[0])  # edge coords replicated identically
  assert np.abs(x - z["x_20"]).max() <= 1e-4
  assert np.abs(ys[0] - z["y_20"]).max() <= 1e-4


@pytest.mark.parametrize("ranges,ks", [(1, 0), (4, 0), (4, 16)])
def test_sharded_algdist_powerlaw_long_rows(tmp_path, ranges, ks):
  """ranges = 4: edge partials per range (each with its own long rows) and
  the exchange of each range issued asynchronously; ks = 16: 64-B
  coordinate rows (the library's choice above 256 MiB of rows), exchange
  buffers sized by the library's row width."""
  import torch.multiprocessing as mp
  world, iters = 2, 10
  out = str(tmp_path / "shard")
  mp.start_processes(_worker, args=(world, _free_port(), out, iters, "powerlaw",
                                    ranges, ks),
                     nprocs=world, join=True, start_method="spawn")
  inc = _graph("powerlaw")
  r = O.Rng(0)
  x0, y0 = r.random((inc.N, 10)), r.random((inc.E, 10))
  xr, yr = O.algdist(inc, x0, y0, iters)
  x = np.zeros((inc.N, 10), np.float32)
  for rk in range(world):
    d = np.load(out + f".{rk}.npz")
    x[int(d["r0"]):int(d["r1"])] = d["x"]
    y = d["y"]
  assert np.abs(x - xr).max() <= 1e-4
  assert np.abs(y - yr).max() <= 1e-4


def _nccl_worker(rank, world, port, out_path, edge_ranges=1):
  import torch
  import torch.distributed as dist
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
  from test_gpu_sharded import _graph
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.algebraic_distance import alg_dist_sharded
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  torch.cuda.set_device(0)
  dist.init_process_group("nccl", rank=rank, world_size=world,
                          device_id=torch.device("cuda", 0))
  inc = _graph("tiny")
  r = O.Rng(0)
  x0, y0 = r.random((inc.N, 10)), r.random((inc.E, 10))
  ctx = _hgx.Context(0)
  (r0, r1, xo), y, ms = alg_dist_sharded(ctx, inc, x0, y0, 20,
                                         edge_ranges=edge_ranges)
  np.savez(out_path, r0=r0, r1=r1, x=xo, y=y)
  dist.destroy_process_group()


@pytest.mark.parametrize("ranges", [1, 3])
def test_sharded_algdist_rccl_single_rank(tmp_path, ranges):
  """The bench's RCCL path (nccl backend, collectives on the shared torch
  stream; with ranges > 1 asynchronous per-range all-reduces) with one rank:
  the only RCCL configuration a 1-GPU box can run."""
  import torch.multiprocessing as mp
  out = str(tmp_path / "nccl.npz")
  mp.start_processes(_nccl_worker, args=(1, _free_port(), out, ranges), nprocs=1,
                     join=True, start_method="spawn")
  z = golden("algdist_tiny.npz")
  d = np.load(out)
  assert int(d["r0"]) == 0 and int(d["r1"]) == d["x"].shape[0]
  assert np.abs(d["x"] - z["x_20"]).max() <= 1e-4
  assert np.abs(d["y"] - z["y_20"]).max() <= 1e-4


# ---- row-sharded sampling -------------------------------
def _sample_setup(inc, kind, ctx):
  ctx.upload(inc)
  if kind == "hobe":
    r = O.Rng(2)
    ctx.alg_set(r.random((inc.N, 10)), r.random((inc.E, 10)))
    ctx.alg_run(5)


def _sample_worker(rank, world, port, out_path, kind, backend):
  import torch
  import torch.distributed as dist
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
  from test_gpu_sharded import _graph, _sample_setup
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.hg2v_sample import sample_sharded
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  torch.cuda.set_device(0)
  if backend == "nccl":
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", 0))
  else:
    dist.init_process_group("gloo", rank=rank, world_size=world)
  inc = _graph("powerlaw")
  ctx = _hgx.Context(0)
  _sample_setup(inc, kind, ctx)
  S = 20
  q = (np.full(inc.N, S, np.int32), np.full(inc.E, S, np.int32))
  total, sizes = sample_sharded(inc, 5, S, ctx=ctx, seed=123, kind=kind,
                                node_quota=q[0], edge_quota=q[1],
                                device=None if backend == "nccl" else "cpu")
  idx, tgt = ctx.records_get()
  assert idx.shape[0] == total == int(sizes.sum())
  np.savez(out_path + f".{rank}.npz", idx=idx, tgt=tgt, sizes=sizes,
           bounds=ctx.records_blocks())
  dist.barrier()
  dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,backend", [("hobe", 2, "gloo"),
                                                ("hobe", 3, "gloo"),
                                                ("fobe", 2, "gloo"),
                                                ("hobe", 1, "nccl")])
def test_row_sharded_sampling_equals_single_process(tmp_path, kind, world,
                                                    backend):
  """Every rank samples only its rows; after the count all-gather and the
  record all-gather, every rank holds the single-process stream: the same
  pairs, neighbour lists and probabilities in the reference's kind-block
  order (every draw is keyed by seed, row and rank in the row), neighbour
  lists drawn from the right rows."""
  import torch.multiprocessing as mp
  from hypergraphembedding_amd import _hgx
  out = str(tmp_path / "samp")
  mp.start_processes(_sample_worker,
                     args=(world, _free_port(), out, kind, backend),
                     nprocs=world, join=True, start_method="spawn")
  inc = _graph("powerlaw")
  ctx = _hgx.Context(0)
  _sample_setup(inc, kind, ctx)
  S = 20
  if kind == "hobe":
    n = ctx.sample_hobe(123, 5, S)
  else:
    n = ctx.sample_fobe(123, 5, np.full(inc.N, S, np.int32),
                        np.full(inc.E, S, np.int32))
  ridx, rtgt = ctx.records_get()
  rb = ctx.records_blocks()
  ctx.close()
  for r in range(world):
    d = np.load(out + f".{r}.npz")
    idx, tgt = d["idx"], d["tgt"]
    assert idx.shape[0] == n
    assert np.array_equal(idx, ridx)  # neighbour draws included
    assert np.array_equal(tgt, rtgt)
    if backend == "nccl":
      assert np.array_equal(d["bounds"], rb)
    assert d["sizes"].shape == (world, 4)
    assert np.array_equal(d["sizes"].sum(0), np.diff(rb))
    ne = (idx[:, 0] > 0) & (idx[:, 3] > 0) & (idx[:, 2] == 0)
    sel = np.flatnonzero(ne)[::97]
    for i in sel:
      v, e = idx[i, 0] - 1, idx[i, 3] - 1
      assert np.isin(idx[i, 4:9] - 1, inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]).all()
      assert np.isin(idx[i, 9:14] - 1, inc.col_n[inc.rp_n[v]:inc.rp_n[v + 1]]).all()


def _pipeline_worker(rank, world, port, out_path, budget, with_coords,
                     backend="gloo"):
  """embedding.hobe_sharded on `world` ranks sharing cuda:0 (gloo; nccl
  only at world 1)."""
  import torch
  import torch.distributed as dist
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  sys.path[:0] = [root, os.path.join(root, "oracle"), os.path.join(root, "tests")]
  from test_gpu_sharded import _graph
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.embedding import hobe_sharded
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  torch.cuda.set_device(0)
  if backend == "nccl":
    dist.init_process_group("nccl", rank=rank, world_size=world,
                            device_id=torch.device("cuda", 0))
  else:
    dist.init_process_group("gloo", rank=rank, world_size=world)
  inc = _graph("powerlaw")
  coords = None
  if with_coords:
    r = O.Rng(0)
    x, y = O.algdist(inc, r.random((inc.N, 10)), r.random((inc.E, 10)), 20)
    coords = (x.astype(np.float32), y.astype(np.float32))
  np.random.seed(7)  # rank 0's draws are broadcast (init coords, seeds)
  ctx = _hgx.Context(0)
  st = {}
  nt, et = hobe_sharded(inc, 16, num_neighbors=5, num_samples=20, epochs=2,
                        records_budget=budget, alg_coords=coords, ctx=ctx,
                        stats=st, edge_ranges=2)
  x, y = ctx.alg_get()
  np.savez(out_path + f".{rank}.npz", nt=nt, et=et, x=x, y=y)
  dist.barrier()
  dist.destroy_process_group()
  ctx.close()


@pytest.mark.parametrize("budget", [10**9, 300_000])
def test_hobe_pipeline_sharded_equals_single_process(tmp_path, budget):
  """The multi-GPU HOBE pipeline as one library call (embedding.hobe_sharded,
  EmbedHg2vAlgDist(group=)): with the same alg coordinates, 2 ranks (each
  sampling a strided share of every chunk's rows, all-gathered in row
  order, replicas training the same chunks) give tables bit-identical to 1
  rank -- with the stream resident (one chunk) and in 4+ strided chunks."""
  import torch.multiprocessing as mp
  out = {}
  for world in (1, 2):
    path = str(tmp_path / f"pipe{world}")
    mp.start_processes(_pipeline_worker,
                       args=(world, _free_port(), path, budget, True),
                       nprocs=world, join=True, start_method="spawn")
    out[world] = [np.load(path + f".{r}.npz") for r in range(world)]
  ref = out[1][0]
  assert np.isfinite(ref["nt"]).all()
  for d in out[2]:
    assert np.array_equal(d["nt"], ref["nt"])
    assert np.array_equal(d["et"], ref["et"])


def test_hobe_pipeline_rccl_single_rank_store_path(tmp_path):
  """The store path of the multi-GPU pipeline over RCCL (device buffers:
  class entries read from the store into a device tensor, all-gathered
  asynchronously, appended from device memory) with one rank -- the only
  RCCL configuration a 1-GPU box runs -- gives the gloo rank's tables bit
  for bit."""
  import torch.multiprocessing as mp
  out = {}
  for backend in ("gloo", "nccl"):
    path = str(tmp_path / backend)
    mp.start_processes(_pipeline_worker,
                       args=(1, _free_port(), path, 300_000, True, backend),
                       nprocs=1, join=True, start_method="spawn")
    out[backend] = np.load(path + ".0.npz")
  assert np.isfinite(out["nccl"]["nt"]).all()
  for k in ("nt", "et"):
    assert np.array_equal(out["nccl"][k], out["gloo"][k]), k


def test_hobe_pipeline_sharded_full_path(tmp_path):
  """Without given coordinates: the node-row-sharded relaxation, the
  all-gather of the node rows, strided chunks: every rank ends with the same
  coordinates (within 1e-4 of the float64 oracle from rank 0's draws) and
  the same tables."""
  import torch.multiprocessing as mp
  world = 2
  path = str(tmp_path / "full")
  mp.start_processes(_pipeline_worker,
                     args=(world, _free_port(), path, 300_000, False),
                     nprocs=world, join=True, start_method="spawn")
  d = [np.load(path + f".{r}.npz") for r in range(world)]
  for k in ("nt", "et", "x", "y"):
    assert np.array_equal(d[0][k], d[1][k]), k
  inc = _graph("powerlaw")
  np.random.seed(7)
  x0, y0 = np.random.random((inc.N, 10)), np.random.random((inc.E, 10))
  xr, yr = O.algdist(inc, x0.astype(np.float32), y0.astype(np.float32), 20)
  assert np.abs(d[0]["x"] - xr).max() <= 1e-4
  assert np.abs(d[0]["y"] - yr).max() <= 1e-4
