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


def _worker(rank, world, port, out_path, iters, graph="tiny"):
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
  (r0, r1, xo), y, ms = alg_dist_sharded(ctx, inc, x0, y0, iters)
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


def test_sharded_algdist_powerlaw_long_rows(tmp_path):
  import torch.multiprocessing as mp
  world, iters = 2, 10
  out = str(tmp_path / "shard")
  mp.start_processes(_worker, args=(world, _free_port(), out, iters, "powerlaw"),
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


def _nccl_worker(rank, world, port, out_path):
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
  (r0, r1, xo), y, ms = alg_dist_sharded(ctx, inc, x0, y0, 20)
  np.savez(out_path, r0=r0, r1=r1, x=xo, y=y)
  dist.destroy_process_group()


def test_sharded_algdist_rccl_single_rank(tmp_path):
  """The bench's RCCL path (nccl backend, collectives on the shared torch
  stream) with one rank: the only RCCL configuration a 1-GPU box can run."""
  import torch.multiprocessing as mp
  out = str(tmp_path / "nccl.npz")
  mp.start_processes(_nccl_worker, args=(1, _free_port(), out), nprocs=1,
                     join=True, start_method="spawn")
  z = golden("algdist_tiny.npz")
  d = np.load(out)
  assert int(d["r0"]) == 0 and int(d["r1"]) == d["x"].shape[0]
  assert np.abs(d["x"] - z["x_20"]).max() <= 1e-4
  assert np.abs(d["y"] - z["y_20"]).max() <= 1e-4
