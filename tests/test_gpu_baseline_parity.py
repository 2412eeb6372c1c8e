"""Trainer parity at BASELINE size (SURVEY §8c tolerance).

C3 (BASELINE.json configs[2]): one full HOBE epoch on the random 100k/50k
graph -- every record the device samples (~60M, d = 128, batch 256) --
trained on the GPU and by the oracle with identical initial tables and the
same batch order (the device takes the permutation as `perms`). The oracle at
this size is cpu_train_mt.c's checker build (oracle/libcpumt_chk.so: the
records of a batch over OpenMP threads, every product and sum rounded like
hgref_train; tests/test_cpu_baseline.py pins it to hgref_train), since the
scalar hgref_train would take ~8 minutes. Bar: epoch loss rtol 1e-4, per-row
cosine p50 >= 0.9999 and p1 >= 0.999 on both tables.

C2 (configs[1]): the same for one full FOBE epoch (BooleanModel: KLD loss,
sigmoid heads, hg2v_model.py:51-125, embedding.py:308-329) at d = 128 --
the model and instantiation bench.py's c2_fobe_d128 leg times.

The C4 windows (configs[3], 10M/5M power-law, d = 256, full-size tables,
the MULTI form on >= 40% of the batches; HOBE and the FOBE half of C5) are
in tests/test_gpu_c4.py, where the graph is already built.

Keras itself is absent from the image: the trainer stays "parity unpinned"
against the reference; these tests pin the device against the restatement
at the sizes the bench runs.
"""

import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def row_cos(a, b):
  a = a.astype(np.float64)
  b = b.astype(np.float64)
  num = (a * b).sum(1)
  den = np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1)
  ok = den > 0
  return num[ok] / den[ok]


def _threads():
  # each checker runs beside the other on the box's 16-core CPU share
  # (conftest.Background: two workers)
  return max(1, min(8, len(os.sched_getaffinity(0))))


def _device_epoch(kind):
  """One full epoch of the C3 HOBE (kind "c3") or C2 FOBE ("c2") stream on
  the GPU from seeded tables and a seeded permutation. Returns what the
  checker needs: the stream in batch order, the initial tables, the device
  loss and tables."""
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import random_hypergraph
  inc = random_hypergraph(seed=0)
  K, S, d = 5, 200, 128
  ctx = _hgx.Context(0)
  try:
    ctx.upload(inc)
    if kind == "c3":
      r = np.random.RandomState(4)
      ctx.alg_set(r.random_sample((inc.N, 10)), r.random_sample((inc.E, 10)))
      ctx.alg_run(20)
      n = ctx.sample_hobe(17, K, S)
      assert n > 55_000_000
      rs = np.random.RandomState(12)
      loss, act = _hgx.LOSS_MSE, _hgx.ACT_RELU
    else:
      n = ctx.sample_fobe(31, K, np.full(inc.N, S, np.int32),
                          np.full(inc.E, S, np.int32))
      assert n > 30_000_000
      rs = np.random.RandomState(14)
      loss, act = _hgx.LOSS_KLD, _hgx.ACT_SIGMOID
    nt = rs.uniform(-0.05, 0.05, (inc.N + 1, d)).astype(np.float32)
    et = rs.uniform(-0.05, 0.05, (inc.E + 1, d)).astype(np.float32)
    perm = rs.permutation(n)
    ctx.model_init(d, inc.N + 1, inc.E + 1, node_tab=nt, edge_tab=et)
    gl = ctx.train(batch=256, max_epochs=1, loss=loss, act=act,
                   perms=perm[None, :], min_delta=-1e30)
    fused, split = ctx.train_path_stats()
    assert split == 0 and fused == -(-n // 256)
    gnt, get_ = ctx.model_get()
    idx, tgt = ctx.records_get()
  finally:
    ctx.close()
  idx = np.ascontiguousarray(idx[perm])
  tgt = np.ascontiguousarray(tgt[perm])
  return dict(idx=idx, tgt=tgt, nt=nt, et=et, gl=gl, gnt=gnt, get=get_, K=K,
              loss=O.LOSS_MSE if kind == "c3" else O.LOSS_KLD,
              act=O.ACT_RELU if kind == "c3" else O.ACT_SIGMOID)


def checker(data):
  """The checker build of the trainer port (bit-for-bit hgref_train
  rounding, threaded) on the device's stream, order and init; returns
  (device loss, oracle loss, [(name, p50, p1, min cosine, max-abs)])."""
  ont, oet, oloss = O.train_mt(data["idx"], data["tgt"], data["K"], data["nt"],
                               data["et"], data["loss"], data["act"], epochs=1,
                               threads=_threads(), copy=False, exact=True)
  rows = []
  for g, o, name in ((data["gnt"], ont, "node"), (data["get"], oet, "edge")):
    c = row_cos(g[1:], o[1:])
    rows.append((name, np.percentile(c, 50), np.percentile(c, 1), c.min(),
                 np.abs(g - o).max()))
  return data["gl"], oloss, rows


def assert_checked(res):
  """epoch loss rtol 1e-4, per-row cosine p50 >= 0.9999 and
  p1 >= 0.999 on both tables."""
  gl, oloss, rows = res
  assert np.isclose(gl[0], oloss, rtol=1e-4), (gl, oloss)
  for name, p50, p1, cmin, mx in rows:
    print(f"{name}: cosine p50 {p50:.8f} p1 {p1:.8f} min {cmin:.8f} "
          f"max-abs {mx:.3e}")
    assert p50 >= 0.9999 and p1 >= 0.999, (name, p50, p1)


@pytest.mark.timeout(900)
def test_c3_full_hobe_epoch_device(background):
  """C3's device epoch; the checker runs in the background and
  test_gpu_zz_deferred.py::test_c3_full_hobe_epoch_vs_oracle asserts."""
  data = _device_epoch("c3")
  background.submit("c3", lambda: checker(data))


@pytest.mark.timeout(900)
def test_c2_full_fobe_epoch_device(background):
  """every record of the C2 FOBE stream (~34M: nn, ee
  and both node-edge blocks at S = 200, K = 5), d = 128, KLD + sigmoid, one
  epoch on the device; checked by test_c2_full_fobe_epoch_vs_oracle."""
  data = _device_epoch("c2")
  background.submit("c2", lambda: checker(data))
