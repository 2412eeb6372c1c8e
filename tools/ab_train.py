"""Interleaved A/B timing of trainer builds in ONE process (box-to-box and
run-to-run drift cancel): each library (same C ABI, e.g. tools/_ab/*.so) gets
its own context with the same records and model; epochs alternate A, B, ...
and the per-batch device time (hgx_train_last_stats) is reported per build as
min / median over rounds. Diagnostic only.

  python tools/ab_train.py D {rand|hobe} lib1.so[:key=v,key=v] lib2.so ...

Also the whole hgx_train call's wall rate (records / s, preparation and host
waits included) per build.
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

d = int(sys.argv[1])
kind = sys.argv[2]
libs = sys.argv[3:]
N, E, K = 100000, 50000, 5
R = 4 + 2 * K
n = int(os.environ.get("AB_N", 2_000_000))
rs = np.random.RandomState(0)
if kind == "hobe":
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import random_hypergraph
  c = _hgx.Context(0)
  inc = random_hypergraph(seed=0)
  c.upload(inc)
  r = np.random.RandomState(4)
  c.alg_set(r.random_sample((inc.N, 10)), r.random_sample((inc.E, 10)))
  c.alg_run(20)
  m = c.sample_hobe(17, 5, 200)
  idx, tgt = c.records_get()
  sel = np.random.RandomState(1).permutation(m)[:n]
  idx, tgt = np.ascontiguousarray(idx[sel]), np.ascontiguousarray(tgt[sel])
  c.close()
else:
  idx = np.zeros((n, R), np.int32)
  kd = rs.randint(0, 3, n)
  m0, m1, m2 = kd == 0, kd == 1, kd == 2
  idx[m0, 0] = rs.randint(1, N + 1, m0.sum()); idx[m0, 2] = rs.randint(1, N + 1, m0.sum())
  idx[m1, 1] = rs.randint(1, E + 1, m1.sum()); idx[m1, 3] = rs.randint(1, E + 1, m1.sum())
  idx[m2, 0] = rs.randint(1, N + 1, m2.sum()); idx[m2, 3] = rs.randint(1, E + 1, m2.sum())
  idx[m2, 4:4 + K] = rs.randint(1, N + 1, (m2.sum(), K))
  idx[m2, 4 + K:] = rs.randint(1, E + 1, (m2.sum(), K))
  tgt = np.zeros((n, 3), np.float32)
  tgt[np.arange(n), kd] = rs.uniform(0, 1, n)

vp = ctypes.c_void_p
hs = []
for spec in libs:
  path, _, tune = spec.partition(":")  # lib.so[:key=value] (hgx_set_tuning)
  L = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
  L.hgx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
  L.hgx_records_set.argtypes = [vp, ctypes.c_int64, ctypes.c_int, vp, vp]
  L.hgx_model_init.argtypes = [vp, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                               ctypes.c_uint64, vp, vp]
  L.hgx_train.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                          ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                          ctypes.c_uint64, vp, vp, ctypes.POINTER(ctypes.c_int)]
  L.hgx_train_last_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_int64),
                                     ctypes.POINTER(ctypes.c_int64)]
  h = vp()
  assert L.hgx_create(0, ctypes.byref(h)) == 0
  for kv in filter(None, tune.split(",")):  # lib.so:k=v,k=v
    key, val = kv.split("=")
    L.hgx_set_tuning.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64]
    assert L.hgx_set_tuning(h, key.encode(), int(val)) == 0
  assert L.hgx_records_set(h, n, K, idx.ctypes.data, tgt.ctypes.data) == 0
  assert L.hgx_model_init(h, d, N + 2, E + 2, 1, None, None) == 0
  hs.append((L, h))

loss = np.zeros(1, np.float32)
ran = ctypes.c_int()
res = [[] for _ in libs]
wall = [[] for _ in libs]
for rnd in range(6):
  for i, (L, h) in enumerate(hs):
    t0 = time.perf_counter()
    assert L.hgx_train(h, 256, 1, 0.01, 1e-7, 1, 1, -1e30, rnd, None,
                       loss.ctypes.data, ctypes.byref(ran)) == 0
    if rnd > 0:
      wall[i].append(n / (time.perf_counter() - t0))
    ms, rec, bat = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
    L.hgx_train_last_stats(h, ctypes.byref(ms), ctypes.byref(rec), ctypes.byref(bat))
    if rnd > 0:
      res[i].append(ms.value * 1e3 / bat.value)
for path, r, w in zip(libs, res, wall):
  print(f"{kind} d={d} {os.path.basename(path):>40s}: us/batch min {min(r):.3f} "
        f"median {np.median(r):.3f}; epoch wall {np.median(w) / 1e6:.2f}M records/s "
        f"(max {max(w) / 1e6:.2f}M)")
