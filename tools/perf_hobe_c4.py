"""HOBE (HG2V_ALG_DIST) on the power-law 10M/5M graph (BASELINE configs[3]
shape): alg-dist k=10 x 20 iterations, AlgebraicDistanceSamples on a seeded
row slice (quota S on a fraction of node rows and edge rows, 0 elsewhere),
one d=256 training epoch. Prints one JSON line with the phase times.

  python tools/perf_hobe_c4.py [--frac 0.02] [--dim 256] [--no-train]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--frac", type=float, default=0.02)
  p.add_argument("--dim", type=int, default=256)
  p.add_argument("--N", type=int, default=10_000_000)
  p.add_argument("--E", type=int, default=5_000_000)
  p.add_argument("--no-train", action="store_true")
  p.add_argument("--mode3", type=int, default=0)
  p.add_argument("--mode3-shift", type=int, default=1)
  p.add_argument("--mode3-shift-e", type=int, default=1)
  a = p.parse_args()
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  out = {}
  t = time.time()
  g = powerlaw_hypergraph(N=a.N, E=a.E, seed=0)
  out["gen_s"] = round(time.time() - t, 2)
  out.update(nodes=g.N, edges=g.E, nnz=g.nnz, max_edge=int(g.edge_size().max()))
  ctx = _hgx.Context(0)
  ctx.set_tuning("sample_mode3", a.mode3)
  ctx.set_tuning("sample_mode3_shift", a.mode3_shift)
  ctx.set_tuning("sample_mode3_shift_e", a.mode3_shift_e)
  ctx.upload(g)
  rs = np.random.RandomState(1)
  ctx.alg_set(rs.random_sample((g.N, 10)).astype(np.float32),
              rs.random_sample((g.E, 10)).astype(np.float32))
  ctx.alg_run(20)
  out["alg_ms_per_iter"] = round(ctx.alg_stats()[0] / 20, 3)
  rsq = np.random.RandomState(2)
  S, K = 200, 5
  nq = np.where(rsq.random_sample(g.N) < a.frac, S, 0).astype(np.int32)
  eq = np.where(rsq.random_sample(g.E) < a.frac, S, 0).astype(np.int32)
  print(json.dumps({"phase": "sampling", **out}), flush=True)
  ctx.synchronize()
  t = time.perf_counter()
  n = ctx.sample_hobe(4000, K, S, node_q=nq, edge_q=eq)
  ctx.synchronize()
  out["sample_s"] = round(time.perf_counter() - t, 3)
  out["records"] = n
  out["rejection_rows"], out["fallback_rows"] = ctx.sample_stats()
  out["uniform_rows"] = ctx.sample_uniform_rows()
  out["rows_sampled"] = int((nq > 0).sum() + (eq > 0).sum())
  print(json.dumps({"phase": "sampled", **out}), flush=True)
  if not a.no_train:
    ctx.model_init(a.dim, g.N + 1, g.E + 1, seed=11)
    t = time.perf_counter()
    ctx.train(batch=256, max_epochs=1, loss=_hgx.LOSS_MSE, act=_hgx.ACT_RELU,
              min_delta=-1e30, shuffle_seed=2)
    ctx.synchronize()
    tt = time.perf_counter() - t
    ms, rec, bat = ctx.train_stats()
    out["train_records_per_s"] = round(n / tt, 1)
    out["per_batch_us"] = round(ms * 1e3 / max(bat, 1), 2)
  print(json.dumps(out), flush=True)


if __name__ == "__main__":
  main()
