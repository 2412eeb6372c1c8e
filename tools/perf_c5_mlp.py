"""C5 combiner throughput: the N_E_SUPERVISED MLP (combine_embeddings_util.py
78-174: two towers in -> (in + d) / 2 -> d, head 2d -> d -> 1, Adagrad, MSE,
batch 256) on the dense-MLP engine (fp32 MFMA), d = 256 (in = 2d = 512 from
[FOBE | HOBE] concatenation), random-init synthetic tables and samples
(1/6 positives as in nnz + 5 nnz), one epoch per measurement. Reports
samples/s, TFLOP/s from the engine's flop count against the 157.3 TF fp32
matrix peak, and the implied time of one epoch at the C4/C5 sample count
(nnz = 2.0e8 positives + 5 nnz negatives = 1.2e9 samples).

  python tools/perf_c5_mlp.py [--samples 20000000] [--rows 1000000]
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
  p.add_argument("--samples", type=int, default=20_000_000)
  p.add_argument("--rows", type=int, default=1_000_000)
  p.add_argument("--dim", type=int, default=256)
  p.add_argument("--epochs", type=int, default=2)
  p.add_argument("--tune", action="append", default=[],
                 help="KEY=VALUE for hgx_set_tuning (repeatable)")
  a = p.parse_args()
  from hypergraphembedding_amd import _hgx
  d, ind = a.dim, 2 * a.dim
  rs = np.random.RandomState(0)
  nt = rs.uniform(-0.05, 0.05, (a.rows, ind)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (a.rows // 2, ind)).astype(np.float32)
  nr = rs.randint(0, a.rows, a.samples).astype(np.int32)
  er = rs.randint(0, a.rows // 2, a.samples).astype(np.int32)
  lab = (rs.random_sample(a.samples) < 1.0 / 6).astype(np.float32)
  ctx = _hgx.Context(0)
  for kv in a.tune:
    k, v = kv.split("=")
    ctx.set_tuning(k, int(v))
  mlp = _hgx.Mlp(ctx, _hgx.MLP_NE_SUPERVISED, ind, d)
  lims = [np.sqrt(6.0 / (k + n)) for k, n in mlp.shapes]
  w0 = np.concatenate([np.concatenate([rs.uniform(-l, l, k * n), np.zeros(n)])
                       for l, (k, n) in zip(lims, mlp.shapes)]).astype(np.float32)
  mlp.set_weights(w0)
  mlp.set_tables(nt, et)
  mlp.set_samples(nr, er, lab)
  out = {"workload": "N_E_SUPERVISED combiner MLP, in=%d d=%d, batch 256, "
                     "synthetic tables %d/%d rows, %d samples" %
                     (ind, d, a.rows, a.rows // 2, a.samples),
         "layers": mlp.shapes}
  runs = []
  for ep in range(a.epochs):
    ctx.synchronize()
    t = time.perf_counter()
    losses = mlp.fit(batch=256, max_epochs=1, min_delta=-1e30, seed=ep + 1)
    ctx.synchronize()
    wall = time.perf_counter() - t
    st = mlp.stats()
    runs.append({"wall_s": round(wall, 3), "device_ms": round(st["ms"], 2),
                 "samples": st["samples"], "loss": float(losses[-1]),
                 "flops": st["flops"]})
    print(json.dumps({"epoch": ep, **runs[-1]}), flush=True)
  best = min(runs, key=lambda r: r["device_ms"])
  sps = best["samples"] / (best["device_ms"] / 1e3)
  tf = best["flops"] / (best["device_ms"] / 1e3) / 1e12
  out.update(samples_per_s=round(sps, 1), tflops=round(tf, 2),
             mfma_f32_peak_tflops=157.3, frac_of_peak=round(tf / 157.3, 4),
             flops_per_sample=round(best["flops"] / best["samples"], 1),
             c4_samples_per_epoch=1.2e9,
             c4_epoch_s_implied=round(1.2e9 / sps, 1))
  print(json.dumps(out), flush=True)
  mlp.close()
  ctx.close()


if __name__ == "__main__":
  main()
