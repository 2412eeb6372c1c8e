"""Interleaved A/B of the trainer's workgroup size (tuning `train_tb`: 128,
256, 512 threads = 2, 4, 8 records per workgroup) at d = 256 on the C4 HOBE
stream (power-law 10M/5M, a seeded 1% row slice, full-size tables), in one
process: epochs alternate between the settings, per-batch device time
(hgx_train_last_stats) per setting. Diagnostic only.

  python tools/ab_tb_d256.py [rounds=3] [frac=0.01]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx  # noqa: E402
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.01
big = powerlaw_hypergraph(seed=0)
ctx = _hgx.Context(0)
ctx.upload(big)
rs4 = np.random.RandomState(1)
ctx.alg_set(rs4.random_sample((big.N, 10)).astype(np.float32),
            rs4.random_sample((big.E, 10)).astype(np.float32))
ctx.alg_run(20)
rsq = np.random.RandomState(2)
nq = np.where(rsq.random_sample(big.N) < frac, 200, 0).astype(np.int32)
eq = np.where(rsq.random_sample(big.E) < frac, 200, 0).astype(np.int32)
n = ctx.sample_hobe(4000, 5, 200, node_q=nq, edge_q=eq)
print(json.dumps({"records": n}), flush=True)
res = {}
for r in range(rounds):
  for tb in (256, 128, 512):
    ctx.set_tuning("train_tb", tb)
    ctx.model_init(256, big.N + 1, big.E + 1, seed=11)
    ctx.train(batch=256, max_epochs=1, loss=_hgx.LOSS_MSE, act=_hgx.ACT_RELU,
              min_delta=-1e30, shuffle_seed=2)
    ms, rec, bat = ctx.train_stats()
    us = ms * 1e3 / bat
    nt, et = ctx.model_get()
    res.setdefault(tb, []).append(us)
    print(json.dumps({"round": r, "tb": tb, "per_batch_us": round(us, 3),
                      "loss": float(ctx.train_loss_sum() / rec),
                      "node_sum": float(np.float64(nt[:100000]).sum())}), flush=True)
    del nt, et
print(json.dumps({"median_us": {k: round(float(np.median(v)), 3) for k, v in res.items()},
                  "min_us": {k: round(float(np.min(v)), 3) for k, v in res.items()}}), flush=True)
ctx.close()
