"""The C4 d = 256 trainer step on a seeded row slice of the power-law
10M/5M HOBE stream (bench.py's hobe_d256 leg at `frac`), `reps` epochs from
the same init: per-batch device time, MULTI batches, loss and a checksum of
the tables (A/B of two builds: HGX_LIB_PATH, run one after the other).

  python tools/ab_multi_d256.py [frac=0.01] [reps=3]"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx  # noqa: E402
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph  # noqa: E402

frac = float(sys.argv[1]) if len(sys.argv) > 1 else 0.01
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
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
for r in range(reps):
  ctx.model_init(256, big.N + 1, big.E + 1, seed=11)
  ctx.train(batch=256, max_epochs=1, loss=_hgx.LOSS_MSE, act=_hgx.ACT_RELU,
            min_delta=-1e30, shuffle_seed=2)
  ms, rec, bat = ctx.train_stats()
  out = {"rep": r, "records": n, "per_batch_us": round(ms * 1e3 / bat, 3),
         "multi": ctx.train_multi_pending(), "loss": ctx.train_loss_sum() / rec}
  if r == reps - 1:
    nt, et = ctx.model_get()
    h = hashlib.sha256()
    h.update(nt.tobytes())
    h.update(et.tobytes())
    out["tables_sha256"] = h.hexdigest()
  print(json.dumps(out), flush=True)
ctx.close()
