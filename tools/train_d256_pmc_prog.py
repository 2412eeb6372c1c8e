"""Program profiled by the r05 d = 256 trainer counter passes (rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE, and --kernel-trace --stats): bench.py's
algdist_c4.hobe_d256 leg alone -- the power-law 10M/5M graph, alg-dist
k=10 x 20 iterations, HOBE on a seeded 2% of node rows and edge rows
(S = 200, K = 5), one training epoch at d = 256 on full-size tables
(train_step<64,4,5,2,256,{false,true}>: the plain and the MULTI
pending-slot form). `python tools/train_d256_pmc_prog.py [row fraction,
default 0.01]` (bench.py's leg: 0.02; per batch the same distribution)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx  # noqa: E402
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph  # noqa: E402

frac = float(sys.argv[1]) if len(sys.argv) > 1 else 0.01
big = powerlaw_hypergraph(seed=0)
print("graph", big.N, big.E, big.nnz, flush=True)
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
print("records", n, flush=True)
ctx.model_init(256, big.N + 1, big.E + 1, seed=11)
ctx.train(batch=256, max_epochs=1, loss=_hgx.LOSS_MSE, act=_hgx.ACT_RELU,
          min_delta=-1e30, shuffle_seed=2)
ms, rec, bat = ctx.train_stats()
print(json.dumps({"records": n, "batches": bat, "multi": ctx.train_multi_pending(),
                  "per_batch_us": round(ms * 1e3 / bat, 3)}), flush=True)
ctx.close()
