"""Trainer timing experiments: one process, variants selected through the
diagnostic env knobs read by each hgx_train call (HGX_TRAIN_ABLATE,
HGX_TRAIN_TB1, HGX_GRAPH). Prints us/batch per variant."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx

d = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
variants = sys.argv[3].split(",") if len(sys.argv) > 3 else ["base"]
rs = np.random.RandomState(0)
N, E, K = 100000, 50000, 5
R = 4 + 2 * K
idx = np.zeros((n, R), np.int32)
kind = rs.randint(0, 3, n)
m0, m1, m2 = kind == 0, kind == 1, kind == 2
idx[m0, 0] = rs.randint(1, N + 1, m0.sum()); idx[m0, 2] = rs.randint(1, N + 1, m0.sum())
idx[m1, 1] = rs.randint(1, E + 1, m1.sum()); idx[m1, 3] = rs.randint(1, E + 1, m1.sum())
idx[m2, 0] = rs.randint(1, N + 1, m2.sum()); idx[m2, 3] = rs.randint(1, E + 1, m2.sum())
idx[m2, 4:4 + K] = rs.randint(1, N + 1, (m2.sum(), K))
idx[m2, 4 + K:] = rs.randint(1, E + 1, (m2.sum(), K))
tgt = np.zeros((n, 3), np.float32)
tgt[np.arange(n), kind] = rs.uniform(0, 1, n)
ctx = _hgx.Context(0)
ctx.records_set(idx, tgt)
ctx.model_init(d, N + 2, E + 2, seed=1)
ENV = {"base": {}, "tb64": {"HGX_TRAIN_TB1": "64"}, "graph": {"HGX_GRAPH": "1"}}
for b in (1, 2, 3, 4, 8, 16, 32, 4 | 8, 16 | 32, 4 | 8 | 16 | 32):
  ENV[f"ab{b}"] = {"HGX_TRAIN_ABLATE": str(b)}
for v in variants:
  env = ENV[v] if v in ENV else dict(kv.split("=") for kv in v.split("+"))
  for k in ("HGX_TRAIN_ABLATE", "HGX_TRAIN_TB1", "HGX_GRAPH",
            "HGX_TRAIN_SERIAL", "HGX_TRAIN_G2"):
    os.environ.pop(k, None)
  os.environ.update(env)
  res = []
  for ep in range(2):
    t = time.time()
    ctx.train(batch=256, max_epochs=1, loss=1, act=1, min_delta=-1e30,
              shuffle_seed=ep)
    wall = time.time() - t
    ms, rec, bat = ctx.train_stats()
    res.append((ms * 1e3 / bat, wall))
  print(f"d={d} n={n} {v:12s} {res[-1][0]:7.2f} us/batch  "
        f"({rec / ms * 1e3 / 1e6:6.2f} Mrec/s, epoch wall {res[-1][1]:.3f}s)",
        flush=True)
