"""Ablation timing of the batch step (diagnostic build tools/_ab/dbg.so,
HGX_TRAIN_ABLATE bits, see hgx_train.hip): per-batch device time with one
part of the step removed at a time, interleaved over rounds in one process.
Results are wrong by construction; only the time is read.
  HGX_LIB_PATH=tools/_ab/dbg.so python tools/ablate_train.py [d] [hobe|rand]"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx
from hypergraphembedding_amd.synthetic import random_hypergraph

d = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ctx = _hgx.Context(0)
inc = random_hypergraph(seed=0)
ctx.upload(inc)
r = np.random.RandomState(4)
ctx.alg_set(r.random_sample((inc.N, 10)), r.random_sample((inc.E, 10)))
ctx.alg_run(20)
m = ctx.sample_hobe(17, 5, 200)
idx, tgt = ctx.records_get()
sel = np.random.RandomState(1).permutation(m)[:2_000_000]
ctx.records_set(idx[sel], tgt[sel])
bits = {0: "none", 2048: "row-0 partial loads", 4096: "forward reductions",
        8192: "Adagrad arithmetic", 16384: "end barrier + partial stores",
        32768: "list-slot gathers", 2048 | 4096 | 8192 | 16384: "all four compute/sync parts"}
res = {b: [] for b in bits}
for rnd in range(4):
  for b in bits:
    os.environ["HGX_TRAIN_ABLATE"] = str(b)
    ctx.model_init(d, inc.N + 1, inc.E + 1, seed=1)
    ctx.train(batch=256, max_epochs=1, min_delta=-1e30, shuffle_seed=rnd)
    ms, rec, bat = ctx.train_stats()
    if rnd:
      res[b].append(ms * 1e3 / bat)
os.environ["HGX_TRAIN_ABLATE"] = "0"
for b, name in bits.items():
  print(json.dumps({"ablate": b, "removed": name, "d": d,
                    "us_per_batch": round(float(np.median(res[b])), 3)}), flush=True)
