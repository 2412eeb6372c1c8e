"""The numpy-seeded HOBE sampler at BASELINE size (C3: random 100k/50k,
S=200, K=5, ~60M records): the device path (hgx_sample_hobe_mt) against the
oracle's single-threaded C replica of AlgebraicDistanceSamples
(run_in_parallel=False) on the same alg-dist coordinates -- every record
and numpy's state afterwards -- with both timings. The reference's own
Python path samples HOBE at ~17k records/s: about an hour
for this stream.

  python tools/mt_c3_hobe.py [--seed 5] [--no-oracle]
"""

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def sha(idx, tgt):
  h = hashlib.sha256()
  h.update(np.ascontiguousarray(idx, np.int32).tobytes())
  h.update(np.ascontiguousarray(tgt, np.float32).tobytes())
  return h.hexdigest()


def main():
  p = argparse.ArgumentParser()
  p.add_argument("--seed", type=int, default=5)
  p.add_argument("--no-oracle", action="store_true")
  a = p.parse_args()
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import random_hypergraph
  inc = random_hypergraph(seed=0)
  ctx = _hgx.Context(0)
  ctx.upload(inc)
  rs = np.random.RandomState(1)
  ctx.alg_set(rs.random_sample((inc.N, 10)), rs.random_sample((inc.E, 10)))
  ctx.alg_run(20)
  ax, ay = ctx.alg_get()
  ctx.alg_set(ax, ay)  # exactly the coordinates the oracle gets
  out = {"workload": "C3 HOBE stream, rng=mt19937 (numpy's MT19937 from "
                     "np.random.seed(%d)), S=200, K=5" % a.seed}
  np.random.seed(a.seed)
  ctx.synchronize()
  t = time.perf_counter()
  n = ctx.sample_hobe_mt(5, 200)
  ctx.synchronize()
  out["device_s"] = round(time.perf_counter() - t, 3)
  out["records"] = n
  out["device_records_per_s"] = round(n / out["device_s"], 1)
  words = np.random.randint(0, 2**32, size=16, dtype=np.uint32).astype(np.int64)
  idx, tgt = ctx.records_get()
  out["sha256"] = sha(idx, tgt)
  print(json.dumps(out), flush=True)
  if not a.no_oracle:
    import threading
    import oracle as O
    done = threading.Event()

    def beat():  # the oracle is minutes of silent CPU work
      t0 = time.time()
      while not done.wait(30):
        print(f"[oracle replica running, {time.time() - t0:.0f} s]",
              file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    r = O.Rng(a.seed)
    t = time.perf_counter()
    oidx, otgt = O.hobe_sample(r, inc, ax, ay, 200, 5)
    out["oracle_s"] = round(time.perf_counter() - t, 3)
    out["oracle_records_per_s"] = round(oidx.shape[0] / out["oracle_s"], 1)
    out["records_equal"] = bool(oidx.shape == idx.shape and np.array_equal(idx, oidx))
    out["max_abs_prob_diff"] = float(np.abs(tgt - otgt).max()) if tgt.size else 0.0
    out["numpy_state_equal"] = bool(np.array_equal(
        words, np.array([r.next32() for _ in range(16)], np.int64)))
    done.set()
    print(json.dumps(out), flush=True)
  ctx.close()


if __name__ == "__main__":
  main()
