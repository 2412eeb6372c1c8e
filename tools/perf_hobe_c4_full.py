"""One full HOBE (HG2V_ALG_DIST) epoch on the power-law 10M/5M graph
(BASELINE configs[3], single GPU): alg-dist k=10 x 20 iterations, then
AlgebraicDistanceSamples over EVERY node and edge row (quota S = 200) in
strided row chunks, each chunk trained after it is sampled
(Hg2vModel.fit_streaming, the path EmbedHg2vAlgDist takes above
RECORDS_BUDGET). --overlap-cus C: chunk c + 1 sampled on a second context
(its stream on C CUs) while chunk c trains on the other CUs (fit_streaming
`side`). Prints one JSON progress line per chunk and a summary line.

  python tools/perf_hobe_c4_full.py [--dim 256] [--epochs 1] [--budget 2**30]
                                    [--overlap-cus 0]
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
  p.add_argument("--dim", type=int, default=256)
  p.add_argument("--epochs", type=int, default=1)
  p.add_argument("--budget", type=int, default=1 << 30)
  p.add_argument("--N", type=int, default=10_000_000)
  p.add_argument("--E", type=int, default=5_000_000)
  p.add_argument("--overlap-cus", type=int, default=0)
  p.add_argument("--tables-out", default="")
  a = p.parse_args()
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.embedding import _row_chunks
  from hypergraphembedding_amd.hg2v_model import Hg2vModel
  from hypergraphembedding_amd.hg2v_sample import row_class_quota
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  S, K = 200, 5
  out = {"workload": "C4 HOBE full epoch, power-law %dx%d, d=%d" %
         (a.N, a.E, a.dim)}
  t0 = time.perf_counter()
  g = powerlaw_hypergraph(N=a.N, E=a.E, seed=0)
  out.update(nodes=g.N, edges=g.E, nnz=g.nnz, gen_s=round(time.perf_counter() - t0, 1))
  ctx = _hgx.Context(0)
  sctx = ctx  # the sampling context
  if a.overlap_cus:
    sctx = _hgx.Context(0)
    sctx.set_tuning("stream_cus", a.overlap_cus)
    ctx.set_tuning("stream_cus", -a.overlap_cus)
  out["overlap_cus"] = a.overlap_cus
  ctx.synchronize()
  t1 = time.perf_counter()
  sctx.upload(g)
  rs = np.random.RandomState(1)
  sctx.alg_set(rs.random_sample((g.N, 10)), rs.random_sample((g.E, 10)))
  sctx.alg_run(20)
  sctx.synchronize()
  out["upload_alg_s"] = round(time.perf_counter() - t1, 2)
  out["alg_ms_per_iter"] = round(sctx.alg_stats()[0] / 20, 3)
  chunks = _row_chunks(g, 2 * S, a.budget)
  out["chunks"] = len(chunks)
  print(json.dumps({"phase": "alg-dist done", **out}), flush=True)

  model = Hg2vModel(g.N + 1, g.E + 1, a.dim, K, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                    ctx=ctx, seed=11)
  st = {"sample_s": 0.0, "train_s": 0.0, "records": 0, "batches": 0,
        "batch_ms": 0.0}
  last = [None]

  def account_train():
    # the previous chunk's training ends where the next chunk (or the epoch) starts
    if last[0] is None:
      return
    ctx.synchronize()
    st["train_s"] += time.perf_counter() - last[0]
    ms, rec, bat = ctx.train_stats()
    st["batch_ms"] += ms
    st["batches"] += bat
    last[0] = None

  def chunk(c):
    if not a.overlap_cus:
      account_train()
    nq = row_class_quota(np.full(g.N, S, np.int32), *chunks[c])
    eq = row_class_quota(np.full(g.E, S, np.int32), *chunks[c])
    t = time.perf_counter()
    m = sctx.sample_hobe(4000 + c, K, S, node_q=nq, edge_q=eq)
    sctx.synchronize()
    ds = time.perf_counter() - t
    st["sample_s"] += ds
    st["records"] += m
    print(json.dumps({"chunk": c, "records": m, "sample_s": round(ds, 2),
                      "records_so_far": st["records"],
                      "elapsed_s": round(time.perf_counter() - t0, 1)}),
          flush=True)
    if not a.overlap_cus:
      last[0] = time.perf_counter()
    return m

  class Side:
    pass
  side = None
  if a.overlap_cus:
    side = Side()
    side.ctx, side.sample = sctx, chunk

  t2 = time.perf_counter()
  losses = model.fit_streaming(chunk, len(chunks), epochs=a.epochs,
                               min_delta=-1e30, seed=3, side=side)
  account_train()
  wall = time.perf_counter() - t2
  if a.overlap_cus:  # training ran beside the sampling: its own clock
    st["train_s"] = wall
    st["batch_ms"] = sum(x[2] for x in model.chunk_stats)
    st["batches"] = sum(x[4] for x in model.chunk_stats)
    out["per_chunk_batch_us"] = [round(x[2] * 1e3 / max(x[4], 1), 2)
                                 for x in model.chunk_stats]
  n = st["records"]
  out.update(
      epochs=len(losses), losses=[round(float(x), 6) for x in losses],
      records=n, records_per_epoch=model.records_per_epoch,
      sample_s=round(st["sample_s"], 2), train_s=round(st["train_s"], 2),
      sample_records_per_s=round(n / st["sample_s"], 1),
      train_records_per_s=round(n / st["train_s"], 1),
      per_batch_us=round(st["batch_ms"] * 1e3 / max(st["batches"], 1), 2),
      epoch_wall_s=round(wall, 2),
      end_to_end_records_per_s=round(
          n / (wall + out["upload_alg_s"]), 1))
  print(json.dumps(out), flush=True)
  if a.tables_out:
    nt, et = model.get_weights()
    import hashlib
    h = hashlib.sha256()
    h.update(nt.tobytes())
    h.update(et.tobytes())
    print(json.dumps({"tables_sha256": h.hexdigest()}), flush=True)
  ctx.close()


if __name__ == "__main__":
  main()
