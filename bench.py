#!/usr/bin/env python3
"""Benchmark: HOBE (HG2V_ALG_DIST) dim=128 on the synthetic random 100k/50k
hypergraph (BASELINE.json configs[2]).

One step = one training epoch (forward + backward + Keras Adagrad over every
HOBE record, batch 256, fresh device shuffle) with the records, tables and
incidence already resident in HBM. Reported beside it, from the same run:
the algebraic-distance relaxation (k=10, 20 iterations) in algorithmic GB/s,
HOBE sampling time, the roofline object of the dominant kernel (the per-batch
train_fwd_bwd + train_update pair), the CPU baseline (the oracle's
single-threaded trainer, oracle/hgref.c, on a bounded slice of the same
records) and, in "algdist_c4", the relaxation on the power-law 10M/5M graph
(the C4 shape; node-row sharded over RCCL when --gpus > 1).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: alg-dist is node-row sharded with RCCL all-reduces
(algebraic_distance.alg_dist_sharded); training runs as independent replicas
(synchronous batch-256 Adagrad does not partition), so `value`
is weak-scaled: total records trained by all ranks / max wall time.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = ("training samples/sec + alg-dist SpMV GB/s, HOBE dim=128 at "
          "1/2/4/8 MI355X")


def gather_roofline(nnz, n_rows, e_rows, ms_per_iter, ks=12):
  """Alg-dist against the chip's random-row gather rate (the bound of a
  gather-dominated SpMM whose rows have no locality): each
  incidence gathers one 4*ks-byte source row per half, edge rows in the node
  half and node rows in the edge half. Peak per half = the measured random
  48-B row rate for a table of that size (profiles/r01_gather_tablesize.json,
  log-interpolated), so the bound is nnz/peak(E table) + nnz/peak(N table)."""
  path = os.path.join(ROOT, "profiles", "r01_gather_tablesize.json")
  if not os.path.exists(path):
    return None
  with open(path) as f:
    curve = json.load(f)["curve"]
  mb = np.log([c["table_mb"] for c in curve])
  rate = [c["g_rows_per_s"] for c in curve]

  def peak(rows):
    x = np.log(max(rows * 4.0 * ks / 2**20, 1e-3))
    return float(np.interp(x, mb, rate)) * 1e9

  t_min = nnz / peak(e_rows) + nnz / peak(n_rows)
  achieved = 2.0 * nnz / (ms_per_iter * 1e-3)
  return {"bound": "random-row gather rate", "unit": "G rows/s",
          "achieved": round(achieved / 1e9, 1),
          "peak": round(2.0 * nnz / t_min / 1e9, 1),
          "frac": round(t_min / (ms_per_iter * 1e-3), 3),
          "source": "profiles/r01_gather_tablesize.json"}


def parse():
  p = argparse.ArgumentParser()
  p.add_argument("--gpus", type=int, default=1)
  p.add_argument("--steps", type=int, default=3)
  p.add_argument("--warmup", type=int, default=1)
  p.add_argument("--dim", type=int, default=128)
  p.add_argument("--num-samples", type=int, default=200)
  p.add_argument("--num-neighbors", type=int, default=5)
  p.add_argument("--batch", type=int, default=256)
  p.add_argument("--alg-iters", type=int, default=20)
  p.add_argument("--cpu-records", type=int, default=4_000_000,
                 help="records of the bounded CPU-baseline slice")
  p.add_argument("--no-cpu", action="store_true")
  p.add_argument("--no-c4", action="store_true",
                 help="skip the power-law 10M/5M alg-dist measurement")
  p.add_argument("--dist-backend", default="nccl",
                 help="torch.distributed backend for --gpus > 1 (nccl = RCCL; "
                      "gloo only to rehearse several ranks on one GPU)")
  p.add_argument("--one-device", action="store_true",
                 help="every rank uses GPU 0 (rehearsal on a 1-GPU box)")
  return p.parse_args()


def main():
  args = parse()
  world = int(os.environ.get("WORLD_SIZE", "1"))
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  dist = None
  if args.one_device:
    local = 0
  if world > 1:
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.dist_backend == "nccl":
      dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
      dist.init_process_group(args.dist_backend)

  def barrier():
    if dist is not None:
      dist.barrier()

  def sync():
    # all device work of this process runs on the context's stream
    if dist is not None:
      import torch
      torch.cuda.synchronize()
    if ctx is not None:
      ctx.synchronize()

  ctx = None

  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import random_hypergraph
  from hypergraphembedding_amd.algebraic_distance import alg_dist_sharded

  t = time.time()
  inc = random_hypergraph(seed=0)
  gen_s = time.time() - t
  ctx = _hgx.Context(local)
  ctx.upload(inc)
  k = 10
  rs = np.random.RandomState(0)
  x0 = rs.random_sample((inc.N, k))
  y0 = rs.random_sample((inc.E, k))
  bytes_iter = 8.0 * inc.nnz + (8.0 + 12.0 * k) * (inc.N + inc.E)

  # ---- algebraic distance (SpMV relaxation) ----
  if world > 1:
    alg_dist_sharded(ctx, inc, x0, y0, args.alg_iters)  # warm
    runs = [alg_dist_sharded(ctx, inc, x0, y0, args.alg_iters)[2]
            for _ in range(3)]
    alg_ms = float(np.median(runs))
    import torch
    tt = torch.tensor([alg_ms], device="cuda")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    alg_ms = float(tt.item())
  else:
    ctx.alg_set(x0, y0)
    ctx.alg_run(args.alg_iters)  # warm
    runs = []
    for _ in range(3):
      ctx.alg_set(x0, y0)
      ctx.alg_run(args.alg_iters)
      runs.append(ctx.alg_stats()[0])
    alg_ms = float(np.median(runs))
  alg_gbps = bytes_iter * args.alg_iters / (alg_ms * 1e-3) / 1e9

  # ---- HOBE records (alg coords resident on the device) ----
  ctx.upload(inc)
  ctx.alg_set(x0, y0)
  ctx.alg_run(args.alg_iters)
  t = time.time()
  n = ctx.sample_hobe(1000 + rank, args.num_neighbors, args.num_samples)
  sample_s = time.time() - t

  # ---- training ----
  ctx.model_init(args.dim, inc.N + 1, inc.E + 1, seed=7 + rank)
  for w in range(args.warmup):
    ctx.train(batch=args.batch, max_epochs=1, loss=_hgx.LOSS_MSE,
              act=_hgx.ACT_RELU, min_delta=-1e30, shuffle_seed=100 + w)
  barrier()
  sync()
  t0 = time.perf_counter()
  dev_ms = 0.0
  batches = fused_b = split_b = 0
  for s in range(args.steps):
    ctx.train(batch=args.batch, max_epochs=1, loss=_hgx.LOSS_MSE,
              act=_hgx.ACT_RELU, min_delta=-1e30, shuffle_seed=200 + s)
    ms, rec, bat = ctx.train_stats()
    fz, sp = ctx.train_path_stats()
    dev_ms += ms
    batches += bat
    fused_b += fz
    split_b += sp
  barrier()
  sync()
  elapsed = time.perf_counter() - t0
  if dist is not None:
    import torch
    tt = torch.tensor([elapsed], device="cuda")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())
  records = n * args.steps * world
  value = records / elapsed

  # ---- roofline of the dominant kernel: one batch step (train_fused, or
  # K1 + K2 for the batches that do not pack) ----
  b_rec = 224.0 * args.dim + 68.0  # SURVEY §8d algorithmic bytes / record
  per_batch_ms = dev_ms / max(batches, 1)
  batch_bytes = b_rec * (n * args.steps / max(batches, 1))
  achieved = batch_bytes / (per_batch_ms * 1e-3) / 1e9
  traffic = None
  pmc = os.path.join(ROOT, "profiles", "r01_pmc_train.json")
  if os.path.exists(pmc):
    with open(pmc) as f:
      traffic = json.load(f).get("hbm_bytes_per_batch")
  roofline = {"bound": "hbm", "achieved": round(achieved, 1),
              "peak": HBM_PEAK_GBPS, "unit": "GB/s",
              "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
              "kernel": ("train_fused (one launch per batch step)" if fused_b
                         else "train_fwd_bwd+train_update (one batch step)"),
              "batch_steps": {"train_fused": fused_b,
                              "train_fwd_bwd+train_update": split_b},
              "per_launch_us": round(per_batch_ms * 1e3, 2),
              "algorithmic_bytes_per_launch": round(batch_bytes)}

  # ---- CPU baseline: the trainer port on a bounded slice (rank 0, N=1) ----
  # oracle/cpu_train_mt.c (Keras semantics, records of a batch over OpenMP
  # threads, unique rows updated in parallel) on the box's CPU share, plus
  # the single-threaded restatement oracle/hgref.c for reference.
  cpu = None
  if rank == 0 and world == 1 and not args.no_cpu:
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    idx, tgt = ctx.records_get()
    m = min(args.cpu_records, idx.shape[0])
    sel = np.random.RandomState(0).permutation(idx.shape[0])[:m]
    cidx, ctgt = np.ascontiguousarray(idx[sel]), np.ascontiguousarray(tgt[sel])
    del idx, tgt
    init = np.random.RandomState(1)
    nt = init.uniform(-0.05, 0.05, (inc.N + 1, args.dim)).astype(np.float32)
    et = init.uniform(-0.05, 0.05, (inc.E + 1, args.dim)).astype(np.float32)
    t = time.perf_counter()
    O.train_mt(cidx, ctgt, args.num_neighbors, nt, et, O.LOSS_MSE, O.ACT_RELU,
               batch=args.batch, epochs=1, threads=threads)
    cpu_s = time.perf_counter() - t
    m1 = min(m, 500_000)
    t = time.perf_counter()
    O.train(cidx[:m1], ctgt[:m1], args.num_neighbors, nt, et, O.LOSS_MSE,
            O.ACT_RELU, batch=args.batch, max_epochs=1, min_delta=-1e30)
    cpu1_s = time.perf_counter() - t
    cpu = {"value": round(m / cpu_s, 1), "unit": "records/s", "cores": threads,
           "kind": "port",
           "sample": f"{m} HOBE records (random slice of this run's stream), "
                     f"1 epoch, d={args.dim}, batch {args.batch}, "
                     f"oracle/cpu_train_mt.c on {threads} OpenMP threads, "
                     f"{cpu_s:.1f} s",
           "single_thread_value": round(m1 / cpu1_s, 1),
           "single_thread_sample": f"first {m1} of those records, "
                                   f"oracle/hgref.c hgref_train, {cpu1_s:.1f} s"}

  # ---- alg-dist on the power-law 10M/5M graph (C4 shape, k=10) ----
  c4 = None
  if not args.no_c4:
    from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
    t = time.time()
    big = powerlaw_hypergraph(seed=0)
    c4_gen = time.time() - t
    ctx.upload(big)
    rs4 = np.random.RandomState(1)
    bx0 = rs4.random_sample((big.N, k)).astype(np.float32)
    by0 = rs4.random_sample((big.E, k)).astype(np.float32)
    b_iter4 = 8.0 * big.nnz + (8.0 + 12.0 * k) * (big.N + big.E)
    if world > 1:
      alg_dist_sharded(ctx, big, bx0, by0, 2)  # warm
      ms4 = alg_dist_sharded(ctx, big, bx0, by0, args.alg_iters)[2]
      import torch
      tt = torch.tensor([ms4], device="cuda")
      dist.all_reduce(tt, op=dist.ReduceOp.MAX)
      ms4 = float(tt.item())
    else:
      ctx.alg_set(bx0, by0)
      ctx.alg_run(2)  # warm
      ctx.alg_set(bx0, by0)
      ctx.alg_run(args.alg_iters)
      ms4 = ctx.alg_stats()[0]
    gbps4 = b_iter4 * args.alg_iters / (ms4 * 1e-3) / 1e9
    c4 = {"graph": "power-law 10M nodes / 5M edges, node degree 1+Poisson(19), "
                   "edge choice ~ rank^-0.8, seed 0 (libhgx host generator)",
          "nodes": big.N, "edges": big.E, "nnz": big.nnz,
          "max_edge": int(big.edge_size().max()), "k": k,
          "iters": args.alg_iters,
          "ms_per_iter": round(ms4 / args.alg_iters, 3),
          "gbps": round(gbps4, 1), "bytes_per_iter": b_iter4,
          "frac_of_hbm_peak": round(gbps4 / HBM_PEAK_GBPS, 4),
          "sharded": world > 1, "graph_gen_s": round(c4_gen, 1),
          "gather_roofline": (gather_roofline(big.nnz, big.N, big.E,
                                              ms4 / args.alg_iters)
                              if world == 1 else None)}
    # 128-B line traffic of the same kernels from the committed PMC run
    # (TCC_MISS x 128 B; random gathers move whole lines, tools/
    # gather_granularity.hip), against this run's time
    prof = os.path.join(ROOT, "profiles", "r01_pmc_algdist_c4.json")
    if os.path.exists(prof) and world == 1:
      with open(prof) as f:
        kern = json.load(f)["kernels"]
      lines = sum(v.get("TCC_MISS_sum", 0.0) for v in kern.values()) * 128.0
      c4["l2_miss_line_bytes_per_iter"] = lines
      c4["line_gbps"] = round(lines / (ms4 / args.alg_iters * 1e-3) / 1e9, 1)
    # ---- FOBE on the same graph (C4 shape), d=256, one GPU ----
    # Quota S on a seeded 2% of node rows and edge rows (others 0: the
    # reference's per-row quota int(weight * S) with weights 1 / 0). Every
    # 2-hop row of a node in a power-law edge is union-sampled.
    rsq = np.random.RandomState(2)
    S4, K4, d4 = args.num_samples, args.num_neighbors, 256
    nq4 = np.where(rsq.random_sample(big.N) < 0.02, S4, 0).astype(np.int32)
    eq4 = np.where(rsq.random_sample(big.E) < 0.02, S4, 0).astype(np.int32)
    sync()
    t = time.perf_counter()
    n4 = ctx.sample_fobe(4000 + rank, K4, nq4, eq4)
    sync()
    fobe_sample_s = time.perf_counter() - t
    union_rows, _ = ctx.sample_stats()
    ctx.model_init(d4, big.N + 1, big.E + 1, seed=11 + rank)
    ctx.train(batch=args.batch, max_epochs=1, loss=_hgx.LOSS_KLD,
              act=_hgx.ACT_SIGMOID, min_delta=-1e30, shuffle_seed=1)  # warm
    sync()
    t = time.perf_counter()
    ctx.train(batch=args.batch, max_epochs=1, loss=_hgx.LOSS_KLD,
              act=_hgx.ACT_SIGMOID, min_delta=-1e30, shuffle_seed=2)
    sync()
    t4 = time.perf_counter() - t
    ms4t, rec4, bat4 = ctx.train_stats()
    fobe4 = {"records": n4, "rows_sampled": int((nq4 > 0).sum() + (eq4 > 0).sum()),
             "union_sampled_rows": union_rows,
             "sampling_s": round(fobe_sample_s, 3), "dim": d4,
             "train_records_per_s": round(n4 / t4, 1),
             "per_batch_us": round(ms4t * 1e3 / max(bat4, 1), 2),
             "loss": "KLD", "act": "sigmoid"}
    if rank == 0 and world == 1 and not args.no_cpu:
      # CPU port on a 100k-record slice of the same stream (ids compacted to
      # the rows it touches, which only helps the CPU's caches)
      sys.path.insert(0, os.path.join(ROOT, "oracle"))
      import oracle as O
      idx4, tgt4 = ctx.records_get()
      sel = np.random.RandomState(3).permutation(n4)[:1_000_000]
      ci, ct = idx4[sel].copy(), tgt4[sel].copy()
      del idx4, tgt4
      R4 = 4 + 2 * K4
      node_cols = [0, 2] + list(range(4, 4 + K4))
      edge_cols = [1, 3] + list(range(4 + K4, R4))
      for cols in (node_cols, edge_cols):
        u, inv = np.unique(ci[:, cols], return_inverse=True)
        ci[:, cols] = inv.reshape(ci[:, cols].shape).astype(np.int32) + (u[0] != 0)
      init = np.random.RandomState(4)
      nt4 = init.uniform(-0.05, 0.05, (int(ci[:, node_cols].max()) + 2, d4)).astype(np.float32)
      et4 = init.uniform(-0.05, 0.05, (int(ci[:, edge_cols].max()) + 2, d4)).astype(np.float32)
      threads = max(1, min(16, len(os.sched_getaffinity(0))))
      t = time.perf_counter()
      O.train_mt(ci, ct, K4, nt4, et4, O.LOSS_KLD, O.ACT_SIGMOID,
                 batch=args.batch, epochs=1, threads=threads)
      cpu4_s = time.perf_counter() - t
      fobe4["cpu_port_records_per_s"] = round(ci.shape[0] / cpu4_s, 1)
      fobe4["cpu_port_cores"] = threads
      fobe4["cpu_port_sample"] = (f"{ci.shape[0]} records of this stream, d={d4}, "
                                  f"1 epoch, oracle/cpu_train_mt.c on {threads} "
                                  f"OpenMP threads, {cpu4_s:.1f} s")
      fobe4["vs_cpu_port"] = round(fobe4["train_records_per_s"] /
                                   fobe4["cpu_port_records_per_s"], 1)
    c4["fobe_d256"] = fobe4
    del big, bx0, by0

  if rank == 0:
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: random hypergraph 100k nodes / 50k edges, node "
                "degree 1+Poisson(19), seed 0; HOBE records sampled on device",
        "config": {
            "workload": "C3 HG2V_ALG_DIST (HOBE) dim=128, random 100k/50k, "
                        "1 step = 1 training epoch",
            "nodes": inc.N, "edges": inc.E, "nnz": inc.nnz,
            "records_per_epoch": n, "batch": args.batch, "dim": args.dim,
            "num_neighbors": args.num_neighbors,
            "num_samples": args.num_samples,
            "parallelism": (f"replicas (training), node-row sharded + "
                            f"{'RCCL' if args.dist_backend == 'nccl' else args.dist_backend}"
                            f" all-reduce (alg-dist)" if world > 1 else
                            "single GPU"),
        },
        "algdist": {"k": k, "iters": args.alg_iters,
                    "ms_per_iter": round(alg_ms / args.alg_iters, 4),
                    "gbps": round(alg_gbps, 1),
                    "bytes_per_iter": bytes_iter,
                    "frac_of_hbm_peak": round(alg_gbps / HBM_PEAK_GBPS, 4),
                    "gather_roofline": (gather_roofline(
                        inc.nnz, inc.N, inc.E, alg_ms / args.alg_iters)
                                        if world == 1 else None),
                    "sharded": world > 1},
        "algdist_c4": c4,
        "hobe_sampling_s": round(sample_s, 3),
        # EmbedHg2vAlgDist's default job (alg-dist 20 iterations, HOBE
        # sampling, 10 epochs) from the measured parts
        "end_to_end_records_per_s": round(
            n * 10 / (alg_ms * 1e-3 + sample_s + 10 * elapsed / args.steps), 1),
        "graph_gen_s": round(gen_s, 2),
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
  if dist is not None:
    dist.destroy_process_group()


if __name__ == "__main__":
  main()
