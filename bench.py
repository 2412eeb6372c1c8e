#!/usr/bin/env python3
"""Benchmark: HOBE (HG2V_ALG_DIST) dim=128 on the synthetic random 100k/50k
hypergraph (BASELINE.json configs[2]).

One step = one training epoch (forward + backward + Keras Adagrad over every
HOBE record, batch 256, fresh device shuffle) with the records, tables and
incidence already resident in HBM. Reported beside it, from the same run:
  * "roofline": the dominant kernel (the fused one-launch batch step) in
    algorithmic GB/s against the 8 TB/s HBM peak, HBM traffic per launch
    from the committed PMC run of this bench;
  * "cpu_baseline": the Keras-semantics trainer restated in C with OpenMP
    (oracle/cpu_train_mt.c) on a bounded slice of the same records;
  * "algdist": the relaxation (k=10, 20 iterations) in algorithmic GB/s;
  * "c2_fobe_d128": FOBE (HG2V_BOOLEAN) d=128 on the same graph
    (configs[1]): sampling and one training epoch; `mt19937_sampling`:
    the same stream drawn from numpy's MT19937 (rng="mt19937", the
    reference's records bit for bit) and, at N = 1, the oracle's C replica;
  * "c3_hobe_mt19937": C3's HOBE stream from numpy's MT19937 (60M records)
    timed, its sha256 checked against the stream the oracle's C replica
    reproduced record for record (profiles/r06/mt_c3/);
  * "end_to_end": one real EmbedHg2vAlgDist(graph, 128) call, timed from the
    compressed incidence to the HypergraphEmbedding message (alg-dist,
    sampling, fit with EarlyStopping, proto);
  * "algdist_c4": the relaxation on the power-law 10M/5M graph (the C4
    shape; node-row sharded over RCCL when --gpus > 1) and, in
    "algdist_c4.hobe_d256", HOBE d=256 on that graph: the north star's
    "10M-node/5M-edge at 1 GPU" workload, sampled on a seeded 2% row slice,
    one training epoch, the CPU port on a slice of the same stream with
    tables of the same size.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: alg-dist is node-row sharded with RCCL all-reduces
(algebraic_distance.alg_dist_sharded); training runs as independent replicas
(synchronous batch-256 Adagrad does not partition), so `value`
is weak-scaled: total records trained by all ranks / max wall time. Beside
it, `distinct_records_per_s` (the records of ONE embedding per second) and
`c4_time_to_embedding_s` (the C4 slice's alg-dist + sampling + epoch) do not
count replicas.

Rank launch. Under torch.distributed.run (WORLD_SIZE in the environment)
this process is one rank. A plain `python bench.py --gpus N` with N > 1 and
no WORLD_SIZE is the launcher: before any GPU call it starts N children of
this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT set, one GPU each), forwards rank 0's JSON line, and exits
non-zero if any child fails or `--launch-timeout` passes (the others are
then killed). A `--gpus` that disagrees with WORLD_SIZE is refused. The
line carries `ranks_seen` (dist.get_world_size()) and `devices_seen`
(torch.cuda.device_count()).

`c4_full` (in the default run at N = 1, ~4.5 min of its ~7.5, started only
if it still fits `--time-budget`, 600 s; `--no-c4-full` skips it,
`--c4-full` forces it, also at N > 1): the WHOLE C4 pipeline --
alg-dist (k=10, 20 iterations; sharded at N > 1), HOBE sampling of every row
into the record store, one global-shuffle d=256 epoch from the store
(embedding.py:389-416's path) -- timed as `c4_full_time_to_embedding_s`.
At N > 1 its epoch is a replica on every rank, so it is skipped by default
there (the ranks would all train the same 223 s epoch).
"""

import argparse
import json
import os
import sys
import time

# CPU-baseline legs: OpenMP threads pinned to cores (set before any OpenMP
# runtime loads), so the box-to-box spread of the CPU numbers is the CPUs'
os.environ.setdefault("OMP_PROC_BIND", "close")
os.environ.setdefault("OMP_PLACES", "cores")

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

T_START = time.time()
# wall time of the whole-C4 leg with its graph build and store release (one
# MI355X: 270 s measured, profiles/r06/bench_default_c4full/) plus margin
C4_FULL_EST_S = 330.0
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFLOPS = 157.3  # f32-in MFMA = the FP32 vector peak (same guide)
METRIC = ("training samples/sec + alg-dist SpMV GB/s, HOBE dim=128 at "
          "1/2/4/8 MI355X")
PMC_TRAIN = os.path.join(ROOT, "profiles", "r06", "pmc_train.json")
# FETCH/WRITE passes of the C4 d = 256 step (tools/train_d256_pmc_prog.py)
PMC_TRAIN_D256 = os.path.join(ROOT, "profiles", "r05", "pmc_train_d256.json")


def parse():
  p = argparse.ArgumentParser()
  p.add_argument("--gpus", type=int, default=None,
                 help="ranks (default: WORLD_SIZE, else 1); > 1 without "
                      "WORLD_SIZE starts that many child ranks")
  p.add_argument("--launch-timeout", type=float, default=3000.0,
                 help="launcher: seconds before unfinished ranks are killed")
  p.add_argument("--launch-selftest", choices=("ok", "fail", "hang"), default=None,
                 help=argparse.SUPPRESS)  # launcher test: trivial children
  p.add_argument("--edge-ranges", type=int, default=4,
                 help="C4 sharded alg-dist: edge ranges the exchange is "
                      "pipelined over (1 = one all-reduce per iteration)")
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
  p.add_argument("--no-c5", action="store_true",
                 help="skip the C5 combiner leg (inside the C4 leg)")
  p.add_argument("--c5-positives", type=int, default=1_000_000)
  p.add_argument("--c5-cpu-samples", type=int, default=100_000,
                 help="samples of the C5 combiner's CPU-baseline slice")
  p.add_argument("--no-c4", action="store_true",
                 help="skip the power-law 10M/5M measurements")
  p.add_argument("--c4-full", action="store_true",
                 help="run the whole C4 HOBE d=256 pipeline (every row "
                      "sampled into the record store, one epoch; ~4.5 min) "
                      "even at N > 1 or with --no-c4")
  p.add_argument("--no-c4-full", action="store_true",
                 help="skip the whole-C4 pipeline (default at N = 1)")
  p.add_argument("--time-budget", type=float, default=600.0,
                 help="seconds the whole run should stay within: the default "
                      "whole-C4 leg (~300 s) starts only if it fits")
  p.add_argument("--no-extra", action="store_true",
                 help="skip the C2 FOBE and end-to-end measurements")
  p.add_argument("--c4-chunks", type=int, default=2,
                 help="--gpus > 1: row-range chunks of the C4 HOBE stream")
  p.add_argument("--c4-cpu-records", type=int, default=10_000_000,
                 help="records of the C4 CPU trainer-port slice")
  p.add_argument("--c4-frac", type=float, default=0.02,
                 help="fraction of C4 rows sampled for the HOBE d=256 line")
  p.add_argument("--dist-backend", default="nccl",
                 help="torch.distributed backend for --gpus > 1 (nccl = RCCL; "
                      "gloo only to rehearse several ranks on one GPU)")
  p.add_argument("--one-device", action="store_true",
                 help="every rank uses GPU 0 (rehearsal on a 1-GPU box)")
  return p.parse_args()


# the process's CPU share, read before any OpenMP runtime binds this thread:
# with OMP_PROC_BIND the runtime pins the calling (main) thread to its first
# place, which would shrink sched_getaffinity for everything after
_AFFINITY = frozenset(os.sched_getaffinity(0))


def cpu_threads():
  """Threads of the CPU legs: every core of the process's affinity, capped by
  OMP_NUM_THREADS where the environment sets one (the GPU pool sets it to
  its per-GPU CPU share, 16: the host's other cores belong to the other
  GPUs' jobs). The affinity size is reported beside it (affinity_cores)."""
  cap = os.environ.get("OMP_NUM_THREADS", "")
  n = len(_AFFINITY)
  if cap.isdigit() and int(cap) > 0:
    n = min(n, int(cap))
  return max(1, n)


def cpu_share_note(threads):
  cap = os.environ.get("OMP_NUM_THREADS")
  return {"cores_used": threads, "affinity_cores": len(_AFFINITY),
          "omp_num_threads_env": cap,
          "policy": "all affinity cores, capped by OMP_NUM_THREADS (the "
                    "pool's per-GPU CPU share) when set"}


def restore_affinity():
  """Give the main thread its whole CPU share back after an OpenMP leg."""
  try:
    os.sched_setaffinity(0, _AFFINITY)
  except OSError:
    pass


def cpu_model():
  try:
    with open("/proc/cpuinfo") as f:
      for line in f:
        if line.startswith("model name"):
          return line.split(":", 1)[1].strip()
  except OSError:
    pass
  return "unknown"


_T0 = time.time()


def progress(msg):
  """A progress line on stderr (long legs: the GPU pool takes a command that
  prints nothing for minutes for a hung one)."""
  if os.environ.get("RANK", "0") == "0":
    print(f"[bench {time.time() - _T0:7.1f} s] {msg}", file=sys.stderr,
          flush=True)


def timed_runs(fn, reps):
  """[seconds] of `reps` calls of fn()."""
  out = []
  for _ in range(reps):
    t = time.perf_counter()
    fn()
    out.append(time.perf_counter() - t)
  return out


def _free_port():
  import socket
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def _kill_group(p, sig):
  import signal
  try:
    os.killpg(p.pid, sig)
  except (ProcessLookupError, PermissionError):
    pass


def _die_with_parent():
  """In a rank child before it starts: SIGKILL it if the launcher dies
  (prctl PR_SET_PDEATHSIG), so a launcher killed outright leaves no rank
  holding a GPU."""
  import ctypes
  import signal
  try:
    ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGKILL))
  except OSError:
    pass


def launch_ranks(n, timeout):
  """Start n ranks of this script as child processes and wait for them.

  The launcher itself never initialises a GPU (it imports no torch) and never
  execs: each rank is a fresh `python bench.py ...` child with RANK /
  LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, in its own process
  group. Rank 0's stdout (the JSON line) is forwarded to ours; the other
  ranks' stdout goes to our stderr. The first child that exits non-zero, or
  the timeout, ends the run: every remaining child group is killed and the
  status is returned (124 on timeout, 1 if rank 0 printed no JSON line)."""
  import signal
  import subprocess
  import threading
  port = os.environ.get("MASTER_PORT") or str(_free_port())
  argv = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
  procs = []
  seen = {"json": 0}

  def pump(stream):
    for line in iter(stream.readline, b""):
      s = line.decode(errors="replace")
      # the JSON line to stdout; anything else rank 0's libraries print
      # there (gloo's connection notes) to stderr
      out = sys.stdout if s.lstrip().startswith("{") else sys.stderr
      if out is sys.stdout:
        seen["json"] += 1
      out.write(s)
      out.flush()
    stream.close()

  def stop_all(sig):
    for p in procs:
      if p.poll() is None:
        _kill_group(p, sig)

  def on_term(signum, frame):
    raise SystemExit(128 + signum)

  old = signal.signal(signal.SIGTERM, on_term)
  pump_t = None
  rc = 0
  try:
    for r in range(n):
      env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                 LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", ROLE_RANK=str(r),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
      p = subprocess.Popen(argv, env=env, start_new_session=True,
                           preexec_fn=_die_with_parent,
                           stdout=subprocess.PIPE if r == 0 else sys.stderr)
      procs.append(p)
      if r == 0:
        pump_t = threading.Thread(target=pump, args=(p.stdout,), daemon=True)
        pump_t.start()
    print(f"[launcher] {n} ranks started, MASTER_PORT {port}", file=sys.stderr,
          flush=True)
    t0 = time.time()
    while True:
      codes = [p.poll() for p in procs]
      bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
      if bad:
        r, c = bad[0]
        print(f"[launcher] rank {r} exited with status {c}; stopping the "
              f"other ranks", file=sys.stderr, flush=True)
        rc = c if c > 0 else 128 - c
        break
      if all(c == 0 for c in codes):
        break
      if time.time() - t0 > timeout:
        print(f"[launcher] ranks still running after {timeout:.0f} s; "
              f"killing them", file=sys.stderr, flush=True)
        rc = 124
        break
      time.sleep(0.2)
  finally:
    stop_all(signal.SIGTERM)
    deadline = time.time() + 10
    for p in procs:
      try:
        p.wait(timeout=max(0.1, deadline - time.time()))
      except subprocess.TimeoutExpired:
        _kill_group(p, signal.SIGKILL)
        p.wait()
    if pump_t is not None:
      pump_t.join(timeout=10)
    signal.signal(signal.SIGTERM, old)
  if rc == 0 and seen["json"] == 0:
    print("[launcher] rank 0 printed no JSON line", file=sys.stderr, flush=True)
    rc = 1
  return rc


def launch_selftest(mode, world, rank):
  """--launch-selftest child: a gloo rendezvous on the CPU (no GPU), rank 0
  prints the ranks it saw; in mode 'fail' the last rank exits 3 and rank 0
  blocks as a rank waiting on a collective would; in mode 'hang' every rank
  blocks."""
  import torch
  import torch.distributed as dist
  print(f"[selftest] rank {rank} of {world}", file=sys.stderr, flush=True)
  if mode == "hang":
    time.sleep(600)
  if mode == "fail" and world > 1:
    if rank == world - 1:
      sys.exit(3)
    time.sleep(600)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  got = [None] * world
  dist.all_gather_object(got, (rank, int(os.environ["LOCAL_RANK"]),
                               int(os.environ["WORLD_SIZE"])))
  if rank == 0:
    print(json.dumps({"selftest": mode, "ranks_seen": dist.get_world_size(),
                      "ranks": got}), flush=True)
  dist.destroy_process_group()


def main():
  args = parse()
  env_world = os.environ.get("WORLD_SIZE")
  if env_world is None:
    want = args.gpus or 1
    if want > 1:
      # the launcher: no GPU call in this process (see launch_ranks)
      sys.exit(launch_ranks(want, args.launch_timeout))
    world = 1
  else:
    world = int(env_world)
    if args.gpus is not None and args.gpus != world:
      print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}",
            file=sys.stderr, flush=True)
      sys.exit(2)
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  if args.launch_selftest:
    launch_selftest(args.launch_selftest, world, rank)
    return
  dist = None
  if args.one_device:
    local = 0
  # library calls without an explicit context (EmbedHg2vAlgDist) use this device
  os.environ["HGX_DEVICE"] = str(local)
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

  def max_over_ranks(x):
    if dist is None:
      return x
    import torch
    tt = torch.tensor([x], device="cuda")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())

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
  progress('C3 graph built; alg-dist')
  exch = {}
  if world > 1:
    alg_dist_sharded(ctx, inc, x0, y0, args.alg_iters)  # warm
    runs = [alg_dist_sharded(ctx, inc, x0, y0, args.alg_iters, stats=exch)[2]
            for _ in range(3)]
    alg_ms = max_over_ranks(float(np.median(runs)))
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
  progress('C3 HOBE sampling')
  ctx.upload(inc)
  ctx.alg_set(x0, y0)
  ctx.alg_run(args.alg_iters)
  barrier()
  t = time.time()
  if world > 1:
    # row-sharded sampling: each rank samples its rows, then an
    # all-gather gives every training replica the whole stream
    from hypergraphembedding_amd.hg2v_sample import sample_sharded
    n, _ = sample_sharded(inc, args.num_neighbors, args.num_samples, ctx=ctx,
                          seed=1000, kind="hobe",
                          device=None if args.dist_backend == "nccl" else "cpu")
  else:
    n = ctx.sample_hobe(1000, args.num_neighbors, args.num_samples)
  sample_s = max_over_ranks(time.time() - t)

  # ---- training: the timed steps ----
  progress('C3 training (timed steps)')
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
  elapsed = max_over_ranks(time.perf_counter() - t0)
  records = n * args.steps * world
  value = records / elapsed

  # ---- roofline of the dominant kernel: one batch step (train_step; K1 + K2
  # only where the step does not apply) ----
  b_rec = 224.0 * args.dim + 68.0  # SURVEY §8d algorithmic bytes / record
  per_batch_ms = dev_ms / max(batches, 1)
  batch_bytes = b_rec * (n * args.steps / max(batches, 1))
  achieved = batch_bytes / (per_batch_ms * 1e-3) / 1e9
  traffic = pmc_src = None
  if os.path.exists(PMC_TRAIN):
    with open(PMC_TRAIN) as f:
      pm = json.load(f)
    traffic = pm.get("hbm_bytes_per_batch")
    pmc_src = os.path.relpath(PMC_TRAIN, ROOT)
  roofline = {"bound": "hbm", "achieved": round(achieved, 1),
              "peak": HBM_PEAK_GBPS, "unit": "GB/s",
              "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
              "traffic_source": pmc_src,
              "kernel": ("train_step (one launch per batch step)" if fused_b
                         else "train_fwd_bwd+train_update (one batch step)"),
              "batch_steps": {"train_step": fused_b,
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
    threads = cpu_threads()
    idx, tgt = ctx.records_get()
    m = min(args.cpu_records, idx.shape[0])
    sel = np.random.RandomState(0).permutation(idx.shape[0])[:m]
    cidx, ctgt = np.ascontiguousarray(idx[sel]), np.ascontiguousarray(tgt[sel])
    del idx, tgt
    init = np.random.RandomState(1)
    nt = init.uniform(-0.05, 0.05, (inc.N + 1, args.dim)).astype(np.float32)
    et = init.uniform(-0.05, 0.05, (inc.E + 1, args.dim)).astype(np.float32)
    # thread scaling of the trainer port on the first 500k records: how its
    # rate grows with cores; the baseline below runs at the sweep's best
    # thread count (the port stops scaling before the box's CPU share)
    ms_ = min(m, 500_000)
    scaling = {}
    for tt in sorted({1 << i for i in range(threads.bit_length())} | {threads}):
      r_ = timed_runs(lambda: O.train_mt(cidx[:ms_], ctgt[:ms_],
                                         args.num_neighbors, nt, et,
                                         O.LOSS_MSE, O.ACT_RELU,
                                         batch=args.batch, epochs=1,
                                         threads=tt), 1)
      scaling[str(tt)] = round(ms_ / r_[0], 1)
    best_t = int(max(scaling, key=lambda k: scaling[k]))
    # three runs of the whole slice (fresh tables each) at that count:
    # median and spread
    runs = timed_runs(lambda: O.train_mt(cidx, ctgt, args.num_neighbors, nt, et,
                                         O.LOSS_MSE, O.ACT_RELU,
                                         batch=args.batch, epochs=1,
                                         threads=best_t), 3)
    cpu_s = float(np.median(runs))
    restore_affinity()
    m1 = min(m, 500_000)
    t = time.perf_counter()
    O.train(cidx[:m1], ctgt[:m1], args.num_neighbors, nt, et, O.LOSS_MSE,
            O.ACT_RELU, batch=args.batch, max_epochs=1, min_delta=-1e30)
    cpu1_s = time.perf_counter() - t
    restore_affinity()
    cpu = {"value": round(m / cpu_s, 1), "unit": "records/s", "cores": best_t,
           "kind": "port", "cpu_model": cpu_model(),
           "omp": {"OMP_PROC_BIND": os.environ.get("OMP_PROC_BIND"),
                   "OMP_PLACES": os.environ.get("OMP_PLACES")},
           "sample": f"{m} HOBE records (random slice of this run's stream), "
                     f"1 epoch, d={args.dim}, batch {args.batch}, "
                     f"oracle/cpu_train_mt.c on {best_t} OpenMP threads "
                     f"(the best of the thread sweep on the {threads}-core "
                     f"share), median of 3 runs ({cpu_s:.1f} s)",
           "runs_records_per_s": [round(m / r, 1) for r in runs],
           "threads": cpu_share_note(threads),
           "thread_scaling_records_per_s": scaling,
           "single_thread_value": round(m1 / cpu1_s, 1),
           "single_thread_sample": f"first {m1} of those records, "
                                   f"oracle/hgref.c hgref_train, {cpu1_s:.1f} s"}
    # HOBE sampling on the CPU: the same algorithm (exact per-row expansion,
    # uniform distinct draws, the reference's probabilities) on a seeded 10%
    # of C3's node rows and edge rows, OpenMP over rows, on this run's
    # coordinates (oracle/cpu_sample_mt.c)
    ax, ay = ctx.alg_get()
    rsq = np.random.RandomState(5)
    nq = np.where(rsq.random_sample(inc.N) < 0.1, args.num_samples, 0).astype(np.int32)
    eq = np.where(rsq.random_sample(inc.E) < 0.1, args.num_samples, 0).astype(np.int32)
    t = time.perf_counter()
    sidx, _, _ = O.cpu_hobe_sample_mt(inc, ax, ay, nq, eq, args.num_neighbors,
                                      seed=1, threads=threads)
    cs_s = time.perf_counter() - t
    restore_affinity()
    n_cs = int(sidx.shape[0])
    del sidx
    cpu["hobe_sampling"] = {
        "value": round(n_cs / cs_s, 1), "unit": "records/s", "cores": threads,
        "kind": "port",
        "sample": f"AlgebraicDistanceSamples on a seeded 10% of C3's node and "
                  f"edge rows (S={args.num_samples}, K={args.num_neighbors}): "
                  f"{n_cs} records in {cs_s:.1f} s, oracle/cpu_sample_mt.c",
        "gpu_records_per_s": round(n / sample_s, 1) if sample_s > 0 else None}

  # ---- C2: FOBE d=128 on the same graph (BASELINE configs[1]) ----
  progress('C2 FOBE + end-to-end legs')
  c2 = e2e = c3mt = None
  if not args.no_extra:
    S, K = args.num_samples, args.num_neighbors
    q_n = np.full(inc.N, S, np.int32)  # int(weight * S), weights 1
    q_e = np.full(inc.E, S, np.int32)
    sync()
    t = time.perf_counter()
    n2 = ctx.sample_fobe(2000 + rank, K, q_n, q_e)
    sync()
    c2_sample_s = time.perf_counter() - t
    ctx.model_init(args.dim, inc.N + 1, inc.E + 1, seed=13 + rank)
    sync()
    t = time.perf_counter()
    ctx.train(batch=args.batch, max_epochs=1, loss=_hgx.LOSS_KLD,
              act=_hgx.ACT_SIGMOID, min_delta=-1e30, shuffle_seed=3)
    sync()
    c2_s = time.perf_counter() - t
    ms2, _, bat2 = ctx.train_stats()
    c2 = {"workload": "C2 HG2V_BOOLEAN (FOBE) dim=128, random 100k/50k, "
                      "1 epoch", "records": n2,
          "sampling_s": round(c2_sample_s, 3),
          "train_records_per_s": round(n2 / c2_s, 1),
          "per_batch_us": round(ms2 * 1e3 / max(bat2, 1), 2),
          "batch_steps": dict(zip(("train_step", "train_fwd_bwd+train_update"),
                                  ctx.train_path_stats()))}
    # the same stream drawn from numpy's own MT19937 stream (rng="mt19937":
    # BooleanSamples' records bit for bit, hgx_sample_fobe_mt); at N = 1 the
    # oracle's single-threaded C replica of the reference's draws beside it
    np.random.seed(2000 + rank)
    sync()
    t = time.perf_counter()
    n_mt = ctx.sample_fobe_mt(K, q_n, q_e)
    sync()
    mt_s = time.perf_counter() - t
    c2["mt19937_sampling"] = {"records": n_mt, "s": round(mt_s, 3),
                              "records_per_s": round(n_mt / mt_s, 1)}
    if rank == 0 and world == 1 and not args.no_cpu:
      sys.path.insert(0, os.path.join(ROOT, "oracle"))
      import oracle as O
      t = time.perf_counter()
      ridx, _ = O.fobe_sample(O.Rng(2000), inc, q_n, q_e, K)
      r_s = time.perf_counter() - t
      c2["mt19937_sampling"]["cpu_replica"] = {
          "s": round(r_s, 3), "records_per_s": round(ridx.shape[0] / r_s, 1),
          "cores": 1, "kind": "port",
          "sample": "the whole C2 stream, oracle/hgref.c hgref_fobe_sample "
                    "(the reference's MT19937 draws restated in C)"}
      del ridx
    # C3's HOBE stream from numpy's MT19937 (AlgebraicDistanceSamples,
    # run_in_parallel=False): tools/mt_c3_hobe.py's procedure, whose stream
    # the oracle's C replica reproduced record for record
    # (profiles/r06/mt_c3/mt_c3_hobe.json: its sha256 is the check here)
    ref = os.path.join(ROOT, "profiles", "r06", "mt_c3", "mt_c3_hobe.json")
    rs1 = np.random.RandomState(1)
    ctx.alg_set(rs1.random_sample((inc.N, 10)), rs1.random_sample((inc.E, 10)))
    ctx.alg_run(20)
    ax, ay = ctx.alg_get()
    ctx.alg_set(ax, ay)
    np.random.seed(5)
    sync()
    t = time.perf_counter()
    n_h = ctx.sample_hobe_mt(args.num_neighbors, args.num_samples)
    sync()
    h_s = time.perf_counter() - t
    import hashlib
    hidx, htgt = ctx.records_get()
    hh = hashlib.sha256()
    hh.update(np.ascontiguousarray(hidx, np.int32).tobytes())
    hh.update(np.ascontiguousarray(htgt, np.float32).tobytes())
    del hidx, htgt
    c3mt = {"records": n_h, "s": round(h_s, 3),
            "records_per_s": round(n_h / h_s, 1), "sha256": hh.hexdigest()}
    if os.path.exists(ref):
      with open(ref) as f:
        rj = [json.loads(l) for l in f if l.startswith("{")][-1]
      if args.num_neighbors == 5 and args.num_samples == 200:
        c3mt["equals_oracle_replica_stream"] = rj.get("sha256") == c3mt["sha256"] \
            and bool(rj.get("records_equal"))
        c3mt["oracle_replica_s"] = rj.get("oracle_s")

    # ---- end to end: one real EmbedHg2vAlgDist call (embedding.py:389) ----
    from hypergraphembedding_amd.embedding import EmbedHg2vAlgDist
    from hypergraphembedding_amd.runtime import get_context
    np.random.seed(rank)
    ectx = get_context(local)
    ectx.synchronize()
    t = time.perf_counter()
    emb = EmbedHg2vAlgDist(inc, args.dim)
    ectx.synchronize()
    e2e_s = time.perf_counter() - t
    _, e_rec, _ = ectx.train_stats()
    n_emb = ectx.records_info()[0]
    e2e = {"call": f"EmbedHg2vAlgDist(C3 incidence, {args.dim}) defaults: "
                   "alg-dist k=10 x 20, HOBE S=200 K=5, fit batch 256 up to "
                   "10 epochs with EarlyStopping, HypergraphEmbedding out",
           "wall_s": round(e2e_s, 3), "records_per_epoch": n_emb,
           "epochs_run": round(e_rec / max(n_emb, 1), 2),
           "records_per_s": round(e_rec / e2e_s, 1),
           "embedding_rows": len(emb.node) + len(emb.edge)}
    del emb

  # ---- power-law 10M/5M graph (C4 shape) ----
  c4 = None
  if not args.no_c4:
    progress("C4 legs (alg-dist, 2% HOBE d=256 slice, C5 combiner)")
    c4 = bench_c4(args, ctx, rank, world, sync, max_over_ranks, alg_dist_sharded)
  c4_full = None
  if args.c4_full or (world == 1 and not args.no_c4 and not args.no_c4_full):
    spent = time.time() - T_START
    if not args.c4_full and spent + C4_FULL_EST_S > args.time_budget:
      # the default leg would not fit the run's time budget on this box
      c4_full = {"skipped": f"{spent:.0f} s spent before the leg, ~{C4_FULL_EST_S:.0f} s "
                            f"needed, budget {args.time_budget:.0f} s (--c4-full forces it)"}
    else:
      progress("c4-full leg")
      c4_full = bench_c4_full(args, ctx, world, sync, max_over_ranks)

  ranks_seen = dist.get_world_size() if dist is not None else 1
  # HIP devices visible to this rank's libhgx (hipGetDeviceCount; torch's
  # own HIP runtime is not initialised at N = 1)
  devices_seen = _hgx.device_count()
  hobe4 = (c4 or {}).get("hobe_d256") or {}
  tte4 = (hobe4.get("time_to_embedding_s") or {}).get("total_s")
  if rank == 0:
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "ranks_seen": ranks_seen,
        "devices_seen": devices_seen,
        # the records of ONE embedding per second (value counts every
        # replica's identical epoch) and the C4 slice's wall time to an
        # embedding (alg-dist + sampling + one epoch, sharded at N > 1)
        "distinct_records_per_s": round(n * args.steps / elapsed, 1),
        "c4_time_to_embedding_s": tte4,
        # the whole C4 pipeline (every row sampled, one epoch; c4_full)
        "c4_full_time_to_embedding_s": (c4_full or {}).get("time_to_embedding_s"),
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
        "roofline": roofline,
        "cpu_baseline": cpu,
        "algdist": {"k": k, "iters": args.alg_iters,
                    "ms_per_iter": round(alg_ms / args.alg_iters, 4),
                    "gbps": round(alg_gbps, 1),
                    "bytes_per_iter": bytes_iter,
                    "frac_of_hbm_peak": round(alg_gbps / HBM_PEAK_GBPS, 4),
                    "note": "C3's 35 MB working set is cache-resident; the "
                            "HBM fraction is judged on algdist_c4",
                    "sharded": world > 1, "exchange": exch or None},
        "hobe_sampling_s": round(sample_s, 3),
        "sampling": ("row-sharded over ranks + record all-gather" if world > 1
                     else "single GPU"),
        "c2_fobe_d128": c2,
        "c3_hobe_mt19937": c3mt,
        "end_to_end": e2e,
        "algdist_c4": c4,
        "c4_full": c4_full,
        "graph_gen_s": round(gen_s, 2),
    }
    print(json.dumps(out), flush=True)
  if dist is not None:
    dist.destroy_process_group()


def bench_c4(args, ctx, rank, world, sync, max_over_ranks, alg_dist_sharded):
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  k = 10
  t = time.time()
  big = powerlaw_hypergraph(seed=0)
  c4_gen = time.time() - t
  ctx.upload(big)
  rs4 = np.random.RandomState(1)
  bx0 = rs4.random_sample((big.N, k)).astype(np.float32)
  by0 = rs4.random_sample((big.E, k)).astype(np.float32)
  b_iter4 = 8.0 * big.nnz + (8.0 + 12.0 * k) * (big.N + big.E)
  exch4 = {}
  if world > 1:
    # exchange pipelined over edge ranges (all-reduce of range r overlaps
    # the partials of range r + 1)
    alg_dist_sharded(ctx, big, bx0, by0, 2, edge_ranges=args.edge_ranges)
    (r0, r1, xo), y_sh, ms_sh = alg_dist_sharded(
        ctx, big, bx0, by0, args.alg_iters, stats=exch4,
        edge_ranges=args.edge_ranges)
    ms4 = max_over_ranks(ms_sh)
    # every rank needs every node's coordinates for the HOBE weights: one
    # all-gather of the node rows (embedding.hobe_sharded's step 1)
    from hypergraphembedding_amd.embedding import _all_gather_rows
    t = time.perf_counter()
    x_sh = _all_gather_rows(xo, r0, r1, big.N, None,
                            None if args.dist_backend == "nccl" else "cpu")
    exch4["coord_allgather_s"] = round(max_over_ranks(time.perf_counter() - t), 3)
    ctx.upload(big)  # HOBE below runs on the whole graph of this rank
  else:
    ctx.alg_set(bx0, by0)
    ctx.alg_run(2)  # warm
    ctx.alg_set(bx0, by0)
    ctx.alg_run(args.alg_iters)
    ms4 = ctx.alg_stats()[0]
  gbps4 = b_iter4 * args.alg_iters / (ms4 * 1e-3) / 1e9
  # the ceiling the sweep is bound by: random row gathers, not stream
  # bandwidth. Two gathers per incidence per iteration (node
  # half, edge half); the device's random 64-B-row rate at the two tables'
  # sizes, best over rows in flight, measured here on the same box.
  ach = 2.0 * big.nnz * args.alg_iters / (ms4 * 1e-3)
  probe = {}
  for tab_mb in (big.E * 64 >> 20, big.N * 64 >> 20):
    probe[f"{tab_mb}MB"] = max(ctx.probe_gather(tab_mb << 20, 16, f)
                               for f in (4, 8, 16))
  ceiling = min(probe.values())
  c4 = {"graph": "power-law 10M nodes / 5M edges, node degree 1+Poisson(19), "
                 "edge choice ~ rank^-0.8, seed 0 (libhgx host generator)",
        "nodes": big.N, "edges": big.E, "nnz": big.nnz,
        "max_edge": int(big.edge_size().max()), "k": k,
        "iters": args.alg_iters,
        "ms_per_iter": round(ms4 / args.alg_iters, 3),
        "gbps": round(gbps4, 1), "bytes_per_iter": b_iter4,
        "frac_of_hbm_peak": round(gbps4 / HBM_PEAK_GBPS, 4),
        "gather_ceiling": {
            "achieved_g_gathers_per_s": round(ach / 1e9, 2),
            "probe_g_rows_per_s": {k: round(v / 1e9, 2) for k, v in probe.items()},
            "ceiling_g_rows_per_s": round(ceiling / 1e9, 2),
            "frac_of_ceiling": round(ach / ceiling, 3),
            "note": "random 64-B row gathers (hgx_probe_gather: quads of "
                    "lanes, 4/8/16 rows in flight, best) from tables of the "
                    "edge and node coordinate sizes; above 1.0 = hot-edge "
                    "L2 hits; 60% of HBM peak would need ~550 G rows/s"},
        "sharded": world > 1, "exchange": exch4 or None,
        "graph_gen_s": round(c4_gen, 1)}
  # ---- HOBE d=256 on the same graph: the north star's 10M/5M workload ----
  # AlgebraicDistanceSamples with quota S on a seeded 2% of node rows and of
  # edge rows (0 elsewhere; the reference samples S per row everywhere, a
  # ~6e9-record epoch), on the alg coords of the run above; one epoch.
  if world > 1:
    ctx.alg_set(x_sh, y_sh)  # the sharded relaxation's coordinates
    del x_sh
  S4, K4, d4 = args.num_samples, args.num_neighbors, 256
  rsq = np.random.RandomState(2)
  nq4 = np.where(rsq.random_sample(big.N) < args.c4_frac, S4, 0).astype(np.int32)
  eq4 = np.where(rsq.random_sample(big.E) < args.c4_frac, S4, 0).astype(np.int32)
  ctx.model_init(d4, big.N + 1, big.E + 1, seed=11 + rank)
  if world > 1:
    # the form the full 5.9e9-record epoch takes over N ranks
    # (embedding.hobe_sharded): the stream sampled once into every rank's
    # record store, strided row classes sampled on the ranks' strided shares
    # with each class's 12-byte entries all-gathered while the next class
    # samples (hg2v_sample.sharded_store_fill), then one epoch of Keras'
    # global shuffle from the store in chunks (Hg2vModel.fit_store)
    from hypergraphembedding_amd.embedding import _row_chunks
    from hypergraphembedding_amd.hg2v_model import Hg2vModel
    from hypergraphembedding_amd.hg2v_sample import sharded_store_fill
    bn = 2 * nq4.astype(np.int64)
    be = 2 * eq4.astype(np.int64)
    bound = int(bn.sum() + be.sum())
    chunk = -(-bound // args.c4_chunks)
    chunks = _row_chunks(bn, be, chunk)
    sync()
    t = time.perf_counter()
    n4 = sharded_store_fill(big, K4, S4, chunks, ctx=ctx, seed=4000,
                            kind="hobe", node_quota=nq4, edge_quota=eq4,
                            device=None if args.dist_backend == "nccl" else "cpu",
                            capacity=bound)
    sync()
    hobe_sample_s = max_over_ranks(time.perf_counter() - t)
    rej_rows, fb_rows = ctx.sample_stats()  # of the last class
    model = Hg2vModel(big.N + 1, big.E + 1, d4, K4, _hgx.LOSS_MSE,
                      _hgx.ACT_RELU, ctx=ctx, seed=11)
    sync()
    t = time.perf_counter()
    model.fit_store(chunk, batch_size=args.batch, epochs=1, min_delta=-1e30,
                    seed=2)
    sync()
    t4 = time.perf_counter() - t
    cs = model.chunk_stats
    ms4t = sum(x[2] for x in cs)
    rec4 = sum(x[3] for x in cs)
    bat4 = sum(x[4] for x in cs)
    fz4, sp4 = bat4, 0  # train_path_stats of the last chunk only
    t4 = max_over_ranks(t4)
  else:
    sync()
    t = time.perf_counter()
    n4 = ctx.sample_hobe(4000, K4, S4, node_q=nq4, edge_q=eq4)
    sync()
    hobe_sample_s = time.perf_counter() - t
    rej_rows, fb_rows = ctx.sample_stats()
    sync()
    t = time.perf_counter()
    ctx.train(batch=args.batch, max_epochs=1, loss=_hgx.LOSS_MSE,
              act=_hgx.ACT_RELU, min_delta=-1e30, shuffle_seed=2)
    sync()
    t4 = time.perf_counter() - t
    ms4t, rec4, bat4 = ctx.train_stats()
    fz4, sp4 = ctx.train_path_stats()
  hobe4 = {"workload": "HG2V_ALG_DIST (HOBE) dim=256 on the 10M/5M power-law "
                       f"graph, rows sampled: a seeded {args.c4_frac:.0%} of "
                       "node rows and edge rows (quota S=200, K=5), 1 epoch",
           "records": n4,
           "chunks": (f"record store: {len(chunks)} strided row classes "
                      "sampled row-sharded, entries all-gathered per class; "
                      f"one global-shuffle epoch in chunks of <= {chunk} records"
                      if world > 1 else "one resident stream"),
           "rows_sampled": int((nq4 > 0).sum() + (eq4 > 0).sum()),
           "rejection_rows": rej_rows, "expansion_fallback_rows": fb_rows,
           "uniform_column_rows": ctx.sample_uniform_rows(),
           "sampling_s": round(hobe_sample_s, 3),
           "sampling_records_per_s": round(n4 / hobe_sample_s, 1),
           "dim": d4, "train_records_per_s": round(n4 / t4, 1),
           "per_batch_us": round(ms4t * 1e3 / max(bat4, 1), 2),
           "batch_steps": {"train_step": fz4, "train_fwd_bwd+train_update": sp4},
           "multi_pending_batches": ctx.train_multi_pending(),
           "loss": "MSE", "act": "relu"}
  # roofline of the north-star config's step (d = 256, the power-law
  # stream: train_step<64,4,5,2,256,{false,true}>, the plain and the MULTI
  # pending-slot form)
  b_rec4 = 224.0 * d4 + 68.0
  pb_us = ms4t * 1e3 / max(bat4, 1)
  ach4 = b_rec4 * (n4 / max(bat4, 1)) / (pb_us * 1e-6) / 1e9
  rf4 = {"bound": "hbm", "achieved": round(ach4, 1), "peak": HBM_PEAK_GBPS,
         "unit": "GB/s", "frac": round(ach4 / HBM_PEAK_GBPS, 4),
         "per_launch_us": round(pb_us, 2),
         "algorithmic_bytes_per_launch": round(b_rec4 * n4 / max(bat4, 1)),
         "traffic": None}
  if os.path.exists(PMC_TRAIN_D256):
    with open(PMC_TRAIN_D256) as f:
      pm4 = json.load(f)
    rf4["traffic"] = pm4.get("hbm_bytes_per_batch")
    rf4["traffic_by_form"] = pm4.get("hbm_bytes_per_batch_by_form")
    rf4["traffic_source"] = os.path.relpath(PMC_TRAIN_D256, ROOT)
    if "per_form_us" in pm4:
      rf4["per_form_us"] = pm4["per_form_us"]
  hobe4["roofline"] = rf4
  # the whole pipeline of this slice on N GPUs: relaxation (20 iterations,
  # node-row sharded at N > 1, plus the node-coordinate all-gather),
  # sampling, one epoch; records/s of ONE embedding (the replicas train the
  # same records, so this is not multiplied by N)
  tte = {"alg_dist_s": round(ms4 / 1e3, 3),
         "coord_allgather_s": exch4.get("coord_allgather_s", 0.0),
         "sampling_s": round(hobe_sample_s, 3), "train_epoch_s": round(t4, 3)}
  tte["total_s"] = round(sum(tte.values()), 3)
  hobe4["time_to_embedding_s"] = tte
  hobe4["distinct_records_per_s"] = round(n4 / t4, 1)
  if rank == 0 and world == 1 and not args.no_cpu:
    # CPU port on 1e7 records of the same stream (BASELINE.md's planned
    # slice), tables of the same size (10M+1 and 5M+1 rows x 256; only the
    # rows the slice touches are initialised, the rest stays untouched)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    idx4, tgt4 = ctx.records_get()
    m4 = min(args.c4_cpu_records, n4)
    sel = np.random.RandomState(3).permutation(n4)[:m4]
    ci, ct = idx4[sel].copy(), tgt4[sel].copy()
    del idx4, tgt4
    R4 = 4 + 2 * K4
    node_cols = [0, 2] + list(range(4, 4 + K4))
    edge_cols = [1, 3] + list(range(4 + K4, R4))
    init = np.random.RandomState(4)
    nt4 = np.empty((big.N + 1, d4), np.float32)
    et4 = np.empty((big.E + 1, d4), np.float32)
    for tab, cols in ((nt4, node_cols), (et4, edge_cols)):
      rows = np.unique(ci[:, cols])
      tab[rows] = init.uniform(-0.05, 0.05, (rows.size, d4)).astype(np.float32)
    threads = cpu_threads()
    t = time.perf_counter()
    O.train_mt(ci, ct, K4, nt4, et4, O.LOSS_MSE, O.ACT_RELU, batch=args.batch,
               epochs=1, threads=threads, copy=False)
    cpu4_s = time.perf_counter() - t
    restore_affinity()
    hobe4["cpu_port_records_per_s"] = round(m4 / cpu4_s, 1)
    hobe4["cpu_port_cores"] = threads
    hobe4["cpu_port_threads"] = cpu_share_note(threads)
    hobe4["cpu_port_sample"] = (f"{m4} random records of this stream, d={d4}, "
                                f"tables {big.N + 1} + {big.E + 1} rows, 1 epoch, "
                                f"oracle/cpu_train_mt.c on {threads} OpenMP "
                                f"threads, {cpu4_s:.1f} s")
    hobe4["vs_cpu_port"] = round(hobe4["train_records_per_s"] /
                                 hobe4["cpu_port_records_per_s"], 1)
    del nt4, et4, ci, ct
    # alg-dist on the CPU: the reference's float64 relaxation restated
    # (oracle/hgref.c hgref_algdist, OpenMP over rows), 3 iterations of the
    # whole 10M/5M graph from the same init
    t = time.perf_counter()
    O.algdist(big, bx0, by0, 3)
    ca_s = time.perf_counter() - t
    restore_affinity()
    c4["cpu_algdist"] = {
        "ms_per_iter": round(ca_s / 3 * 1e3, 1),
        "gbps": round(b_iter4 * 3 / ca_s / 1e9, 2),
        "cores": threads, "kind": "port", "dtype": "f64",
        "threads": cpu_share_note(threads),
        "sample": "3 iterations on the whole power-law 10M/5M graph, "
                  "oracle/hgref.c hgref_algdist (float64 like the reference, "
                  f"OpenMP over rows), {ca_s:.1f} s; gbps in the fp32 "
                  "algorithmic bytes of the GPU line",
        "vs_gpu": round((ca_s / 3 * 1e3) / (ms4 / args.alg_iters), 1)}
  c4["hobe_d256"] = hobe4
  if not args.no_c5:
    if rank == 0:
      c4["c5_combiner"] = bench_c5(args, ctx, big)
    sync()
  return c4


def bench_c4_full(args, ctx, world, sync, max_over_ranks):
  """--c4-full: the north star's 10M/5M HOBE d=256 embedding end to end, as
  EmbedHg2vAlgDist runs it past RECORDS_BUDGET (embedding.py:389-416):
  alg-dist k=10 x 20 iterations (node-row sharded over RCCL at N > 1),
  AlgebraicDistanceSamples on EVERY node and edge row (S=200, K=5) sampled
  once into the record store in strided row classes (row-sharded, entries
  all-gathered, at N > 1), one global-shuffle epoch of d=256 Adagrad from
  the store (Hg2vModel.fit_store). Timed per stage; the store is released
  afterwards. At N > 1 every rank trains the same epoch (replicas)."""
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.embedding import (STORE_CHUNK, fill_store,
                                                 hobe_sharded)
  from hypergraphembedding_amd.hg2v_model import Hg2vModel
  from hypergraphembedding_amd.hg2v_sample import row_class_quota
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  S, K, d = args.num_samples, args.num_neighbors, 256
  t = time.perf_counter()
  g = powerlaw_hypergraph(seed=0)
  gen_s = time.perf_counter() - t
  ctx.store_release()  # the C4 slice's records: their HBM back
  st = {}
  sync()
  t0 = time.perf_counter()
  if world > 1:
    hobe_sharded(g, d, K, S, args.batch, epochs=1, ctx=ctx, stats=st,
                 edge_ranges=args.edge_ranges)
    sync()
    total = max_over_ranks(time.perf_counter() - t0)
    stages = {"alg_dist_s": st.get("alg_s"), "sampling_s": st.get("sampling_s"),
              "train_epoch_s": st.get("train_s")}
    n = int(st.get("records", 0))
  else:
    ctx.upload(g)
    rs = np.random.RandomState(1)
    ctx.alg_set(rs.random_sample((g.N, 10)), rs.random_sample((g.E, 10)))
    ctx.alg_run(args.alg_iters)
    sync()
    t1 = time.perf_counter()
    bn = np.full(g.N, 2 * S, np.int64)
    be = np.full(g.E, 2 * S, np.int64)
    fq = (np.full(g.N, S, np.int32), np.full(g.E, S, np.int32))
    def sample(off, stride):
      m = ctx.sample_hobe(4000, K, S, *(row_class_quota(q, off, stride)
                                        for q in fq))
      progress(f"c4-full: row class {off} of {stride} sampled ({m} records)")
      return m
    try:
      n = fill_store(ctx, g, sample, bn, be, STORE_CHUNK)
      sync()
      t2 = time.perf_counter()
      model = Hg2vModel(g.N + 1, g.E + 1, d, K, _hgx.LOSS_MSE, _hgx.ACT_RELU,
                        ctx=ctx, seed=11)
      model.fit_store(STORE_CHUNK, batch_size=args.batch, epochs=1,
                      min_delta=-1e30, seed=3,
                      on_chunk=lambda ep, c, nc: progress(
                          f"c4-full: chunk {c + 1} of {nc} trained"))
      sync()
      t3 = time.perf_counter()
      free, tot = ctx.mem_info()
      cs = model.chunk_stats
    finally:
      ctx.store_release()
    total = t3 - t0
    stages = {"alg_dist_s": round(t1 - t0, 3), "sampling_s": round(t2 - t1, 3),
              "train_epoch_s": round(t3 - t2, 3)}
    st["per_batch_us"] = round(sum(x[2] for x in cs) * 1e3 /
                               max(sum(x[4] for x in cs), 1), 2)
    st["chunks"] = len(cs)
    st["device_mem_used_gb_at_epoch_end"] = round((tot - free) / 1e9, 1)
  out = {"workload": "C4 HOBE d=256 end to end on the power-law 10M/5M graph: "
                     "alg-dist k=10 x %d, every row sampled (S=%d, K=%d) into "
                     "the record store, one global-shuffle epoch" %
                     (args.alg_iters, S, K),
         "records": n, "time_to_embedding_s": round(total, 2),
         "stages_s": {k: (round(v, 3) if v is not None else None)
                      for k, v in stages.items()},
         "train_records_per_s": (round(n / stages["train_epoch_s"], 1)
                                 if stages.get("train_epoch_s") else None),
         "graph_gen_s": round(gen_s, 1), "ranks": world}
  for k in ("per_batch_us", "chunks", "device_mem_used_gb_at_epoch_end",
            "sampling_chunks"):
    if k in st:
      out[k] = st[k]
  return out


def bench_c5(args, ctx, big):
  """C5 (configs[4]) combiner: CombineEmbeddings' N_E_SUPERVISED MLP
  (combine_embeddings_util.py:78-174) on the 10M/5M graph's own tables --
  [FOBE | HOBE] d = 256 each (HOBE: the table the leg above trained; FOBE:
  its uniform(-0.05, 0.05) init) -- and samples of the graph (a seeded
  subset of the incidences labelled 1 plus 5x as many Python-random-exact
  missing pairs, combine_embeddings_util.incidence_samples). One epoch
  timed after a warm epoch: samples/s and TFLOP/s of the fp32 MFMA engine."""
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.combine_embeddings_util import incidence_samples
  import random as _random
  d = 256
  t = time.perf_counter()
  hn, he = ctx.model_get()
  rs = np.random.RandomState(21)
  nt = np.empty((big.N, 2 * d), np.float32)
  et = np.empty((big.E, 2 * d), np.float32)
  nt[:, :d] = rs.uniform(-0.05, 0.05, (big.N, d))
  et[:, :d] = rs.uniform(-0.05, 0.05, (big.E, d))
  nt[:, d:] = hn[1:]
  et[:, d:] = he[1:]
  del hn, he
  tables_s = time.perf_counter() - t
  _random.seed(5)
  t = time.perf_counter()
  nr, er, lab = incidence_samples(big, args.c5_positives, np.random.RandomState(6))
  samples_s = time.perf_counter() - t
  mlp = _hgx.Mlp(ctx, _hgx.MLP_NE_SUPERVISED, 2 * d, d)
  lims = [np.sqrt(6.0 / (k + n)) for k, n in mlp.shapes]
  w0 = np.concatenate([np.concatenate([rs.uniform(-l, l, k * n), np.zeros(n)])
                       for l, (k, n) in zip(lims, mlp.shapes)]).astype(np.float32)
  mlp.set_weights(w0)
  # the CPU baseline's slice: its samples and only the table rows they read
  # (relabelled; the arithmetic does not depend on row ids)
  cpu_slice = None
  if not args.no_cpu and args.c5_cpu_samples > 0:
    m = min(args.c5_cpu_samples, lab.size)
    sel = np.random.RandomState(22).choice(lab.size, m, replace=False)
    un, inv_n = np.unique(nr[sel], return_inverse=True)
    ue, inv_e = np.unique(er[sel], return_inverse=True)
    cpu_slice = (nt[un], et[ue], inv_n.astype(np.int32), inv_e.astype(np.int32),
                 lab[sel].copy())
  mlp.set_tables(nt, et)
  del nt, et
  mlp.set_samples(nr, er, lab)
  runs = []
  for ep in range(2):
    ctx.synchronize()
    t = time.perf_counter()
    mlp.fit(batch=args.batch, max_epochs=1, min_delta=-1e30, seed=ep + 1)
    ctx.synchronize()
    wall = time.perf_counter() - t
    st = mlp.stats()
    runs.append((st["ms"], st["samples"], st["flops"], wall))
  mlp.close()
  ms, n, flops, wall = runs[-1]
  sps = n / (ms / 1e3)
  tf = flops / (ms / 1e3) / 1e12
  cpu5 = None
  if cpu_slice is not None:
    # CPU baseline (reference fit: combine_embeddings_util.py:151-157): the
    # Keras-semantics restatement oracle/mlpref.c (-O3 AVX2, OpenMP over
    # output rows; the checker the device is bit-exact against) on a random
    # slice of the same samples, one epoch of batch 256
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = cpu_threads()
    O.mlp_set_threads(threads)
    cn, ce, cnr, cer, clab = cpu_slice
    t = time.perf_counter()
    O.mlp_fit(_hgx.MLP_NE_SUPERVISED, 2 * d, d, w0, cn, ce, cnr, cer, clab,
              np.arange(clab.size)[None, :], batch=args.batch, min_delta=-1e30,
              seed=1)
    c_s = time.perf_counter() - t
    restore_affinity()
    c_sps = clab.size / c_s
    cpu5 = {"value": round(c_sps, 1), "unit": "samples/s", "cores": threads,
            "threads": cpu_share_note(threads), "kind": "port",
            "gflops": round(flops / n * c_sps / 1e9, 2),
            "sample": f"{clab.size} random samples of this leg (one epoch, "
                      f"batch {args.batch}), oracle/mlpref.c on {threads} "
                      f"OpenMP threads, {c_s:.1f} s",
            "gpu_vs_cpu": round(sps / c_sps, 1)}
  return {"workload": "N_E_SUPERVISED combiner, in = 512 ([FOBE | HOBE] "
                      "d = 256), d = 256, batch 256, tables of every node "
                      f"and edge of the 10M/5M graph, {n} samples "
                      f"({args.c5_positives} incidences + 5x missing pairs)",
          "samples": n, "epoch_ms": round(ms, 1),
          "samples_per_s": round(sps, 1), "tflops": round(tf, 2),
          "mfma_f32_peak_tflops": MFMA_F32_PEAK_TFLOPS,
          "frac_of_mfma_peak": round(tf / MFMA_F32_PEAK_TFLOPS, 4),
          "c4_epoch_s_implied": round(1.2e9 / sps, 1),
          "host_prep_s": {"tables": round(tables_s, 2),
                          "samples": round(samples_s, 2)},
          "cpu_baseline": cpu5}


if __name__ == "__main__":
  main()
