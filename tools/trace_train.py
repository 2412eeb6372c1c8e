"""Phase trace of the trainer kernels (HGX_TRAIN_TRACE): per batch, the
K1/K2 spans, inter-kernel gaps and per-workgroup phase durations from
s_memrealtime stamps (10 ns ticks). Diagnostic only."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx

d = int(sys.argv[1]) if len(sys.argv) > 1 else 128
hobe = len(sys.argv) > 2 and sys.argv[2] == "hobe"  # the C3 HOBE stream
n = int(sys.argv[2]) if len(sys.argv) > 2 and not hobe else 400_000
extra = dict(kv.split("=") for kv in sys.argv[3].split("+")) if len(sys.argv) > 3 else {}
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
if hobe:
  from hypergraphembedding_amd.synthetic import random_hypergraph
  inc = random_hypergraph(seed=0)
  ctx.upload(inc)
  r = np.random.RandomState(4)
  ctx.alg_set(r.random_sample((inc.N, 10)), r.random_sample((inc.E, 10)))
  ctx.alg_run(20)
  m = ctx.sample_hobe(17, 5, 200)
  idx, tgt = ctx.records_get()
  sel = np.random.RandomState(1).permutation(m)[:n]
  idx, tgt = idx[sel], tgt[sel]
ctx.records_set(idx, tgt)
ctx.model_init(d, N + 2, E + 2, seed=1)
os.environ.update(extra)
ctx.train(batch=256, max_epochs=1, loss=1, act=1, min_delta=-1e30)  # warm
path = "gpurun_out/trace.bin" if os.path.isdir("gpurun_out") else "/tmp/trace.bin"
os.environ["HGX_TRAIN_TRACE"] = path
ctx.train(batch=256, max_epochs=1, loss=1, act=1, min_delta=-1e30)
ms, rec, bat = ctx.train_stats()
print(f"{extra} {ms * 1e3 / bat:.2f} us/batch (traced run)")
t = np.fromfile(path, np.uint64).reshape(256, 2, 1024, 8).astype(np.int64)
print("path (fused, split):", ctx.train_path_stats())
if ctx.train_path_stats()[0] > 0:
  # chunk preparation (train_prep of the first chunk: kern slot 1 of batch 0)
  pp = t[0, 1][t[0, 1, :, 0] > 0][:, :6]
  if len(pp):
    dd = np.diff(pp, axis=1) * 0.01
    print(f"train_prep chunk 0: {len(pp)} workgroups, span {(pp[:, 5].max() - pp[:, 0].min()) * 0.01:.1f} us, "
          f"per-WG median total {np.median(pp[:, 5] - pp[:, 0]) * 0.01:.2f} us")
    print("  per-WG median: ids %.2f slot gathers %.2f sort %.2f unique %.2f codes %.2f" %
          tuple(np.median(dd, axis=0)))
    print("  per-WG max:    ids %.2f slot gathers %.2f sort %.2f unique %.2f codes %.2f" %
          tuple(np.max(dd, axis=0)))
  # fused step: kern slot 0 only, stamps start, ids, gathers+row0, compute,
  # emits, multi rows, end
  rows = []
  for b in range(16, 250):
    a1 = t[b, 0][t[b, 0, :, 0] > 0][:, :7]
    n1 = t[b + 1, 0][t[b + 1, 0, :, 0] > 0]
    act = a1[a1[:, 3] > 0]
    if len(a1) == 0 or len(n1) == 0 or len(act) == 0:
      continue
    rows.append([a1[:, 6].max() - a1[:, 0].min(), n1[:, 0].min() - a1[:, 6].max(),
                 n1[:, 0].min() - a1[:, 0].min(), a1[:, 0].max() - a1[:, 0].min(),
                 len(a1), len(act)]
                + list(np.median(np.diff(act, axis=1), axis=0))
                + list(np.max(np.diff(act, axis=1), axis=0)))
  r = np.array(rows, np.float64) * 0.01
  m = np.median(r, axis=0)
  print(f"fused span {m[0]:.2f} us  gap {m[1]:.2f}  batch {m[2]:.2f}  launch skew {m[3]:.2f}  "
        f"blocks {m[4]*100:.0f} active {m[5]*100:.0f}")
  print("per-WG median: ids %.2f gathers+row0 %.2f compute %.2f emits %.2f multi %.2f tail %.2f" % tuple(m[6:12]))
  print("per-WG max:    ids %.2f gathers+row0 %.2f compute %.2f emits %.2f multi %.2f tail %.2f" % tuple(m[12:18]))
  # per workgroup index: median phase durations over batches (which block is slow)
  nb_ = int(m[4] * 100)
  per = np.array([np.median(np.diff(t[16:250, 0, w, :7], axis=1), axis=0) for w in range(nb_)]) * 0.01
  for w in range(nb_):
    print("  wg %2d: " % w + " ".join("%.2f" % v for v in per[w]))
  sys.exit(0)
k1 = t[:, 0, :, :6]
k2 = t[:, 1, :, :4]
rows = []
for b in range(16, 250):
  a1 = k1[b][k1[b, :, 0] > 0]
  a2 = k2[b][k2[b, :, 0] > 0]
  n1 = k1[b + 1][k1[b + 1, :, 0] > 0]
  if len(a1) == 0 or len(a2) == 0 or len(n1) == 0:
    continue
  rows.append([a1[:, 0].min(), a1[:, 5].max(), a2[:, 0].min(), a2[:, 3].max(),
               n1[:, 0].min(), a1[:, 0].max() - a1[:, 0].min(),
               a2[:, 0].max() - a2[:, 0].min(), len(a1), len(a2)]
              + list(np.median(np.diff(a1, axis=1), axis=0))
              + list(np.median(np.diff(a2, axis=1), axis=0))
              + list(np.max(np.diff(a1, axis=1), axis=0)))
r = np.array(rows, np.float64) * 0.01  # ticks -> us
print(f"batches {len(r)}  K1 blocks {int(np.median(r[:, 7] * 100))}  "
      f"K2 blocks {int(np.median(r[:, 8] * 100))}")
m = np.median(r, axis=0)
print(f"K1 span {m[1] - m[0]:.2f} us   gap K1->K2 {np.median(r[:, 2] - r[:, 1]):.2f}   "
      f"K2 span {np.median(r[:, 3] - r[:, 2]):.2f}   gap K2->K1' {np.median(r[:, 4] - r[:, 3]):.2f}   "
      f"batch {np.median(r[:, 4] - r[:, 0]):.2f}")
print(f"launch skew K1 {m[5]:.2f}  K2 {m[6]:.2f}")
print("K1 per-WG median phases: idx %.2f rows %.2f compute %.2f stores %.2f tail %.2f" % tuple(m[9:14]))
print("K1 per-WG max phases:    idx %.2f rows %.2f compute %.2f stores %.2f tail %.2f" % tuple(m[17:22]))
print("K2 per-WG median phases: idx %.2f sums %.2f update %.2f" % tuple(m[14:17]))
