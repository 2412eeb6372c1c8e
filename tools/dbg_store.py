"""Debug: HOBE records' neighbour draws vs a host replica of the keyed
draws (hgx::draw_record_neighbors), per node-edge block."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle as O
from store_keys import mix64
from hypergraphembedding_amd import _hgx
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph

def rand64_key(seed, stream):
  return mix64(np.uint64(seed) ^ mix64(np.uint64((stream + 0x632be59bd9b4e019) & (2**64-1))))

inc = powerlaw_hypergraph(N=20_000, E=10_000, seed=5)
ctx = _hgx.Context(0)
ctx.upload(inc)
r = O.Rng(3)
ctx.alg_set(r.random((inc.N, 10)), r.random((inc.E, 10)))
ctx.alg_run(20)
seed = 17
n = ctx.sample_hobe(seed, 5, 20)
idx, tgt = ctx.records_get()
b = ctx.records_blocks()
print("blocks", b.tolist(), "N E", inc.N, inc.E)
K = 5
for blk, stream in ((2, 0x500), (3, 0x501)):
  rec = idx[b[blk]:b[blk + 1]]
  print("block", blk, "ids range", rec[:, :4].min(0).tolist(), rec[:, :4].max(0).tolist())
  sel = rec[::max(1, rec.shape[0] // 2000)]
  bad = 0
  for ri in sel:
    v, e = int(ri[0]) - 1, int(ri[3]) - 1
    row, key = (v, e) if blk == 2 else (e, v)
    rk = rand64_key(seed, (stream << 32) | row)
    nb, nl = int(inc.rp_e[e]), int(inc.rp_e[e + 1] - inc.rp_e[e])
    eb, el = int(inc.rp_n[v]), int(inc.rp_n[v + 1] - inc.rp_n[v])
    ks = np.arange(K, dtype=np.uint64)
    with np.errstate(over="ignore"):
      h = mix64(rk + np.uint64(key) * np.uint64(64) + ks)
      h2 = mix64(rk + np.uint64(key) * np.uint64(64) + np.uint64(32) + ks)
    a = inc.col_e[nb + ((h.astype(object) * nl) >> 64).astype(np.int64)] + 1
    c = inc.col_n[eb + ((h2.astype(object) * el) >> 64).astype(np.int64)] + 1
    if not (np.array_equal(a, ri[4:4 + K]) and np.array_equal(c, ri[4 + K:])):
      bad += 1
      if bad <= 3:
        print(" mismatch", ri.tolist(), "want", a.tolist(), c.tolist())
  print("block", blk, "checked", sel.shape[0], "bad", bad)
ctx.store_reset(n)
try:
  ctx.store_append()
  print("append ok")
except Exception as ex:
  print("append:", ex)
ctx.close()

# host emulation of store_pack's check for every record of blocks 2 and 3
def host_check(blk, stream):
  rec = idx[b[blk]:b[blk + 1]]
  tg = tgt[b[blk]:b[blk + 1]]
  if blk == 2:
    row, col = rec[:, 0] - 1, rec[:, 3] - 1
    v, e = row, col
  else:
    row, col = rec[:, 3] - 1, rec[:, 0] - 1
    v, e = col, row
  bits = 0
  if (row < 0).any() or (col < 0).any(): bits |= 32
  if blk == 2 and ((row >= inc.N).any() or (col >= inc.E).any()): bits |= 32
  if blk == 3 and ((row >= inc.E).any() or (col >= inc.N).any()): bits |= 32
  if not (np.all(rec[:, 1] == 0) and np.all(rec[:, 2] == 0)): bits |= 4
  if not (np.all(tg[:, 0] == 0) and np.all(tg[:, 1] == 0)): bits |= 8
  return bits
for blk in (2, 3):
  print("host check block", blk, "bits", hex(host_check(blk, 0)))
# and the other blocks' ids
print("nn block: le/re zero", np.all(idx[b[0]:b[1], [1, 3]] == 0), "ee block: ln/rn zero", np.all(idx[b[1]:b[2], [0, 2]] == 0))
print("block3 sample rows", idx[b[3]:b[3] + 3].tolist(), tgt[b[3]:b[3] + 3].tolist())
print("block3 last rows", idx[b[4] - 3:b[4]].tolist())
