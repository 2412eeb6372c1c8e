"""Test double: a numpy restatement of libhgx's alg_shard_* protocol
(csrc/hgx_algdist.hip hgx_alg_shard_begin/node/edge_partial/edge_final/end)
so the real multi-rank driver (algebraic_distance.alg_dist_sharded) can be
exercised with gloo on CPU. Test infrastructure only.

Buffers are the caller's CPU tensors (passed as data pointers, as the C ABI
passes device pointers):
  partial  float32 E x KS   [sum w, sum w * x_new]  over this rank's node rows
  mm       int32 iters x 2 x KS x 64   order-preserving words, MAX-reduced:
           max slot i holds f2ord(v), min slot KS+i holds ~f2ord(v)
Coordinates are kept unscaled between iterations and the previous
iteration's min/max are applied on read, as the kernels do.
"""

import ctypes

import numpy as np

REP = 64
INT_MIN = np.int32(-2**31)


def f2ord(v):
  u = np.asarray(v, np.float32).view(np.uint32)
  s = np.where(u & 0x80000000, ~u, u | 0x80000000).astype(np.uint32)
  return (s ^ np.uint32(0x80000000)).view(np.int32)


def ord2f(e):
  s = np.asarray(e, np.int32).view(np.uint32) ^ np.uint32(0x80000000)
  u = np.where(s & 0x80000000, s & 0x7fffffff, ~s).astype(np.uint32)
  return u.view(np.float32)


def _view(ptr, n, ctype, dtype):
  return np.ctypeslib.as_array((ctype * n).from_address(ptr)).view(dtype)


class ShardEmu:
  device = None

  def upload(self, inc):
    self.inc = inc

  def alg_set(self, x, y):
    self.k = x.shape[1]
    self.ks = ((self.k + 1) + 3) // 4 * 4
    self.X = np.asarray(x, np.float32).copy()
    self.Y = np.asarray(y, np.float32).copy()

  def alg_shard_begin(self, row0, row1, d_partial, d_mm, iters):
    inc = self.inc
    self.row0, self.row1, self.iters = row0, row1, iters
    self.part = _view(d_partial, inc.E * self.ks, ctypes.c_float,
                      np.float32).reshape(inc.E, self.ks)
    self.mm = _view(d_mm, iters * 2 * self.ks * REP, ctypes.c_int32,
                    np.int32).reshape(iters, 2 * self.ks, REP)
    self.mm[:] = INT_MIN
    self.deg_n = np.diff(inc.rp_n).astype(np.float32)
    self.deg_e = np.diff(inc.rp_e).astype(np.float32)
    self.slot = None
    return self.ks

  def alg_shard_wire(self, d_wire, n_shared, edge_slot):
    """hgx_alg_shard_wire: shared edges' [sum w, sum w x] rows on the wire."""
    self.slot = np.asarray(edge_slot, np.int32)
    self.wire = (_view(d_wire, n_shared * (self.k + 1), ctypes.c_float,
                       np.float32).reshape(n_shared, self.k + 1)
                 if n_shared else np.zeros((0, self.k + 1), np.float32))

  def _affine(self, it):
    """(min, 1/(max-min)) per dim from slot it-1 (identity for it == 0)."""
    if it == 0:
      return np.zeros(self.k, np.float32), np.ones(self.k, np.float32)
    w = self.mm[it - 1].max(axis=1)
    hi = ord2f(w[1:self.k + 1])
    lo = ord2f(~w[self.ks + 1:self.ks + self.k + 1])
    return lo, (np.float32(1) / (hi - lo)).astype(np.float32)

  def _fold(self, it, v):
    slot = self.mm[it]
    hi = f2ord(v.max(axis=0))
    lo = ~f2ord(v.min(axis=0))
    slot[1:self.k + 1, 0] = np.maximum(slot[1:self.k + 1, 0], hi)
    slot[self.ks + 1:self.ks + self.k + 1, 0] = np.maximum(
        slot[self.ks + 1:self.ks + self.k + 1, 0], lo)

  def alg_shard_node(self, it):
    inc, (m, d) = self.inc, self._affine(it)
    ys = (self.Y.astype(np.float64) - m) * d
    xn = self.X.copy()
    for r in range(self.row0, self.row1):
      c = inc.col_n[inc.rp_n[r]:inc.rp_n[r + 1]]
      w = 1.0 / self.deg_e[c].astype(np.float64)
      mean = (w[:, None] * ys[c]).sum(0) / w.sum()
      xn[r] = (((self.X[r] - m) * d + mean) * 0.5).astype(np.float32)
    if self.row1 > self.row0:
      self._fold(it, xn[self.row0:self.row1])
    self.Xn = xn

  def alg_shard_edge_partial(self, it):
    inc = self.inc
    self.part[:] = 0
    for e in range(inc.E):
      c = inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]
      c = c[(c >= self.row0) & (c < self.row1)]
      w = 1.0 / self.deg_n[c].astype(np.float64)
      self.part[e, 0] = w.sum()
      self.part[e, 1:self.k + 1] = (w[:, None] * self.Xn[c]).sum(0)
    if self.slot is not None:
      sh = self.slot >= 0
      self.wire[self.slot[sh]] = self.part[sh, :self.k + 1]

  def alg_shard_ranges(self, n):
    """hgx_alg_shard_ranges: edge ranges balanced by all incidences."""
    rp = np.asarray(self.inc.rp_e, np.int64)
    b = [0]
    for r in range(1, n):
      e = int(np.searchsorted(rp, rp[-1] * r // n, side="left"))
      b.append(max(b[-1], min(e, self.inc.E)))
    b.append(self.inc.E)
    self.bounds = np.array(b, np.int32)
    return self.bounds

  def alg_shard_edge_partial_range(self, it, r):
    inc, e0, e1 = self.inc, int(self.bounds[r]), int(self.bounds[r + 1])
    for e in range(e0, e1):
      c = inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]
      c = c[(c >= self.row0) & (c < self.row1)]
      w = 1.0 / self.deg_n[c].astype(np.float64)
      self.part[e, :] = 0
      self.part[e, 0] = w.sum()
      self.part[e, 1:self.k + 1] = (w[:, None] * self.Xn[c]).sum(0)
      if self.slot is not None and self.slot[e] >= 0:
        self.wire[self.slot[e]] = self.part[e, :self.k + 1]

  def alg_shard_edge_final(self, it):
    m, d = self._affine(it)
    P = self.part[:, :self.k + 1].copy()
    keep = np.ones(self.inc.E, bool)
    if self.slot is not None:
      sh = self.slot >= 0
      P[sh] = self.wire[self.slot[sh]]
      keep = self.slot != -2
    with np.errstate(invalid="ignore", divide="ignore"):
      mean = P[:, 1:] / P[:, :1]
    yn = (((self.Y - m) * d + mean) * 0.5).astype(np.float32)
    yn[~keep] = self.Y[~keep]  # another rank's private edge: not ours
    self._fold(it, yn[keep])
    self.X, self.Y = self.Xn, yn

  def alg_shard_end(self):
    m, d = self._affine(self.iters)
    self.X = ((self.X - m) * d).astype(np.float32)
    self.Y = ((self.Y - m) * d).astype(np.float32)

  def alg_get(self):
    return self.X, self.Y


class SampleEmu:
  """Test double of the row-keyed device samplers for the row-sharded
  sampling drivers (hg2v_sample.sample_sharded / sharded_store_fill): the same
  contract as hgx_sample_hobe_rows / hgx_sample_fobe -- kind blocks nn, ee,
  ne node rows, ne edge rows, each in row order; every draw keyed by (seed,
  block, row, rank in row) -- on a small incidence with numpy. Records are
  host arrays; records_blocks / records_get / records_set as the Context."""
  device = None

  def upload(self, inc):
    self.inc = inc
    A = np.zeros((inc.N, inc.E), bool)
    A[np.repeat(np.arange(inc.N), np.diff(inc.rp_n)), inc.col_n] = True
    self.pat = [A.astype(int) @ A.T.astype(int) > 0,       # nn  (A A^T)
                A.T.astype(int) @ A.astype(int) > 0,       # ee  (A^T A)
                (A.astype(int) @ A.T.astype(int) @ A.astype(int)) > 0,  # ne
                (A.T.astype(int) @ A.astype(int) @ A.T.astype(int)) > 0]

  def _rows(self, blk, q, seed, K):
    inc, out = self.inc, []
    for r in np.flatnonzero(q):
      cols = np.flatnonzero(self.pat[blk][r])
      rs = np.random.RandomState([seed & 0xFFFFFFFF, blk, int(r)])
      pick = np.sort(rs.choice(cols, min(int(q[r]), cols.size), replace=False))
      for j, c in enumerate(pick):
        rec = np.zeros(4 + 2 * K, np.int32)
        t = np.zeros(3, np.float32)
        v, e = (r, c) if blk == 2 else (c, r)
        if blk == 0:
          rec[0], rec[2] = r + 1, c + 1
        elif blk == 1:
          rec[1], rec[3] = r + 1, c + 1
        else:
          rec[0], rec[3] = v + 1, e + 1
          ns = np.random.RandomState([seed & 0xFFFFFFFF, 16 + blk, int(r), j])
          nodes_e = inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]
          edges_v = inc.col_n[inc.rp_n[v]:inc.rp_n[v + 1]]
          rec[4:4 + K] = ns.choice(nodes_e, K) + 1
          rec[4 + K:] = ns.choice(edges_v, K) + 1
        t[min(blk, 2)] = ((r * 131 + c * 7 + blk) % 97) / 97.0
        out.append((rec, t))
    return out

  def sample_hobe(self, seed, K, S, node_q=None, edge_q=None):
    inc = self.inc
    nq = np.full(inc.N, S) if node_q is None else np.asarray(node_q)
    eq = np.full(inc.E, S) if edge_q is None else np.asarray(edge_q)
    blocks = [self._rows(0, nq, seed, K), self._rows(1, eq, seed, K),
              self._rows(2, nq, seed, K), self._rows(3, eq, seed, K)]
    self.K = K
    self.seed = seed
    self.bounds = np.concatenate([[0], np.cumsum([len(b) for b in blocks])])
    recs = [x for b in blocks for x in b]
    self.idx = (np.stack([r for r, _ in recs]) if recs
                else np.zeros((0, 4 + 2 * K), np.int32))
    self.tgt = (np.stack([t for _, t in recs]) if recs
                else np.zeros((0, 3), np.float32))
    return self.idx.shape[0]

  def records_blocks(self):
    return self.bounds.astype(np.int64)

  def records_get(self):
    return self.idx.copy(), self.tgt.copy()

  def records_set(self, idx, tgt):
    self.idx = np.asarray(idx, np.int32).copy()
    self.tgt = np.asarray(tgt, np.float32).copy()
    self.bounds = np.array([0, self.idx.shape[0]], np.int64)

  # ---- the record store's host contract (hgx_store_reset / _append /
  # _info / _read / _write): entries {block << 28 | row, column, target
  # bits} of the HOBE blocks ----
  def store_reset(self, capacity=0):
    self.store = np.zeros((0, 3), np.uint32)
    self.store_meta = None

  def store_append(self):
    meta = (1, self.K, self.seed & (2**64 - 1))
    assert self.store_meta in (None, meta)
    self.store_meta = meta
    ents = []
    cols = ((0, 2, 0), (1, 3, 1), (0, 3, 2), (3, 0, 2))  # row, col, target
    for b in range(4):
      blk = slice(int(self.bounds[b]), int(self.bounds[b + 1]))
      rc, cc, tc = cols[b]
      row = self.idx[blk, rc].astype(np.uint32) - 1
      e = np.stack([(np.uint32(b) << np.uint32(28)) | row,
                    self.idx[blk, cc].astype(np.uint32) - 1,
                    self.tgt[blk, tc].view(np.uint32)], 1)
      ents.append(e)
    self.store = np.concatenate([self.store] + ents).astype(np.uint32)

  def store_info(self):
    fam, K, seed = self.store_meta or (-1, 0, 0)
    return self.store.shape[0], fam, K, seed

  def store_read(self, start=0, n=None, dst_ptr=None):
    assert dst_ptr is None
    n = self.store.shape[0] - start if n is None else n
    return self.store[start:start + n].copy()

  def store_write(self, entries, family, K, seed, n=None, src_ptr=None):
    assert src_ptr is None
    meta = (family, K, seed & (2**64 - 1))
    assert self.store_meta in (None, meta)
    self.store_meta = meta
    self.store = np.concatenate([self.store,
                                 np.asarray(entries, np.uint32).reshape(-1, 3)])
