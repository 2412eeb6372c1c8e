"""ctypes/numpy front-end of the CPU oracle (oracle/hgref.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the CHECKER or the timed CPU baseline, never by
the product package. See hgref.c for the reference file:line each routine
restates and for the parity-pinning status (trainer: parity unpinned).
"""

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_int = ctypes.c_int


def build():
  src = os.path.join(_HERE, "hgref.c")
  if (not os.path.exists(_LIB_PATH) or
      os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
    subprocess.run(["make", "-C", _HERE, "-s"], check=True)
  return _LIB_PATH


def lib():
  global _lib
  if _lib is None:
    build()
    L = ctypes.CDLL(_LIB_PATH)
    L.hgref_rng_create.restype = _vp
    L.hgref_rng_create.argtypes = [ctypes.c_uint32]
    L.hgref_rng_destroy.argtypes = [_vp]
    L.hgref_rng_copy.argtypes = [_vp, _vp]
    L.hgref_rng_next32.restype = ctypes.c_uint32
    L.hgref_rng_next32.argtypes = [_vp]
    L.hgref_rng_random.argtypes = [_vp, _i64, _f64p]
    L.hgref_rng_randint.restype = _i64
    L.hgref_rng_randint.argtypes = [_vp, _i64]
    L.hgref_rng_permutation.argtypes = [_vp, _i64, _i64p]
    L.hgref_spgemm.restype = _i64
    L.hgref_spgemm.argtypes = [_i64, _i32p, _i32p, _i64, _i64, _i32p, _i32p,
                               _vp, _vp]
    L.hgref_algdist.restype = _int
    L.hgref_algdist.argtypes = [_i64, _i64, _int, _int, _i32p, _i32p, _i32p,
                                _i32p, _f64p, _f64p]
    L.hgref_fobe_sample.restype = _i64
    L.hgref_fobe_sample.argtypes = [_vp, _i64, _i64, _i32p, _i32p, _i32p,
                                    _i32p, _i32p, _i32p, _vp, _vp, _int, _i64,
                                    _i32p, _f32p]
    L.hgref_hobe_sample.restype = _i64
    L.hgref_hobe_sample.argtypes = [_vp, _i64, _i64, _i32p, _i32p, _i32p,
                                    _i32p, _f32p, _f32p, _int, _int, _int, _i64,
                                    _i32p, _f32p]
    L.hgref_hobe_probs.argtypes = [_int, _i64, _i32p, _i32p, _i32p, _i32p,
                                   _i32p, _i32p, _f32p, _f32p, _int, _f32p]
    L.hgref_dist_weight.restype = ctypes.c_float
    L.hgref_dist_weight.argtypes = [_f32p, _f32p, _int]
    L.hgref_train.restype = _int
    L.hgref_train.argtypes = [_i64, _int, _i32p, _f32p, _int, _i64, _i64,
                              _f32p, _f32p, _f32p, _f32p, _int, _int, _int,
                              ctypes.c_float, ctypes.c_float, _int, _vp,
                              ctypes.c_float, _f32p,
                              ctypes.POINTER(ctypes.c_int)]
    L.hgref_jaccard_sample.restype = _i64
    L.hgref_jaccard_sample.argtypes = [_vp, _i64, _i64, _i32p, _i32p, _i32p,
                                       _i32p, _f32p, _f32p, _i32p, _i32p, _int,
                                       _i64, _i32p, _f32p]
    L.hgref_jaccard_probs.argtypes = [_int, _i64, _i32p, _i32p, _i64, _i64,
                                      _i32p, _i32p, _i32p, _i32p, _f32p, _f32p,
                                      _f32p]
    L.hgref_centroids.restype = _i64
    L.hgref_centroids.argtypes = [_i64, _i32p, _i32p, _i64, _i32p, _i32p,
                                  _f32p, _i64p, _vp, _vp]
    L.hgref_train_set_dup_f64.argtypes = [_int]
    L.hgref_norm32.restype = ctypes.c_float
    L.hgref_norm32.argtypes = [_f32p, _f32p, _int, _int]
    L.hgref_norm64.restype = ctypes.c_double
    L.hgref_norm64.argtypes = [_f32p, _f32p, _int, _int]
    L.hgref_weight_distance.argtypes = [_i64, _i64, _i32p, _i32p, _i32p, _i32p,
                                        _f32p, _f32p, _int, _int,
                                        ctypes.c_double, _f32p, _f32p]
    L.hgref_weight_same_type.restype = _i64
    L.hgref_weight_same_type.argtypes = [_i64, _i32p, _i32p, _i32p, _i32p,
                                         _f32p, _int, _int, ctypes.c_double,
                                         _vp, _vp, _vp]
    L.hgref_weight_span.argtypes = [_i64, _i64, _i32p, _i32p, _i32p, _i32p,
                                    _f32p, _f32p, _int, ctypes.c_double, _f32p,
                                    _f32p, _f32p, _f32p]
    _lib = L
  return _lib


class Rng:
  """numpy legacy RandomState(seed) stream (MT19937), restated in C."""

  def __init__(self, seed):
    self.h = lib().hgref_rng_create(seed & 0xFFFFFFFF)

  def __del__(self):
    if getattr(self, "h", None) and _lib is not None:
      _lib.hgref_rng_destroy(self.h)
      self.h = None

  def next32(self):
    return lib().hgref_rng_next32(self.h)

  def random(self, shape):
    out = np.empty(int(np.prod(shape)), dtype=np.float64)
    lib().hgref_rng_random(self.h, out.size, out)
    return out.reshape(shape)

  def randint(self, n):
    return lib().hgref_rng_randint(self.h, n)

  def permutation(self, n):
    out = np.empty(n, dtype=np.int64)
    lib().hgref_rng_permutation(self.h, n, out)
    return out


def spgemm(ap, aj, nrow_b, ncol_b, bp, bj):
  """Pattern of A*B with scipy's SMMP column order: (indptr int64, indices)."""
  ap = np.ascontiguousarray(ap, np.int32)
  aj = np.ascontiguousarray(aj, np.int32)
  bp = np.ascontiguousarray(bp, np.int32)
  bj = np.ascontiguousarray(bj, np.int32)
  nrow = ap.size - 1
  nnz = lib().hgref_spgemm(nrow, ap, aj, nrow_b, ncol_b, bp, bj, None, None)
  outp = np.empty(nrow + 1, np.int64)
  outj = np.empty(max(nnz, 1), np.int32)
  lib().hgref_spgemm(nrow, ap, aj, nrow_b, ncol_b, bp, bj,
                     outp.ctypes.data, outj.ctypes.data)
  return outp, outj[:nnz]


def algdist(inc, x, y, iters):
  """In-place float64 relaxation; returns (x, y). Raises ZeroDivisionError on
  an isolated row like algebraic_distance.py:49."""
  x = np.ascontiguousarray(x, np.float64).copy()
  y = np.ascontiguousarray(y, np.float64).copy()
  k = x.shape[1]
  rc = lib().hgref_algdist(inc.N, inc.E, k, iters, inc.rp_n, inc.col_n,
                           inc.rp_e, inc.col_e, x, y)
  if rc != 0:
    raise ZeroDivisionError("isolated node or edge in algebraic distance")
  return x, y


def _q(a):
  return None if a is None else np.ascontiguousarray(a, np.int32)


def fobe_sample(rng, inc, node_q, edge_q, K, neg_node_q=None, neg_edge_q=None):
  """BooleanSamples -> SamplesToModelInput arrays (idx (n,4+2K), tgt (n,3))."""
  node_q, edge_q = _q(node_q), _q(edge_q)
  nnq, neq = _q(neg_node_q), _q(neg_edge_q)
  cap = 2 * int(node_q.sum()) + 2 * int(edge_q.sum()) + 1
  if nnq is not None:
    cap += int(nnq.sum()) * 2 + int(neq.sum()) * 3
  idx = np.zeros((cap, 4 + 2 * K), np.int32)
  tgt = np.zeros((cap, 3), np.float32)
  n = lib().hgref_fobe_sample(
      rng.h, inc.N, inc.E, inc.rp_n, inc.col_n, inc.rp_e, inc.col_e, node_q,
      edge_q, None if nnq is None else nnq.ctypes.data,
      None if neq is None else neq.ctypes.data, K, cap, idx, tgt)
  assert n >= 0
  return idx[:n].copy(), tgt[:n].copy()


def hobe_sample(rng, inc, alg_node, alg_edge, S, K):
  """AlgebraicDistanceSamples (run_in_parallel=False) -> model input arrays."""
  alg_node = np.ascontiguousarray(alg_node, np.float32)
  alg_edge = np.ascontiguousarray(alg_edge, np.float32)
  cap = 2 * S * (inc.N + inc.E) + 1
  idx = np.zeros((cap, 4 + 2 * K), np.int32)
  tgt = np.zeros((cap, 3), np.float32)
  n = lib().hgref_hobe_sample(rng.h, inc.N, inc.E, inc.rp_n, inc.col_n,
                              inc.rp_e, inc.col_e, alg_node, alg_edge,
                              alg_node.shape[1], S, K, cap, idx, tgt)
  assert n >= 0
  return idx[:n].copy(), tgt[:n].copy()


HOBE_NN, HOBE_EE, HOBE_NE = 0, 1, 2
JAC_NN, JAC_EE, JAC_NE = 0, 1, 2


def jaccard_sample(rng, inc, fn, fe, node_q, edge_q, K):
  """WeightedJaccardSamples (run_in_parallel=False) -> model input arrays.
  fn / fe: feature values on A's pattern, node-major / edge-major order."""
  fn = np.ascontiguousarray(fn, np.float32)
  fe = np.ascontiguousarray(fe, np.float32)
  node_q, edge_q = _q(node_q), _q(edge_q)
  cap = 2 * int(node_q.sum()) + 2 * int(edge_q.sum()) + 1
  idx = np.zeros((cap, 4 + 2 * K), np.int32)
  tgt = np.zeros((cap, 3), np.float32)
  n = lib().hgref_jaccard_sample(rng.h, inc.N, inc.E, inc.rp_n, inc.col_n,
                                 inc.rp_e, inc.col_e, fn, fe, node_q, edge_q,
                                 K, cap, idx, tgt)
  assert n >= 0
  return idx[:n].copy(), tgt[:n].copy()


def jaccard_probs(kind, a, b, inc, fn, fe):
  a = np.ascontiguousarray(a, np.int32)
  b = np.ascontiguousarray(b, np.int32)
  out = np.empty(a.size, np.float32)
  lib().hgref_jaccard_probs(kind, a.size, a, b, inc.N, inc.E, inc.rp_n,
                            inc.col_n, inc.rp_e, inc.col_e,
                            np.ascontiguousarray(fn, np.float32),
                            np.ascontiguousarray(fe, np.float32), out)
  return out


def centroids(R, rp, col, ncols, frp, fcol, fval):
  """CSR (p int64, j, v) of GetAllCentroids."""
  rp = np.ascontiguousarray(rp, np.int32)
  col = np.ascontiguousarray(col, np.int32)
  frp = np.ascontiguousarray(frp, np.int32)
  fcol = np.ascontiguousarray(fcol, np.int32)
  fval = np.ascontiguousarray(fval, np.float32)
  p = np.empty(R + 1, np.int64)
  nnz = lib().hgref_centroids(R, rp, col, ncols, frp, fcol, fval, p, None, None)
  j = np.empty(nnz, np.int32)
  v = np.empty(nnz, np.float32)
  lib().hgref_centroids(R, rp, col, ncols, frp, fcol, fval, p, j.ctypes.data,
                        v.ctypes.data)
  return p, j, v


def hobe_probs(kind, a, b, inc, alg_node, alg_edge):
  a = np.ascontiguousarray(a, np.int32)
  b = np.ascontiguousarray(b, np.int32)
  alg_node = np.ascontiguousarray(alg_node, np.float32)
  alg_edge = np.ascontiguousarray(alg_edge, np.float32)
  out = np.empty(a.size, np.float32)
  lib().hgref_hobe_probs(kind, a.size, a, b, inc.rp_n, inc.col_n, inc.rp_e,
                         inc.col_e, alg_node, alg_edge, alg_node.shape[1], out)
  return out


LOSS_KLD, LOSS_MSE = 0, 1
ACT_SIGMOID, ACT_RELU = 0, 1


def train(idx, tgt, K, node_tab, edge_tab, loss, act, batch=256, lr=0.01,
          eps=1e-7, max_epochs=10, perms=None, min_delta=1e-3, node_acc=None,
          edge_acc=None, dup_f64=False):
  """Keras-semantics Adagrad restatement. Tables are float32 (rows = max+2,
  row 0 = padding). dup_f64: a row's gradients summed in float64 and
  rounded once (the exact member of the fp32 summation orders TF allows)
  instead of float32 in emit order. Returns (node_tab, edge_tab,
  epoch_losses, node_acc, edge_acc)."""
  idx = np.ascontiguousarray(idx, np.int32)
  tgt = np.ascontiguousarray(tgt, np.float32)
  nt = np.ascontiguousarray(node_tab, np.float32).copy()
  et = np.ascontiguousarray(edge_tab, np.float32).copy()
  na = (np.zeros_like(nt) if node_acc is None
        else np.ascontiguousarray(node_acc, np.float32).copy())
  ea = (np.zeros_like(et) if edge_acc is None
        else np.ascontiguousarray(edge_acc, np.float32).copy())
  n = idx.shape[0]
  d = nt.shape[1]
  pp = None
  if perms is not None:
    perms = np.ascontiguousarray(perms, np.int64)
    assert perms.shape[1] == n and perms.shape[0] >= 1
    max_epochs = min(max_epochs, perms.shape[0])
    pp = perms.ctypes.data
  losses = np.zeros(max(max_epochs, 1), np.float32)
  ran = ctypes.c_int(0)
  lib().hgref_train_set_dup_f64(1 if dup_f64 else 0)
  lib().hgref_train(n, K, idx, tgt, d, nt.shape[0], et.shape[0], nt, et, na,
                    ea, loss, act, batch, lr, eps, max_epochs, pp, min_delta,
                    losses, ctypes.byref(ran))
  return nt, et, losses[:ran.value].copy(), na, ea


_mt = {}


def _mt_lib(exact):
  name = "libcpumt_chk.so" if exact else "libcpumt.so"
  if name not in _mt:
    build()
    path = os.path.join(_HERE, name)
    src = os.path.join(_HERE, "cpu_train_mt.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
      subprocess.run(["make", "-C", _HERE, "-s", name], check=True)
    L = ctypes.CDLL(path)
    L.cpu_train_mt.restype = _int
    L.cpu_train_mt.argtypes = [_i64, _int, _i32p, _f32p, _int, _i64, _i64,
                               _f32p, _f32p, _f32p, _f32p, _int, _int, _int,
                               ctypes.c_float, ctypes.c_float, _int, _int,
                               ctypes.POINTER(ctypes.c_double)]
    _mt[name] = L
  return _mt[name]


def train_mt(idx, tgt, K, node_tab, edge_tab, loss, act, batch=256, lr=0.01,
             eps=1e-7, epochs=1, threads=0, copy=True, exact=False):
  """Multi-threaded CPU trainer (cpu_train_mt.c; records in the given
  order). exact=False: the bench's CPU baseline build (-O3, AVX2/FMA);
  exact=True: the checker build, rounding like hgref_train (no contraction)
  -- used as the oracle where the stream is too long for the scalar one.
  Updates copies of the tables (copy=False: the given float32 tables in
  place); returns (nt, et, mean loss)."""
  lib_ = _mt_lib(exact)
  idx = np.ascontiguousarray(idx, np.int32)
  tgt = np.ascontiguousarray(tgt, np.float32)
  nt = np.ascontiguousarray(node_tab, np.float32)
  et = np.ascontiguousarray(edge_tab, np.float32)
  if copy:
    nt, et = nt.copy(), et.copy()
  na, ea = np.zeros_like(nt), np.zeros_like(et)
  lo = ctypes.c_double()
  lib_.cpu_train_mt(idx.shape[0], K, idx, tgt, nt.shape[1], nt.shape[0],
                    et.shape[0], nt, et, na, ea, loss, act, batch, lr, eps,
                    epochs, threads, ctypes.byref(lo))
  return nt, et, lo.value

_mlp = None


def _mlp_lib():
  global _mlp
  if _mlp is None:
    path = os.path.join(_HERE, "libmlpref.so")
    src = os.path.join(_HERE, "mlpref.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
      subprocess.run(["make", "-C", _HERE, "-s", "libmlpref.so"], check=True)
    L = ctypes.CDLL(path)
    L.mlpref_num_weights.argtypes = [_int, _int, _int, ctypes.POINTER(_i64)]
    L.mlpref_fit.restype = _int
    L.mlpref_fit.argtypes = [_int, _int, _int, _f32p, _i64, _f32p, _i64, _f32p,
                             _i64, _i32p, _i32p, _f32p, _int, _int,
                             ctypes.c_float, ctypes.c_float, ctypes.c_float,
                             ctypes.c_uint64, _i64p, _i64, _f32p,
                             ctypes.POINTER(ctypes.c_int)]
    L.mlpref_set_threads.argtypes = [_int]
    L.mlpref_predict.restype = _int
    L.mlpref_predict.argtypes = [_int, _int, _int, _f32p, _i64, _f32p, _i64,
                                 _f32p, _int, _i64, _vp, _vp, _f32p]
    _mlp = L
  return _mlp


def mlp_set_threads(threads):
  """OpenMP threads of mlpref.c's loops (timing only; results unchanged)."""
  _mlp_lib().mlpref_set_threads(int(threads))


def mlp_num_weights(kind, in_dim, out_dim):
  n = _i64()
  _mlp_lib().mlpref_num_weights(kind, in_dim, out_dim, ctypes.byref(n))
  return n.value


def mlp_fit(kind, in_dim, out_dim, weights, node_tab, edge_tab, node_row,
            edge_row, label, perms, batch=256, lr=0.01, eps=1e-7, min_delta=0.0,
            seed=0, max_batches=0):
  """mlpref.c: Keras-semantics fit of the combiner / classifier MLP with the
  device's dropout masks; batches in `perms` order (epochs x n). Returns
  (weights after training, epoch losses)."""
  w = np.ascontiguousarray(weights, np.float32).copy()
  nt = np.ascontiguousarray(node_tab, np.float32)
  et = np.ascontiguousarray(edge_tab, np.float32)
  nr = np.ascontiguousarray(node_row, np.int32)
  er = np.ascontiguousarray(edge_row, np.int32)
  lab = np.ascontiguousarray(label, np.float32)
  perms = np.ascontiguousarray(perms, np.int64)
  epochs = perms.shape[0]
  losses = np.zeros(max(epochs, 1), np.float32)
  ran = ctypes.c_int()
  _mlp_lib().mlpref_fit(kind, in_dim, out_dim, w, nt.shape[0], nt, et.shape[0],
                        et, nr.size, nr, er, lab, batch, epochs, lr, eps,
                        min_delta, seed & (2**64 - 1), perms, max_batches,
                        losses, ctypes.byref(ran))
  return w, losses[:ran.value].copy()


def mlp_predict(kind, in_dim, out_dim, weights, node_tab, edge_tab, output,
                node_row=None, edge_row=None):
  w = np.ascontiguousarray(weights, np.float32)
  nt = np.ascontiguousarray(node_tab, np.float32)
  et = np.ascontiguousarray(edge_tab, np.float32)
  nr = None if node_row is None else np.ascontiguousarray(node_row, np.int32)
  er = None if edge_row is None else np.ascontiguousarray(edge_row, np.int32)
  n = (nr if nr is not None else er).size
  out = np.empty(n if output == 0 else n * out_dim, np.float32)
  _mlp_lib().mlpref_predict(kind, in_dim, out_dim, w, nt.shape[0], nt,
                            et.shape[0], et, output, n,
                            None if nr is None else nr.ctypes.data,
                            None if er is None else er.ctypes.data, out)
  return out if output == 0 else out.reshape(n, out_dim)


_smp = None


def cpu_hobe_sample_mt(inc, alg_node, alg_edge, node_q, edge_q, K, seed=0,
                       threads=0):
  """Multi-threaded CPU HOBE sampler (cpu_sample_mt.c; bench baseline, exact
  expansion per row). Returns (idx, tgt, block bounds[5])."""
  global _smp
  if _smp is None:
    path = os.path.join(_HERE, "libcpusample.so")
    src = os.path.join(_HERE, "cpu_sample_mt.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
      subprocess.run(["make", "-C", _HERE, "-s", "libcpusample.so"], check=True)
    _smp = ctypes.CDLL(path)
    _smp.cpu_hobe_sample_mt.restype = _i64
    _smp.cpu_hobe_sample_mt.argtypes = [ctypes.c_int32, ctypes.c_int32, _i32p,
                                        _i32p, _i32p, _i32p, _f32p, _f32p, _int,
                                        _i32p, _i32p, _int, ctypes.c_uint64,
                                        _int, _i32p, _f32p, _i64p]
  nq = np.ascontiguousarray(node_q, np.int32)
  eq = np.ascontiguousarray(edge_q, np.int32)
  an = np.ascontiguousarray(alg_node, np.float32)
  ae = np.ascontiguousarray(alg_edge, np.float32)
  cap = 2 * (int(nq.sum()) + int(eq.sum())) + 1
  idx = np.empty((cap, 4 + 2 * K), np.int32)
  tgt = np.empty((cap, 3), np.float32)
  b = np.zeros(5, np.int64)
  n = _smp.cpu_hobe_sample_mt(inc.N, inc.E, np.ascontiguousarray(inc.rp_n, np.int32),
                              np.ascontiguousarray(inc.col_n, np.int32),
                              np.ascontiguousarray(inc.rp_e, np.int32),
                              np.ascontiguousarray(inc.col_e, np.int32), an, ae,
                              an.shape[1], nq, eq, K, seed & (2**64 - 1),
                              threads, idx, tgt, b)
  assert n >= 0
  return idx[:n], tgt[:n], b


# ---- hg2v_weighting distance / span weights (hgref.c) ----------------------
NORM_L2, NORM_INF = 0, 1


def _csr(inc):
  return (np.ascontiguousarray(inc.rp_n, np.int32),
          np.ascontiguousarray(inc.col_n, np.int32),
          np.ascontiguousarray(inc.rp_e, np.int32),
          np.ascontiguousarray(inc.col_e, np.int32))


def weight_distance(inc, X, Y, norm=NORM_L2, alpha=0.0):
  """WeightByDistance values per incidence (A, A^T order; zeros kept)."""
  X = np.ascontiguousarray(X, np.float32)
  Y = np.ascontiguousarray(Y, np.float32)
  out_n = np.empty(inc.nnz, np.float32)
  out_e = np.empty(inc.nnz, np.float32)
  lib().hgref_weight_distance(inc.N, inc.E, *_csr(inc), X, Y, X.shape[1], norm,
                              float(alpha), out_n, out_e)
  return out_n, out_e


def weight_same_type(inc, side, tab, norm=NORM_L2, alpha=0.0):
  """WeightBySameTypeDistance half: (rowptr int64, col int32, val float32)
  over compressed ids (zeros kept)."""
  rp_n, col_n, rp_e, col_e = _csr(inc)
  P = (rp_n, col_n, rp_e, col_e) if side == 0 else (rp_e, col_e, rp_n, col_n)
  R = inc.N if side == 0 else inc.E
  tab = np.ascontiguousarray(tab, np.float32)
  rowptr = np.empty(R + 1, np.int64)
  nnz = lib().hgref_weight_same_type(R, *P, tab, tab.shape[1], norm,
                                     float(alpha), rowptr.ctypes.data, None,
                                     None)
  col = np.empty(max(nnz, 1), np.int32)
  val = np.empty(max(nnz, 1), np.float32)
  lib().hgref_weight_same_type(R, *P, tab, tab.shape[1], norm, float(alpha),
                               rowptr.ctypes.data, col.ctypes.data,
                               val.ctypes.data)
  return rowptr, col[:nnz], val[:nnz]


def weight_span(inc, X, Y, alpha=0.0):
  """ComputeSpans (float32) + WeightByAlgebraicSpan values per incidence."""
  X = np.ascontiguousarray(X, np.float32)
  Y = np.ascontiguousarray(Y, np.float32)
  sn = np.empty(inc.N, np.float32)
  se = np.empty(inc.E, np.float32)
  wn = np.empty(inc.nnz, np.float32)
  we = np.empty(inc.nnz, np.float32)
  lib().hgref_weight_span(inc.N, inc.E, *_csr(inc), X, Y, X.shape[1],
                          float(alpha), sn, se, wn, we)
  return sn, se, wn, we
