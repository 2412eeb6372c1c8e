"""ctypes binding of libhgx.so (include/hgx.h) -- the only way the package
reaches the GPU. There is no CPU fallback: if the library or a HIP device is
missing, every entry point raises.
"""

import ctypes
import os
import re
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libhgx.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "hgx.h")

HGX_OK, HGX_EINVAL, HGX_EHIP, HGX_ENOMEM = 0, -1, -2, -3
HGX_EZERODIV, HGX_ESTATE, HGX_EUNSUP, HGX_EVALUE = -4, -5, -6, -7
HGX_ENUMERIC = -8
LOSS_KLD, LOSS_MSE = 0, 1
ACT_SIGMOID, ACT_RELU = 0, 1
HOBE_NN, HOBE_EE, HOBE_NE = 0, 1, 2
WEIGHT_UNIFORM, WEIGHT_NEIGHBORHOOD, WEIGHT_DISTANCE = 0, 1, 2
NORM_L2, NORM_INF = 0, 1
MLP_LP_CLASSIFIER, MLP_NE_SUPERVISED, MLP_NE_SEMI_SUPERVISED = 0, 1, 2
STORE_FOBE, STORE_HOBE = 0, 1
STORE_BINS = 16384

_lib = None

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_int = ctypes.c_int
_f32 = ctypes.c_float
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pint = ctypes.POINTER(ctypes.c_int)
_pdbl = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); mirrors include/hgx.h one to one.
SIGNATURES = {
    "hgx_create": (_int, [_int, ctypes.POINTER(_vp)]),
    "hgx_destroy": (_int, [_vp]),
    "hgx_last_error": (ctypes.c_char_p, [_vp]),
    "hgx_version": (_int, []),
    "hgx_set_stream": (_int, [_vp, _vp]),
    "hgx_synchronize": (_int, [_vp]),
    "hgx_device_count": (_int, [_pint]),
    "hgx_mem_info": (_int, [_vp, _pi64, _pi64]),
    "hgx_set_tuning": (_int, [_vp, ctypes.c_char_p, _i64]),
    "hgx_upload_incidence": (_int, [_vp, _i32, _i32, _i64, _vp, _vp, _vp, _vp]),
    "hgx_alg_dist": (_int, [_vp, _int, _int, _vp, _vp]),
    "hgx_alg_set": (_int, [_vp, _int, _vp, _vp]),
    "hgx_alg_run": (_int, [_vp, _int]),
    "hgx_alg_get": (_int, [_vp, _vp, _vp]),
    "hgx_alg_last_stats": (_int, [_vp, _pdbl, _pdbl]),
    "hgx_alg_shard_begin": (_int, [_vp, _i32, _i32, _vp, _vp, _int, _pint]),
    "hgx_alg_shard_node": (_int, [_vp, _int]),
    "hgx_alg_shard_edge_partial": (_int, [_vp, _int]),
    "hgx_alg_shard_edge_final": (_int, [_vp, _int]),
    "hgx_alg_shard_end": (_int, [_vp]),
    "hgx_alg_shard_wire": (_int, [_vp, _vp, _i64, _vp]),
    "hgx_alg_shard_ranges": (_int, [_vp, _int, _vp]),
    "hgx_alg_shard_edge_partial_range": (_int, [_vp, _int, _int]),
    "hgx_hobe_probs": (_int, [_vp, _int, _i64, _vp, _vp, _vp]),
    "hgx_incidence_weights": (_int, [_vp, _int, ctypes.c_double, _vp, _vp]),
    "hgx_weight_distance": (_int, [_vp, _int, ctypes.c_double, _vp, _vp]),
    "hgx_weight_same_type": (_int, [_vp, _int, _int, ctypes.c_double, _pi64,
                                    _vp, _vp, _vp]),
    "hgx_weight_span": (_int, [_vp, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "hgx_sample_fobe": (_int, [_vp, _u64, _int, _vp, _vp, _vp, _vp, _pi64]),
    "hgx_sample_hobe": (_int, [_vp, _u64, _int, _int, _pi64]),
    "hgx_sample_hobe_rows": (_int, [_vp, _u64, _int, _vp, _vp, _int, _pi64]),
    "hgx_sample_fobe_mt": (_int, [_vp, _vp, _pint, _int, _vp, _vp, _vp, _vp,
                                  _pi64]),
    "hgx_sample_hobe_mt": (_int, [_vp, _vp, _pint, _int, _int, _pi64]),
    "hgx_sample_jaccard_mt": (_int, [_vp, _vp, _pint, _int, _vp, _vp, _pi64]),
    "hgx_sample_last_stats": (_int, [_vp, _pi64, _pi64]),
    "hgx_sample_uniform_rows": (_int, [_vp, _pi64]),
    "hgx_features_set": (_int, [_vp, _vp, _vp]),
    "hgx_sample_jaccard": (_int, [_vp, _u64, _int, _vp, _vp, _pi64]),
    "hgx_jaccard_probs": (_int, [_vp, _int, _i64, _vp, _vp, _vp]),
    "hgx_jaccard_centroids": (_int, [_vp, _int, _pi64, _vp, _vp, _vp]),
    "hgx_records_set": (_int, [_vp, _i64, _int, _vp, _vp]),
    "hgx_records_info": (_int, [_vp, _pi64, _pint]),
    "hgx_records_copy": (_int, [_vp, _vp]),
    "hgx_records_get": (_int, [_vp, _vp, _vp]),
    "hgx_records_blocks": (_int, [_vp, _pint, _vp]),
    "hgx_records_export": (_int, [_vp, _vp, _vp]),
    "hgx_records_import": (_int, [_vp, _i64, _int, _vp, _vp, _int, _vp]),
    "hgx_store_reset": (_int, [_vp, _i64]),
    "hgx_store_append": (_int, [_vp]),
    "hgx_store_info": (_int, [_vp, _pi64, _pint, _pint,
                              ctypes.POINTER(ctypes.c_uint64)]),
    "hgx_store_read": (_int, [_vp, _i64, _i64, _vp, _int]),
    "hgx_store_write": (_int, [_vp, _i64, _vp, _int, _int, _int, _u64]),
    "hgx_store_plan": (_int, [_vp, _u64, _i64, _pint, _vp, _vp]),
    "hgx_store_load": (_int, [_vp, _u64, _i32, _i32, _int, _int, _pi64]),
    "hgx_store_release": (_int, [_vp]),
    "hgx_model_init": (_int, [_vp, _int, _i64, _i64, _u64, _vp, _vp]),
    "hgx_model_get": (_int, [_vp, _vp, _vp]),
    "hgx_model_get_rows": (_int, [_vp, _int, _i64, _vp, _vp]),
    "hgx_probe_gather": (_int, [_vp, _i64, _int, _int, _int, _pdbl]),
    "hgx_train": (_int, [_vp, _int, _int, _f32, _f32, _int, _int, _f32, _u64,
                         _vp, _vp, _pint]),
    "hgx_train_last_stats": (_int, [_vp, _pdbl, _pi64, _pi64]),
    "hgx_train_path_stats": (_int, [_vp, _pi64, _pi64]),
    "hgx_train_multi_pending": (_int, [_vp, _pi64]),
    "hgx_train_last_loss": (_int, [_vp, _pdbl]),
    "hgx_synth_powerlaw": (_int, [_i32, _i32, ctypes.c_double, ctypes.c_double,
                                  _u64, _vp, _vp, _pi64,
                                  ctypes.POINTER(ctypes.c_int32)]),
    "hgx_csr_transpose": (_int, [_i32, _i32, _vp, _vp, _vp, _vp]),
    "hgx_proto_parse_hypergraph": (_int, [_vp, _i64, ctypes.POINTER(_vp),
                                          ctypes.POINTER(_i32),
                                          ctypes.POINTER(_i32), _pi64]),
    "hgx_proto_hypergraph_fill": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "hgx_proto_hypergraph_free": (None, [_vp]),
    "hgx_proto_write_embedding": (_int, [_i64, _vp, _vp, _i64, _vp, _vp, _int,
                                         ctypes.c_char_p, _vp, _i64, _pi64]),
    "hgx_host_last_error": (ctypes.c_char_p, []),
    "hgx_proto_parse_embedding": (_int, [_vp, _i64, ctypes.POINTER(_vp), _pi64,
                                         _pi64, _pi64,
                                         ctypes.POINTER(_i32)]),
    "hgx_proto_embedding_fill": (_int, [_vp, _vp, _vp, _vp, _vp,
                                        ctypes.c_char_p, _i64]),
    "hgx_proto_embedding_method_len": (_i64, [_vp]),
    "hgx_proto_embedding_free": (None, [_vp]),
    "hgx_proto_write_hypergraph": (_int, [_i32, _i32, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _i64, _pi64]),
    "hgx_mlp_create": (_int, [_vp, _int, _int, _int, ctypes.POINTER(_vp)]),
    "hgx_mlp_destroy": (_int, [_vp]),
    "hgx_mlp_layers": (_int, [_vp, _pint, _vp]),
    "hgx_mlp_set_weights": (_int, [_vp, _vp]),
    "hgx_mlp_get_weights": (_int, [_vp, _vp]),
    "hgx_mlp_set_tables": (_int, [_vp, _i64, _vp, _i64, _vp]),
    "hgx_mlp_set_samples": (_int, [_vp, _i64, _vp, _vp, _vp]),
    "hgx_mlp_fit": (_int, [_vp, _int, _int, _f32, _f32, _f32, _u64, _vp, _vp,
                           _pint]),
    "hgx_mlp_predict": (_int, [_vp, _int, _i64, _vp, _vp, _vp]),
    "hgx_mlp_last_stats": (_int, [_vp, _pdbl, _pi64, _pi64, _pdbl]),
    "hgx_pyrandom_sample_missing": (_int, [_vp, _i32, _i32, _vp, _vp, _i64,
                                           _vp, _vp, _pi64]),
    "hgx_pyrandom_remove_connections": (_int, [_vp, _i64, _vp, _vp, _vp, _vp,
                                               ctypes.c_double, _vp, _pi64]),
    "hgx_lp_last_error": (ctypes.c_char_p, []),
}


def header_symbols():
  """Function names declared in include/hgx.h."""
  with open(HEADER) as f:
    text = f.read()
  text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
  return sorted(set(re.findall(r"\b(hgx_[a-z0-9_]+)\s*\(", text)))


def lib():
  """Load libhgx.so (raises if it was not built)."""
  global _lib
  if _lib is None:
    # HGX_LIB_PATH: load another build of the same ABI (A/B timing)
    path = os.environ.get("HGX_LIB_PATH") or LIB_PATH
    if not os.path.exists(path):
      raise ImportError(
          f"{path} missing: run hypergraphembedding_amd.build.build() "
          "(there is no CPU fallback)")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
      fn = getattr(L, name)
      fn.restype = res
      fn.argtypes = args
    _lib = L
  return _lib


class HgxError(RuntimeError):
  pass


def _raise(rc, msg):
  if rc == HGX_EINVAL:
    raise AssertionError(msg)
  if rc == HGX_EZERODIV:
    raise ZeroDivisionError(msg)
  if rc == HGX_EVALUE:
    raise ValueError(msg)
  if rc == HGX_ENUMERIC:
    raise FloatingPointError(msg)
  raise HgxError(f"libhgx error {rc}: {msg}")


def _ptr(a):
  return None if a is None else a.ctypes.data


def _c(a, dtype):
  return None if a is None else np.ascontiguousarray(a, dtype=dtype)


def device_count():
  """HIP devices visible to libhgx (hipGetDeviceCount)."""
  n = ctypes.c_int()
  lib().hgx_device_count(ctypes.byref(n))
  return n.value


class Context:
  """One device context (owns device memory and one HIP stream)."""

  def __init__(self, device=0):
    h = _vp()
    rc = lib().hgx_create(device, ctypes.byref(h))
    if rc != HGX_OK:
      _raise(rc, f"hgx_create(device={device}) failed: no usable HIP device")
    self.h = h
    self.device = device
    self._engines = weakref.WeakSet()  # Mlp engines living on this context

  def close(self):
    if getattr(self, "h", None):
      for e in list(getattr(self, "_engines", ())):
        e.close()
      lib().hgx_destroy(self.h)
      self.h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

  def _chk(self, rc):
    if rc != HGX_OK:
      _raise(rc, lib().hgx_last_error(self.h).decode(errors="replace"))

  # ---- plumbing ----
  def set_stream(self, stream_ptr):
    self._chk(lib().hgx_set_stream(self.h, stream_ptr))

  def synchronize(self):
    self._chk(lib().hgx_synchronize(self.h))

  def mem_info(self):
    """(free, total) bytes of the context's device (hipMemGetInfo)."""
    f, t = ctypes.c_int64(), ctypes.c_int64()
    self._chk(lib().hgx_mem_info(self.h, ctypes.byref(f), ctypes.byref(t)))
    return f.value, t.value

  def set_tuning(self, key, value):
    """Pick between exact implementations (hgx_set_tuning): sample_reject_w,
    sample_mode3, sample_mode3_shift, sample_mode3_shift_e, train_fused,
    train_lanes, train_tb, train_prep_overlap, train_prep_cus, alg_long,
    alg_ks, alg_push, mlp_fuse_head, mlp_prefetch, mlp_wgrad_split,
    stream_cus."""
    self._chk(lib().hgx_set_tuning(self.h, key.encode(), int(value)))

  # ---- incidence ----
  def upload(self, inc):
    self.inc = inc
    self._keep = (_c(inc.rp_n, np.int32), _c(inc.col_n, np.int32),
                  _c(inc.rp_e, np.int32), _c(inc.col_e, np.int32))
    a, b, c, d = self._keep
    self._chk(lib().hgx_upload_incidence(self.h, inc.N, inc.E, inc.nnz,
                                         _ptr(a), _ptr(b), _ptr(c), _ptr(d)))

  # ---- algebraic distance ----
  def alg_set(self, x, y):
    x = _c(x, np.float32)
    y = _c(y, np.float32)
    assert x.ndim == 2 and y.ndim == 2 and x.shape[1] == y.shape[1]
    self.k = x.shape[1]
    self._chk(lib().hgx_alg_set(self.h, self.k, _ptr(x), _ptr(y)))

  def alg_run(self, iters):
    self._chk(lib().hgx_alg_run(self.h, iters))

  def alg_get(self):
    x = np.empty((self.inc.N, self.k), np.float32)
    y = np.empty((self.inc.E, self.k), np.float32)
    self._chk(lib().hgx_alg_get(self.h, _ptr(x), _ptr(y)))
    return x, y

  def alg_dist(self, x, y, iters):
    self.alg_set(x, y)
    self.alg_run(iters)
    return self.alg_get()

  def alg_stats(self):
    ms, by = ctypes.c_double(), ctypes.c_double()
    self._chk(lib().hgx_alg_last_stats(self.h, ctypes.byref(ms),
                                       ctypes.byref(by)))
    return ms.value, by.value

  # sharded relaxation (exchange buffers are caller-owned device pointers)
  def alg_shard_begin(self, row0, row1, d_partial, d_mm, iters):
    ks = ctypes.c_int()
    self._chk(lib().hgx_alg_shard_begin(self.h, row0, row1, d_partial, d_mm,
                                        iters, ctypes.byref(ks)))
    return ks.value

  def alg_shard_node(self, it):
    self._chk(lib().hgx_alg_shard_node(self.h, it))

  def alg_shard_edge_partial(self, it):
    self._chk(lib().hgx_alg_shard_edge_partial(self.h, it))

  def alg_shard_ranges(self, n):
    """Split the local edge rows into n ranges; returns the n + 1 bounds."""
    b = np.zeros(n + 1, np.int32)
    self._chk(lib().hgx_alg_shard_ranges(self.h, n, _ptr(b)))
    return b

  def alg_shard_edge_partial_range(self, it, r):
    self._chk(lib().hgx_alg_shard_edge_partial_range(self.h, it, r))

  def alg_shard_edge_final(self, it):
    self._chk(lib().hgx_alg_shard_edge_final(self.h, it))

  def alg_shard_end(self):
    self._chk(lib().hgx_alg_shard_end(self.h))

  def alg_shard_wire(self, d_wire, n_shared, edge_slot):
    es = _c(edge_slot, np.int32)
    self._keep_slot = es
    self._chk(lib().hgx_alg_shard_wire(self.h, d_wire, n_shared, _ptr(es)))

  # ---- HOBE probabilities / incidence weights ----
  def hobe_probs(self, kind, a, b):
    a = _c(a, np.int32)
    b = _c(b, np.int32)
    out = np.empty(a.size, np.float32)
    self._chk(lib().hgx_hobe_probs(self.h, kind, a.size, _ptr(a), _ptr(b),
                                   _ptr(out)))
    return out

  def incidence_weights(self, which, alpha=0.0):
    n = np.empty(self.inc.nnz, np.float32)
    e = np.empty(self.inc.nnz, np.float32)
    self._chk(lib().hgx_incidence_weights(self.h, which, alpha, _ptr(n),
                                          _ptr(e)))
    return n, e

  # hg2v_weighting distance / span weights (vectors = the alg coordinates)
  def weight_distance(self, norm=NORM_L2, alpha=0.0):
    """WeightByDistance values per incidence, A and A^T CSR order."""
    n = np.empty(self.inc.nnz, np.float32)
    e = np.empty(self.inc.nnz, np.float32)
    self._chk(lib().hgx_weight_distance(self.h, norm, float(alpha), _ptr(n),
                                        _ptr(e)))
    return n, e

  def weight_same_type(self, side, norm=NORM_L2, alpha=0.0):
    """WeightBySameTypeDistance CSR (rowptr int64, col int32, val float32)
    of the node (side 0) or edge (side 1) pattern, compressed ids."""
    R = self.inc.N if side == 0 else self.inc.E
    nnz = ctypes.c_int64()
    rp = np.empty(R + 1, np.int64)
    self._chk(lib().hgx_weight_same_type(self.h, side, norm, float(alpha),
                                         ctypes.byref(nnz), _ptr(rp), None, None))
    col = np.empty(nnz.value, np.int32)
    val = np.empty(nnz.value, np.float32)
    self._chk(lib().hgx_weight_same_type(self.h, side, norm, float(alpha),
                                         ctypes.byref(nnz), _ptr(rp), _ptr(col),
                                         _ptr(val)))
    return rp, col, val

  def weight_span(self, alpha=0.0):
    """(node spans, edge spans) float32 and the span weights per incidence
    (A and A^T CSR order)."""
    sn = np.empty(self.inc.N, np.float32)
    se = np.empty(self.inc.E, np.float32)
    n = np.empty(self.inc.nnz, np.float32)
    e = np.empty(self.inc.nnz, np.float32)
    self._chk(lib().hgx_weight_span(self.h, float(alpha), _ptr(sn), _ptr(se),
                                    _ptr(n), _ptr(e)))
    return sn, se, n, e

  def probe_gather(self, table_bytes, row_floats=16, in_flight=8, reps=3):
    """Random-row gather rate (rows/s) of the device (hgx_probe_gather)."""
    v = ctypes.c_double()
    self._chk(lib().hgx_probe_gather(self.h, int(table_bytes), row_floats,
                                     in_flight, reps, ctypes.byref(v)))
    return v.value

  # ---- samplers / records ----
  def sample_fobe(self, seed, K, node_q, edge_q, neg_node_q=None,
                  neg_edge_q=None):
    nq, eq = _c(node_q, np.int32), _c(edge_q, np.int32)
    nnq, neq = _c(neg_node_q, np.int32), _c(neg_edge_q, np.int32)
    n = ctypes.c_int64()
    self._chk(lib().hgx_sample_fobe(self.h, seed & (2**64 - 1), K, _ptr(nq),
                                    _ptr(eq), _ptr(nnq), _ptr(neq),
                                    ctypes.byref(n)))
    return n.value

  def sample_hobe(self, seed, K, S, node_q=None, edge_q=None):
    """AlgebraicDistanceSamples on the device; with node_q / edge_q only
    those rows (quota per row instead of S)."""
    n = ctypes.c_int64()
    if node_q is None and edge_q is None:
      self._chk(lib().hgx_sample_hobe(self.h, seed & (2**64 - 1), K, S,
                                      ctypes.byref(n)))
    else:
      nq, eq = _c(node_q, np.int32), _c(edge_q, np.int32)
      assert nq.size == self.inc.N and eq.size == self.inc.E
      self._chk(lib().hgx_sample_hobe_rows(self.h, seed & (2**64 - 1), K,
                                           _ptr(nq), _ptr(eq), S,
                                           ctypes.byref(n)))
    return n.value

  def _mt_call(self, fn, *args):
    """Run a numpy-seeded sampler on numpy's global RandomState: its MT19937
    state goes in, the state the reference leaves behind comes back."""
    st = np.random.get_state()
    if st[0] != "MT19937":
      raise ValueError("numpy's global RandomState is not MT19937")
    key = np.array(st[1], dtype=np.uint32, copy=True)
    pos = ctypes.c_int(int(st[2]))
    n = ctypes.c_int64()
    self._chk(fn(self.h, _ptr(key), ctypes.byref(pos), *args, ctypes.byref(n)))
    np.random.set_state((st[0], key, pos.value, st[3], st[4]))
    return n.value

  def sample_fobe_mt(self, K, node_q, edge_q, neg_node_q=None, neg_edge_q=None):
    """BooleanSamples drawing from numpy's global RandomState (the
    reference's stream bit for bit; hgx_sample_fobe_mt)."""
    nq, eq = _c(node_q, np.int32), _c(edge_q, np.int32)
    nnq, neq = _c(neg_node_q, np.int32), _c(neg_edge_q, np.int32)
    for q, n in ((nq, self.inc.N), (eq, self.inc.E), (nnq, self.inc.N),
                 (neq, self.inc.E)):
      assert q is None or q.size == n, "one quota per row"
    return self._mt_call(lib().hgx_sample_fobe_mt, K, _ptr(nq), _ptr(eq),
                         _ptr(nnq), _ptr(neq))

  def sample_hobe_mt(self, K, S):
    """AlgebraicDistanceSamples(run_in_parallel=False) drawing from numpy's
    global RandomState (hgx_sample_hobe_mt)."""
    return self._mt_call(lib().hgx_sample_hobe_mt, K, S)

  def sample_jaccard_mt(self, K, node_q, edge_q):
    """WeightedJaccardSamples(run_in_parallel=False) drawing from numpy's
    global RandomState (hgx_sample_jaccard_mt; features_set first)."""
    nq, eq = _c(node_q, np.int32), _c(edge_q, np.int32)
    assert nq.size == self.inc.N and eq.size == self.inc.E
    return self._mt_call(lib().hgx_sample_jaccard_mt, K, _ptr(nq), _ptr(eq))

  # weighted-Jaccard samplers
  def features_set(self, node_major, edge_major):
    fn, fe = _c(node_major, np.float32), _c(edge_major, np.float32)
    assert fn.size == self.inc.nnz and fe.size == self.inc.nnz
    self._chk(lib().hgx_features_set(self.h, _ptr(fn), _ptr(fe)))

  def sample_jaccard(self, seed, K, node_q, edge_q):
    nq, eq = _c(node_q, np.int32), _c(edge_q, np.int32)
    n = ctypes.c_int64()
    self._chk(lib().hgx_sample_jaccard(self.h, seed & (2**64 - 1), K, _ptr(nq),
                                       _ptr(eq), ctypes.byref(n)))
    return n.value

  def jaccard_probs(self, kind, a, b):
    a, b = _c(a, np.int32), _c(b, np.int32)
    out = np.empty(a.size, np.float32)
    self._chk(lib().hgx_jaccard_probs(self.h, kind, a.size, _ptr(a), _ptr(b),
                                      _ptr(out)))
    return out

  def jaccard_centroids(self, which):
    """(p int64, j int32, v float32) of the node (0) / edge (1) centroids."""
    R = self.inc.N if which == 0 else self.inc.E
    nnz = ctypes.c_int64()
    self._chk(lib().hgx_jaccard_centroids(self.h, which, ctypes.byref(nnz),
                                          None, None, None))
    p = np.empty(R + 1, np.int64)
    j = np.empty(nnz.value, np.int32)
    v = np.empty(nnz.value, np.float32)
    self._chk(lib().hgx_jaccard_centroids(self.h, which, ctypes.byref(nnz),
                                          _ptr(p), _ptr(j), _ptr(v)))
    return p, j, v

  def sample_stats(self):
    """(rows sampled by rejection, fallbacks to expansion) of the last call."""
    u, f = ctypes.c_int64(), ctypes.c_int64()
    self._chk(lib().hgx_sample_last_stats(self.h, ctypes.byref(u),
                                          ctypes.byref(f)))
    return u.value, f.value

  def sample_uniform_rows(self):
    """3-hop rows of the last call sampled by uniform-column rejection."""
    u = ctypes.c_int64()
    self._chk(lib().hgx_sample_uniform_rows(self.h, ctypes.byref(u)))
    return u.value

  def records_set(self, idx, tgt):
    idx = _c(idx, np.int32)
    tgt = _c(tgt, np.float32)
    n, R = idx.shape
    assert R % 2 == 0 and R >= 4 and tgt.shape == (n, 3)
    self._chk(lib().hgx_records_set(self.h, n, (R - 4) // 2, _ptr(idx),
                                    _ptr(tgt)))

  def records_copy_from(self, other):
    """This context's records := `other`'s (device to device, same GPU)."""
    self._chk(lib().hgx_records_copy(self.h, other.h))

  def records_info(self):
    n, K = ctypes.c_int64(), ctypes.c_int()
    self._chk(lib().hgx_records_info(self.h, ctypes.byref(n), ctypes.byref(K)))
    return n.value, K.value

  def records_blocks(self):
    """Kind-block bounds of the record stream (nblocks + 1 int64)."""
    nb = ctypes.c_int()
    b = np.zeros(17, np.int64)
    self._chk(lib().hgx_records_blocks(self.h, ctypes.byref(nb), _ptr(b)))
    return b[:nb.value + 1].copy()

  def records_export(self, d_idx, d_tgt):
    """Copy the records into caller device buffers (data pointers)."""
    self._chk(lib().hgx_records_export(self.h, d_idx, d_tgt))

  def records_import(self, n, K, d_idx, d_tgt, bounds=None):
    """Set the records from caller device buffers (data pointers)."""
    b = None if bounds is None else _c(bounds, np.int64)
    nb = 0 if b is None else b.size - 1
    self._chk(lib().hgx_records_import(self.h, n, K, d_idx, d_tgt, nb, _ptr(b)))

  def records_get(self):
    n, K = self.records_info()
    idx = np.empty((n, 4 + 2 * K), np.int32)
    tgt = np.empty((n, 3), np.float32)
    self._chk(lib().hgx_records_get(self.h, _ptr(idx), _ptr(tgt)))
    return idx, tgt

  # ---- compact record store (streams larger than HBM, hgx_store_*) ----
  def store_reset(self, capacity=0):
    self._chk(lib().hgx_store_reset(self.h, int(capacity)))

  def store_release(self):
    """Free the store, its load scratch and the loaded records."""
    self._chk(lib().hgx_store_release(self.h))

  def store_append(self):
    """Pack the records of the last sample_fobe / sample_hobe call."""
    self._chk(lib().hgx_store_append(self.h))

  def store_info(self):
    """(records, family, K, seed) of the store."""
    n, fam, K = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
    seed = ctypes.c_uint64()
    self._chk(lib().hgx_store_info(self.h, ctypes.byref(n), ctypes.byref(fam),
                                   ctypes.byref(K), ctypes.byref(seed)))
    return n.value, fam.value, K.value, seed.value

  def store_read(self, start=0, n=None, dst_ptr=None):
    """Entries [start, start + n) as an (n, 3) uint32 host array, or into
    the device buffer at dst_ptr."""
    if n is None:
      n = self.store_info()[0] - start
    if dst_ptr is not None:
      self._chk(lib().hgx_store_read(self.h, start, n, dst_ptr, 1))
      return None
    out = np.empty((n, 3), np.uint32)
    self._chk(lib().hgx_store_read(self.h, start, n, _ptr(out), 0))
    return out

  def store_write(self, entries, family, K, seed, n=None, src_ptr=None):
    """Append raw entries ((n, 3) uint32 host array, or n at device src_ptr)
    packed by a sampler of `family` / K / seed (another rank's store)."""
    if src_ptr is None:
      e = _c(entries, np.uint32).reshape(-1, 3)
      self._chk(lib().hgx_store_write(self.h, e.shape[0], _ptr(e), 0, family, K,
                                      seed & (2**64 - 1)))
    else:
      self._chk(lib().hgx_store_write(self.h, int(n), src_ptr, 1, family, K,
                                      seed & (2**64 - 1)))

  def store_plan(self, epoch_seed, budget):
    """The epoch's chunks: (bin bounds, record counts)."""
    nc = ctypes.c_int()
    b = np.zeros(STORE_BINS + 1, np.int32)
    c = np.zeros(STORE_BINS + 1, np.int64)
    self._chk(lib().hgx_store_plan(self.h, epoch_seed & (2**64 - 1), int(budget),
                                   ctypes.byref(nc), _ptr(b), _ptr(c)))
    return b[:nc.value + 1].copy(), c[:nc.value].copy()

  def store_load(self, epoch_seed, bin_lo, bin_hi, batch, last):
    """One chunk of the epoch as the record stream (trained in order);
    returns the records to train."""
    n = ctypes.c_int64()
    self._chk(lib().hgx_store_load(self.h, epoch_seed & (2**64 - 1), int(bin_lo),
                                   int(bin_hi), int(batch), 1 if last else 0,
                                   ctypes.byref(n)))
    return n.value

  # ---- model / trainer ----
  def model_init(self, d, node_rows, edge_rows, seed=0, node_tab=None,
                 edge_tab=None):
    nt, et = _c(node_tab, np.float32), _c(edge_tab, np.float32)
    if nt is not None:
      assert nt.shape == (node_rows, d) and et.shape == (edge_rows, d)
    self.d, self.node_rows, self.edge_rows = d, node_rows, edge_rows
    self._chk(lib().hgx_model_init(self.h, d, node_rows, edge_rows,
                                   seed & (2**64 - 1), _ptr(nt), _ptr(et)))

  def model_get(self):
    nt = np.empty((self.node_rows, self.d), np.float32)
    et = np.empty((self.edge_rows, self.d), np.float32)
    self._chk(lib().hgx_model_get(self.h, _ptr(nt), _ptr(et)))
    return nt, et

  def model_get_rows(self, table, rows):
    """Rows of the node (0) or edge (1) table, (len(rows), d) float32."""
    r = _c(rows, np.int64).ravel()
    out = np.empty((r.size, self.d), np.float32)
    self._chk(lib().hgx_model_get_rows(self.h, table, r.size, _ptr(r), _ptr(out)))
    return out

  def train(self, batch=256, max_epochs=10, lr=0.01, eps=1e-7, loss=LOSS_MSE,
            act=ACT_RELU, min_delta=1e-3, shuffle_seed=0, perms=None):
    pp = None
    if perms is not None:
      pp = _c(perms, np.int64)
      max_epochs = min(max_epochs, pp.shape[0])
    losses = np.zeros(max(max_epochs, 1), np.float32)
    ran = ctypes.c_int()
    self._chk(lib().hgx_train(self.h, batch, max_epochs, lr, eps, loss, act,
                              min_delta, shuffle_seed & (2**64 - 1), _ptr(pp),
                              _ptr(losses), ctypes.byref(ran)))
    return losses[:ran.value].copy()

  def train_stats(self):
    ms, rec, bat = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
    self._chk(lib().hgx_train_last_stats(self.h, ctypes.byref(ms),
                                         ctypes.byref(rec), ctypes.byref(bat)))
    return ms.value, rec.value, bat.value

  def train_loss_sum(self):
    """Sum of the per-record losses of the last trained epoch (double)."""
    v = ctypes.c_double()
    self._chk(lib().hgx_train_last_loss(self.h, ctypes.byref(v)))
    return v.value

  def train_path_stats(self):
    """(fused, split) batch counts of the last train() call."""
    f, sp = ctypes.c_int64(), ctypes.c_int64()
    self._chk(lib().hgx_train_path_stats(self.h, ctypes.byref(f),
                                         ctypes.byref(sp)))
    return f.value, sp.value

  def train_multi_pending(self):
    """Step batches of the last train() in the MULTI pending-slot form."""
    v = ctypes.c_int64()
    self._chk(lib().hgx_train_multi_pending(self.h, ctypes.byref(v)))
    return v.value


class Mlp:
  """One hgx_mlp engine (include/hgx.h, dense MLP section) on a Context."""

  def __init__(self, ctx, kind, in_dim, out_dim=0):
    self.ctx, self.kind, self.in_dim, self.out_dim = ctx, kind, in_dim, out_dim
    h = _vp()
    ctx._chk(lib().hgx_mlp_create(ctx.h, kind, in_dim, out_dim, ctypes.byref(h)))
    self.h = h
    ctx._engines.add(self)
    n = ctypes.c_int()
    ctx._chk(lib().hgx_mlp_layers(self.h, ctypes.byref(n), None))
    sh = np.empty((n.value, 2), np.int32)
    ctx._chk(lib().hgx_mlp_layers(self.h, ctypes.byref(n), _ptr(sh)))
    self.shapes = [tuple(int(v) for v in r) for r in sh]

  def close(self):
    if getattr(self, "h", None):
      lib().hgx_mlp_destroy(self.h)
      self.h = None

  def __del__(self):
    try:
      self.close()
    except Exception:
      pass

  def num_weights(self):
    return sum(k * n + n for k, n in self.shapes)

  def set_weights(self, flat):
    flat = _c(flat, np.float32)
    assert flat.size == self.num_weights()
    self.ctx._chk(lib().hgx_mlp_set_weights(self.h, _ptr(flat)))

  def get_weights(self):
    flat = np.empty(self.num_weights(), np.float32)
    self.ctx._chk(lib().hgx_mlp_get_weights(self.h, _ptr(flat)))
    return flat

  def set_tables(self, node_tab, edge_tab):
    nt, et = _c(node_tab, np.float32), _c(edge_tab, np.float32)
    assert nt.ndim == 2 and et.ndim == 2
    assert nt.shape[1] == self.in_dim and et.shape[1] == self.in_dim
    self.ctx._chk(lib().hgx_mlp_set_tables(self.h, nt.shape[0], _ptr(nt),
                                           et.shape[0], _ptr(et)))

  def set_samples(self, node_row, edge_row, label):
    nr, er = _c(node_row, np.int32), _c(edge_row, np.int32)
    lab = _c(label, np.float32)
    assert nr.shape == er.shape == lab.shape
    self.ctx._chk(lib().hgx_mlp_set_samples(self.h, nr.size, _ptr(nr), _ptr(er),
                                            _ptr(lab)))

  def fit(self, batch=256, max_epochs=1, lr=0.01, eps=1e-7, min_delta=0.0,
          seed=0, perms=None):
    pp = None
    if perms is not None:
      pp = _c(perms, np.int64)
      max_epochs = min(max_epochs, pp.shape[0])
    losses = np.zeros(max(max_epochs, 1), np.float32)
    ran = ctypes.c_int()
    self.ctx._chk(lib().hgx_mlp_fit(self.h, batch, max_epochs, lr, eps,
                                    min_delta, seed & (2**64 - 1), _ptr(pp),
                                    _ptr(losses), ctypes.byref(ran)))
    return losses[:ran.value].copy()

  def predict(self, output, node_row=None, edge_row=None):
    nr, er = _c(node_row, np.int32), _c(edge_row, np.int32)
    n = (nr if nr is not None else er).size
    shape = (n,) if output == 0 else (n, self.out_dim)
    out = np.empty(shape, np.float32)
    self.ctx._chk(lib().hgx_mlp_predict(self.h, output, n, _ptr(nr), _ptr(er),
                                        _ptr(out)))
    return out

  def stats(self):
    ms, fl = ctypes.c_double(), ctypes.c_double()
    sm, bt = ctypes.c_int64(), ctypes.c_int64()
    self.ctx._chk(lib().hgx_mlp_last_stats(self.h, ctypes.byref(ms),
                                           ctypes.byref(sm), ctypes.byref(bt),
                                           ctypes.byref(fl)))
    return {"ms": ms.value, "samples": sm.value, "batches": bt.value,
            "flops": fl.value}


# ---- host utilities (no context, no device) --------------------------------
def synth_powerlaw(N, E, mean_degree=20.0, exponent=0.8, seed=0):
  """(rp_n, col_n, E_kept) of hgx_synth_powerlaw."""
  rp = np.zeros(N + 1, np.int32)
  nnz = ctypes.c_int64()
  rc = lib().hgx_synth_powerlaw(N, E, mean_degree, exponent, seed, _ptr(rp),
                                None, ctypes.byref(nnz), None)
  if rc != HGX_OK:
    _raise(rc, "hgx_synth_powerlaw failed")
  col = np.empty(nnz.value, np.int32)
  e_out = ctypes.c_int32()
  rc = lib().hgx_synth_powerlaw(N, E, mean_degree, exponent, seed, _ptr(rp),
                                _ptr(col), ctypes.byref(nnz),
                                ctypes.byref(e_out))
  if rc != HGX_OK:
    _raise(rc, "hgx_synth_powerlaw failed")
  return rp, col, int(e_out.value)


def csr_transpose(nrow, ncol, rp, col):
  rp = _c(rp, np.int32)
  col = _c(col, np.int32)
  rpt = np.empty(ncol + 1, np.int32)
  colt = np.empty(col.size, np.int32)
  rc = lib().hgx_csr_transpose(nrow, ncol, _ptr(rp), _ptr(col), _ptr(rpt),
                               _ptr(colt))
  if rc != HGX_OK:
    _raise(rc, "hgx_csr_transpose: column index out of range")
  return rpt, colt


def _host_raise(rc):
  _raise(rc, lib().hgx_host_last_error().decode(errors="replace"))


def parse_hypergraph(buf):
  """Serialized Hypergraph bytes (bytes / memoryview / uint8 array) ->
  dict of compressed-incidence arrays (hgx_proto_parse_hypergraph)."""
  a = np.frombuffer(buf, dtype=np.uint8)
  h = _vp()
  n, e, nnz = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
  rc = lib().hgx_proto_parse_hypergraph(_ptr(a) if a.size else None, a.size,
                                        ctypes.byref(h), ctypes.byref(n),
                                        ctypes.byref(e), ctypes.byref(nnz))
  if rc != HGX_OK:
    _host_raise(rc)
  try:
    out = {"N": n.value, "E": e.value,
           "rp_n": np.empty(n.value + 1, np.int32),
           "col_n": np.empty(nnz.value, np.int32),
           "node_ids": np.empty(n.value, np.int64),
           "edge_ids": np.empty(e.value, np.int64),
           "node_weight": np.empty(n.value, np.float32),
           "edge_weight": np.empty(e.value, np.float32)}
    rc = lib().hgx_proto_hypergraph_fill(
        h, _ptr(out["rp_n"]), _ptr(out["col_n"]), _ptr(out["node_ids"]),
        _ptr(out["edge_ids"]), _ptr(out["node_weight"]),
        _ptr(out["edge_weight"]))
    if rc != HGX_OK:
      _host_raise(rc)
  finally:
    lib().hgx_proto_hypergraph_free(h)
  return out


def write_embedding_bytes(node_ids, node_tab, edge_ids, edge_tab, method_name):
  """HypergraphEmbedding wire bytes (hgx_proto_write_embedding)."""
  node_ids = _c(node_ids, np.int64)
  edge_ids = _c(edge_ids, np.int64)
  node_tab = _c(node_tab, np.float32)
  edge_tab = _c(edge_tab, np.float32)
  d = int(node_tab.shape[1]) if node_tab.ndim == 2 else int(edge_tab.shape[1])
  assert node_tab.shape == (node_ids.size, d) and edge_tab.shape == (edge_ids.size, d)
  name = None if method_name is None else method_name.encode()
  ln = ctypes.c_int64()
  args = (node_ids.size, _ptr(node_ids), _ptr(node_tab), edge_ids.size,
          _ptr(edge_ids), _ptr(edge_tab), d, name)
  rc = lib().hgx_proto_write_embedding(*args, None, 0, ctypes.byref(ln))
  if rc != HGX_OK:
    _host_raise(rc)
  out = np.empty(ln.value, np.uint8)
  rc = lib().hgx_proto_write_embedding(*args, _ptr(out), out.size,
                                       ctypes.byref(ln))
  if rc != HGX_OK:
    _host_raise(rc)
  return out


def parse_embedding(buf):
  """Serialized HypergraphEmbedding bytes (one message or concatenated
  shards; bytes / memoryview / uint8 array / mmap) -> dict(node_ids,
  node_tab, edge_ids, edge_tab, dim, width, method_name)
  (hgx_proto_parse_embedding)."""
  a = np.frombuffer(buf, dtype=np.uint8)
  h = _vp()
  nn, ne, w = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
  dim = ctypes.c_int32()
  rc = lib().hgx_proto_parse_embedding(_ptr(a) if a.size else None, a.size,
                                       ctypes.byref(h), ctypes.byref(nn),
                                       ctypes.byref(ne), ctypes.byref(w),
                                       ctypes.byref(dim))
  if rc != HGX_OK:
    _host_raise(rc)
  try:
    W = w.value
    out = {"node_ids": np.empty(nn.value, np.int64),
           "node_tab": np.empty((nn.value, W), np.float32),
           "edge_ids": np.empty(ne.value, np.int64),
           "edge_tab": np.empty((ne.value, W), np.float32),
           "dim": dim.value, "width": W}
    mlen = lib().hgx_proto_embedding_method_len(h)
    name = ctypes.create_string_buffer(mlen + 1)
    rc = lib().hgx_proto_embedding_fill(
        h, _ptr(out["node_ids"]), _ptr(out["node_tab"]), _ptr(out["edge_ids"]),
        _ptr(out["edge_tab"]), name, mlen + 1)
    if rc != HGX_OK:
      _host_raise(rc)
    out["method_name"] = name.value.decode()
  finally:
    lib().hgx_proto_embedding_free(h)
  return out


def write_hypergraph_bytes(inc):
  """Hypergraph wire bytes of an Incidence (hgx_proto_write_hypergraph)."""
  ids = (_c(inc.node_ids, np.int64), _c(inc.edge_ids, np.int64))
  args = (inc.N, inc.E, _ptr(inc.rp_n), _ptr(inc.col_n), _ptr(inc.rp_e),
          _ptr(inc.col_e), _ptr(ids[0]), _ptr(ids[1]))
  ln = ctypes.c_int64()
  rc = lib().hgx_proto_write_hypergraph(*args, None, 0, ctypes.byref(ln))
  if rc != HGX_OK:
    _host_raise(rc)
  out = np.empty(ln.value, np.uint8)
  rc = lib().hgx_proto_write_hypergraph(*args, _ptr(out), out.size,
                                        ctypes.byref(ln))
  if rc != HGX_OK:
    _host_raise(rc)
  return out


# ---- Python-`random`-compatible link-prediction loops (host) ---------------
def _mt_state(rnd):
  ver, st, gauss = rnd.getstate()
  return np.array(st, np.uint32), (ver, gauss)


def _mt_restore(rnd, arr, meta):
  rnd.setstate((meta[0], tuple(int(v) for v in arr), meta[1]))


def _lp_chk(rc):
  if rc != HGX_OK:
    _raise(rc, lib().hgx_lp_last_error().decode())


def pyrandom_sample_missing(rnd, n_nodes, n_edges, rowptr, col, num_samples):
  """(node positions, edge positions) drawn as SampleMissingConnections
  draws them with the `random.Random` instance `rnd` (advanced)."""
  st, meta = _mt_state(rnd)
  rp = _c(rowptr, np.int64)
  cl = _c(col, np.int32)
  npos = np.empty(max(num_samples, 1), np.int32)
  epos = np.empty(max(num_samples, 1), np.int32)
  got = ctypes.c_int64()
  _lp_chk(lib().hgx_pyrandom_sample_missing(
      _ptr(st), n_nodes, n_edges, _ptr(rp), _ptr(cl), num_samples, _ptr(npos),
      _ptr(epos), ctypes.byref(got)))
  _mt_restore(rnd, st, meta)
  return npos[:got.value].copy(), epos[:got.value].copy()


def pyrandom_remove_connections(rnd, pair_node, pair_edge, node_deg,
                                edge_size, probability):
  """Indices of the pairs RemoveRandomConnections removes, in order."""
  st, meta = _mt_state(rnd)
  pn, pe = _c(pair_node, np.int32), _c(pair_edge, np.int32)
  nd = np.array(node_deg, np.int32)
  es = np.array(edge_size, np.int32)
  out = np.empty(max(pn.size, 1), np.int64)
  got = ctypes.c_int64()
  _lp_chk(lib().hgx_pyrandom_remove_connections(
      _ptr(st), pn.size, _ptr(pn), _ptr(pe), _ptr(nd), _ptr(es),
      float(probability), _ptr(out), ctypes.byref(got)))
  _mt_restore(rnd, st, meta)
  return out[:got.value].copy()
