// Context lifetime, errors, incidence upload. See include/hgx.h.
#include <algorithm>
#include <cstring>
#include <vector>

#include "hgx_internal.h"

int hgx_fail(hgx_ctx *ctx, int code, const char *fmt, ...) {
  if (ctx) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    ctx->err = buf;
  }
  return code;
}

int hgx_ensure(hgx_ctx *ctx, DevBuf &b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return HGX_OK;
  if (b.p) {
    hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) {
    b.p = nullptr;
    (void)hipGetLastError();
    return hgx_fail(ctx, HGX_ENOMEM, "hipMalloc(%zu bytes) failed: %s", bytes,
                    hipGetErrorString(e));
  }
  b.bytes = bytes;
  return HGX_OK;
}

void hgx_release(DevBuf &b) {
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

extern "C" int hgx_version(void) { return 1; }

extern "C" int hgx_create(int device, hgx_ctx **out) {
  if (!out) return HGX_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return HGX_EHIP;
  }
  if (device < 0 || device >= n) return HGX_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return HGX_EHIP;
  hgx_ctx *ctx = new hgx_ctx();
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) !=
      hipSuccess) {
    delete ctx;
    return HGX_EHIP;
  }
  ctx->stream = ctx->own_stream;
  hipEventCreate(&ctx->ev0);
  hipEventCreate(&ctx->ev1);
  *out = ctx;
  return HGX_OK;
}

extern "C" int hgx_destroy(hgx_ctx *ctx) {
  if (!ctx) return HGX_OK;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  DevBuf *bufs[] = {&ctx->rp_n, &ctx->col_n, &ctx->rp_e, &ctx->col_e,
                    &ctx->X[0], &ctx->X[1], &ctx->Y[0], &ctx->Y[1], &ctx->mm,
                    &ctx->rp_el, &ctx->col_el, &ctx->blk_n, &ctx->blk_e,
                    &ctx->blk_sn, &ctx->blk_el,
                    &ctx->rec_idx, &ctx->rec_tgt, &ctx->ntab, &ctx->etab,
                    &ctx->nacc, &ctx->eacc, &ctx->s0, &ctx->s1, &ctx->s2,
                    &ctx->s3, &ctx->s4, &ctx->s5, &ctx->s6, &ctx->s7,
                    &ctx->feat_n, &ctx->feat_e, &ctx->cn_p, &ctx->cn_j,
                    &ctx->cn_v, &ctx->ce_p, &ctx->ce_j, &ctx->ce_v,
                    &ctx->hw_n, &ctx->hw_e, &ctx->hw_self, &ctx->bloom_off, &ctx->bloom_bits, &ctx->store,
                    &ctx->st_sel, &ctx->st_keys, &ctx->st_vals, &ctx->st_tmp,
                    &ctx->st_hist};
  for (DevBuf *b : bufs) hgx_release(*b);
  for (LongRows *l : {&ctx->long_n, &ctx->long_e, &ctx->long_sn, &ctx->long_el})
    for (DevBuf *b : {&l->seg, &l->off, &l->rows, &l->part}) hgx_release(*b);
  for (LongRows &l : ctx->long_elr)
    for (DevBuf *b : {&l.seg, &l.off, &l.rows, &l.part}) hgx_release(*b);
  for (hipStream_t &s : ctx->tstream)
    if (s) hipStreamDestroy(s);
  if (ctx->ev0) hipEventDestroy(ctx->ev0);
  if (ctx->ev1) hipEventDestroy(ctx->ev1);
  if (ctx->own_stream) hipStreamDestroy(ctx->own_stream);
  delete ctx;
  return HGX_OK;
}

extern "C" const char *hgx_last_error(const hgx_ctx *ctx) {
  return ctx ? ctx->err.c_str() : "null context";
}

extern "C" int hgx_set_stream(hgx_ctx *ctx, void *hip_stream) {
  if (!ctx) return HGX_EINVAL;
  ctx->stream = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
  return HGX_OK;
}

extern "C" int hgx_set_tuning(hgx_ctx *ctx, const char *key, int64_t value) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, key, HGX_EINVAL, "null tuning key");
  const std::string k(key);
  Tuning &t = ctx->tune;
  if (k == "sample_reject_w") {
    HGX_CHECK(ctx, value >= 0, HGX_EINVAL, "sample_reject_w must be >= 0");
    t.sample_reject_w = value;
  } else if (k == "sample_mode3_shift_e") {
    HGX_CHECK(ctx, value >= -10 && value <= 10, HGX_EINVAL,
              "sample_mode3_shift_e must be in [-10, 10]");
    t.sample_mode3_shift_e = (int)value;
  } else if (k == "sample_mode3_shift") {
    HGX_CHECK(ctx, value >= -10 && value <= 10, HGX_EINVAL,
              "sample_mode3_shift must be in [-10, 10]");
    t.sample_mode3_shift = (int)value;
  } else if (k == "sample_mode3") {
    HGX_CHECK(ctx, value >= 0 && value <= 2, HGX_EINVAL, "sample_mode3 must be 0, 1 or 2");
    t.sample_mode3 = (int)value;
  } else if (k == "train_fused") {
    HGX_CHECK(ctx, value == 0 || value == 1, HGX_EINVAL, "train_fused must be 0 or 1");
    t.train_fused = (int)value;
  } else if (k == "train_lanes") {
    HGX_CHECK(ctx, value == 0 || value == 32 || value == 64, HGX_EINVAL,
              "train_lanes must be 0, 32 or 64");
    t.train_lanes = (int)value;
  } else if (k == "train_tb") {
    HGX_CHECK(ctx, value == 0 || value == 128 || value == 256 || value == 512, HGX_EINVAL,
              "train_tb must be 0, 128, 256 or 512");
    t.train_tb = (int)value;
  } else if (k == "alg_long") {
    HGX_CHECK(ctx, value == 0 || (value >= 64 && value <= (1 << 20)), HGX_EINVAL,
              "alg_long must be 0 or in [64, 2^20]");
    t.alg_long = (int)value;
  } else if (k == "alg_push") {
    HGX_CHECK(ctx, value == 0 || value == 1, HGX_EINVAL, "alg_push must be 0 or 1");
    t.alg_push = (int)value;
  } else if (k == "mlp_fuse_head") {
    HGX_CHECK(ctx, value == 0 || value == 1, HGX_EINVAL, "mlp_fuse_head must be 0 or 1");
    t.mlp_fuse_head = (int)value;
  } else if (k == "mlp_prefetch") {
    HGX_CHECK(ctx, value >= 0 && value <= 2, HGX_EINVAL, "mlp_prefetch must be 0, 1 or 2");
    t.mlp_prefetch = (int)value;
  } else if (k == "mlp_wgrad_split") {
    HGX_CHECK(ctx, value >= 0 && value <= 1, HGX_EINVAL, "mlp_wgrad_split must be 0 or 1");
    t.mlp_wgrad_split = (int)value;
  } else if (k == "train_prep_overlap") {
    HGX_CHECK(ctx, value >= 0 && value <= 2, HGX_EINVAL, "train_prep_overlap must be 0, 1 or 2");
    t.train_prep_overlap = (int)value;
  } else if (k == "train_prep_cus") {
    HGX_CHECK(ctx, value >= 0 && value <= 128, HGX_EINVAL, "train_prep_cus must be in [0, 128]");
    t.train_prep_cus = (int)value;
  } else if (k == "alg_ks") {
    HGX_CHECK(ctx, value == 0 || (value % 4 == 0 && value <= 20), HGX_EINVAL,
              "alg_ks must be 0 or a multiple of 4 <= 20");
    t.alg_ks = (int)value;
  } else if (k == "stream_cus") {
    // The context's own stream on a CU subset: v > 0 the first
    // round_up(v, 8) CU-mask bits, v < 0 every bit but those of |v|, 0 all.
    // Mask bit i = CU i / 8 of XCD i % 8 (tools/cumask_probe.hip), so a
    // multiple of 8 bits is the same CU count on every XCD. Two contexts on
    // one device with +v / -v run concurrent work (e.g. the sampler of
    // chunk c + 1 beside the trainer of chunk c) on disjoint CUs.
    int ncu = 0;
    HGX_HIP(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount,
                                       ctx->device));
    const int nb = (int)((std::abs(value) + 7) / 8 * 8);
    HGX_CHECK(ctx, value == 0 || (nb > 0 && nb < ncu), HGX_EINVAL,
              "stream_cus must be 0 or in (-%d, %d)", ncu, ncu);
    HGX_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t ns = nullptr;
    if (value == 0) {
      HGX_HIP(ctx, hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
    } else {
      const int W = (ncu + 31) / 32;
      std::vector<uint32_t> m(W, 0u);
      for (int i = 0; i < ncu; i++)
        if ((i < nb) == (value > 0)) m[i / 32] |= 1u << (i % 32);
      HGX_HIP(ctx, hipExtStreamCreateWithCUMask(&ns, W, m.data()));
    }
    HGX_HIP(ctx, hipStreamSynchronize(ctx->own_stream));
    const bool cur = ctx->stream == ctx->own_stream;
    HGX_HIP(ctx, hipStreamDestroy(ctx->own_stream));
    ctx->own_stream = ns;
    if (cur) ctx->stream = ns;
  } else {
    return hgx_fail(ctx, HGX_EINVAL, "unknown tuning key '%s'", key);
  }
  return HGX_OK;
}

extern "C" int hgx_synchronize(hgx_ctx *ctx) {
  if (!ctx) return HGX_EINVAL;
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_device_count(int *n) {
  if (!n) return HGX_EINVAL;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return HGX_OK;
}

extern "C" int hgx_mem_info(hgx_ctx *ctx, int64_t *free_bytes, int64_t *total_bytes) {
  if (!ctx) return HGX_EINVAL;
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  size_t f = 0, t = 0;
  HGX_HIP(ctx, hipMemGetInfo(&f, &t));
  if (free_bytes) *free_bytes = (int64_t)f;
  if (total_bytes) *total_bytes = (int64_t)t;
  return HGX_OK;
}

static int check_csr(hgx_ctx *ctx, const char *name, int32_t R, int32_t C,
                     int64_t nnz, const int32_t *rp, const int32_t *col) {
  HGX_CHECK(ctx, rp && (nnz == 0 || col), HGX_EINVAL, "%s: null pointer", name);
  HGX_CHECK(ctx, rp[0] == 0 && rp[R] == nnz, HGX_EINVAL,
            "%s: rowptr must start at 0 and end at nnz", name);
  for (int32_t r = 0; r < R; r++) {
    HGX_CHECK(ctx, rp[r + 1] >= rp[r], HGX_EINVAL, "%s: rowptr not monotone",
              name);
    for (int32_t t = rp[r]; t < rp[r + 1]; t++) {
      HGX_CHECK(ctx, col[t] >= 0 && col[t] < C, HGX_EINVAL,
                "%s: column %d out of range [0,%d)", name, col[t], C);
      HGX_CHECK(ctx, t == rp[r] || col[t] > col[t - 1], HGX_EINVAL,
                "%s: columns of row %d not strictly increasing", name, r);
    }
  }
  return HGX_OK;
}

extern "C" int hgx_upload_incidence(hgx_ctx *ctx, int32_t N, int32_t E,
                                    int64_t nnz, const int32_t *rowptr_n,
                                    const int32_t *col_n,
                                    const int32_t *rowptr_e,
                                    const int32_t *col_e) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, N > 0 && E > 0, HGX_EINVAL, "empty hypergraph (N=%d E=%d)",
            N, E);
  HGX_CHECK(ctx, nnz >= 0 && nnz < (int64_t)INT32_MAX, HGX_EUNSUP,
            "nnz %lld outside int32 CSR range", (long long)nnz);
  // Host-side validation: the kernels index without bounds checks, so an
  // out-of-range column must be rejected here, never reach the GPU.
  HGX_TRY(check_csr(ctx, "node-major", N, E, nnz, rowptr_n, col_n));
  HGX_TRY(check_csr(ctx, "edge-major", E, N, nnz, rowptr_e, col_e));
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, ctx->rp_n, sizeof(int32_t) * (N + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->rp_e, sizeof(int32_t) * (E + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->col_n, sizeof(int32_t) * (nnz + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->col_e, sizeof(int32_t) * (nnz + 1)));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->rp_n.p, rowptr_n, sizeof(int32_t) * (N + 1),
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->rp_e.p, rowptr_e, sizeof(int32_t) * (E + 1),
                              hipMemcpyHostToDevice, ctx->stream));
  if (nnz) {
    HGX_HIP(ctx, hipMemcpyAsync(ctx->col_n.p, col_n, sizeof(int32_t) * nnz,
                                hipMemcpyHostToDevice, ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->col_e.p, col_e, sizeof(int32_t) * nnz,
                                hipMemcpyHostToDevice, ctx->stream));
  }
  HGX_TRY(hgx_make_row_blocks(ctx, rowptr_n, 0, N, ctx->blk_n, ctx->nblk_n));
  HGX_TRY(hgx_make_row_blocks(ctx, rowptr_e, 0, E, ctx->blk_e, ctx->nblk_e));
  HGX_TRY(hgx_make_long_rows(ctx, rowptr_n, 0, N, ctx->long_n));
  HGX_TRY(hgx_make_long_rows(ctx, rowptr_e, 0, E, ctx->long_e));
  int32_t mn = 0, me = 0;
  for (int32_t r = 0; r < N; r++) mn = std::max(mn, rowptr_n[r + 1] - rowptr_n[r]);
  for (int32_t r = 0; r < E; r++) me = std::max(me, rowptr_e[r + 1] - rowptr_e[r]);
  ctx->N = N;
  ctx->E = E;
  ctx->nnz = nnz;
  ctx->max_deg_n = mn;
  ctx->max_deg_e = me;
  ctx->avg_deg_n = (double)nnz / N;
  ctx->avg_deg_e = (double)nnz / E;
  ctx->k = 0;  // alg coords belong to the previous incidence
  ctx->tpos_ok = false;
  ctx->n_rec = 0;
  ctx->smp_family = -1;
  ctx->rec_in_order = false;
  ctx->store_carry = 0;
  ctx->bloom_ok = false;  // member filters of the previous incidence
  ctx->n_store = 0;  // stored records name rows of the previous incidence
  ctx->st_hist_ok = false;
  ctx->store_family = -1;
  ctx->features_ok = ctx->centroids_ok = false;
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

int hgx_make_row_blocks(hgx_ctx *ctx, const int32_t *rp, int32_t r0, int32_t r1,
                        DevBuf &blk, int &nblk) {
  constexpr int kRows = 64, kNnz = 256;  // must match hgx_algdist.hip
  std::vector<int32_t> b;
  b.reserve((size_t)(r1 - r0) / 8 + 2);
  b.push_back(r0);
  int rows = 0;
  int64_t nz = 0;
  for (int32_t r = r0; r < r1; r++) {
    const int64_t len = rp[r + 1] - rp[r];
    if (rows > 0 && (rows + 1 > kRows || nz + len > kNnz)) {
      b.push_back(r);
      rows = 0;
      nz = 0;
    }
    rows++;
    nz += len;
  }
  if (r1 > r0) b.push_back(r1);
  nblk = (int)b.size() - 1;
  if (nblk < 0) nblk = 0;
  HGX_TRY(hgx_ensure(ctx, blk, sizeof(int32_t) * b.size()));
  HGX_HIP(ctx, hipMemcpy(blk.p, b.data(), sizeof(int32_t) * b.size(),
                         hipMemcpyHostToDevice));
  return HGX_OK;
}

int hgx_make_long_rows(hgx_ctx *ctx, const int32_t *rp, int32_t r0, int32_t r1,
                       LongRows &out) {
  const int thresh = ctx->tune.alg_long >= 64 ? ctx->tune.alg_long : kLongRow;
  std::vector<int32_t> rows, off(1, 0);
  std::vector<int32_t> seg;  // pairs {row, piece}
  for (int32_t r = r0; r < r1; r++) {
    const int64_t len = rp[r + 1] - rp[r];
    if (len <= thresh) continue;
    const int pieces = (int)((len + thresh - 1) / thresh);
    rows.push_back(r);
    for (int p = 0; p < pieces; p++) {
      seg.push_back(r);
      seg.push_back(p);
    }
    off.push_back(off.back() + pieces);
  }
  out.thresh = thresh;
  out.nlong = (int)rows.size();
  out.nseg = off.back();
  if (out.nlong == 0) return HGX_OK;
  HGX_TRY(hgx_ensure(ctx, out.rows, sizeof(int32_t) * rows.size()));
  HGX_TRY(hgx_ensure(ctx, out.off, sizeof(int32_t) * off.size()));
  HGX_TRY(hgx_ensure(ctx, out.seg, sizeof(int32_t) * seg.size()));
  HGX_HIP(ctx, hipMemcpy(out.rows.p, rows.data(), sizeof(int32_t) * rows.size(),
                         hipMemcpyHostToDevice));
  HGX_HIP(ctx, hipMemcpy(out.off.p, off.data(), sizeof(int32_t) * off.size(),
                         hipMemcpyHostToDevice));
  HGX_HIP(ctx, hipMemcpy(out.seg.p, seg.data(), sizeof(int32_t) * seg.size(),
                         hipMemcpyHostToDevice));
  return HGX_OK;
}
