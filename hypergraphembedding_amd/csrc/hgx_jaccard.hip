// Weighted-Jaccard samples on MI355X: HG2V_ADJ_JAC / HG2V_NEIGH_JAC
// (reference: hg2v_sample.py:395-510 WeightedJaccardSamples, :250-273
// SparseWeightedJaccard, :276-326 GetAllCentroids / CentroidFromRows,
// :329-392 Same/DiffTypeJaccardSample; embedding.py:330-386).
//
// Features are per-incidence values on A's pattern (node2features N x E in
// A's CSR order, edge2features E x N in A^T's), as UniformWeight /
// WeightByNeighborhood produce. Pairs come from the same device samplers as
// HOBE (A A^T, A^T A, A A^T A, A^T A A^T rows) with FOBE-style per-row
// quotas; probabilities are computed per pair with the reference's float32
// arithmetic, so for a given pair they are bit-identical to the reference:
//   nn / ee: SparseWeightedJaccard of the two feature rows,
//   ne(v, e): SWJ(node2features[v], edge centroid[e]) *
//             SWJ(edge2features[e], node centroid[v]),
// with the centroids (mean of the neighbours' feature rows, float32 sums in
// ascending neighbour order, then / count) built once per call, one
// workgroup per row.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <vector>

#include "hgx_internal.h"

namespace {

constexpr int kCB = 256;

int grid_for(int64_t work, int per_block, int cap = 4096) {
  int64_t g = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// SparseWeightedJaccard over two sorted sparse rows (float32, sequential in
// the sorted union order, num += min / den += max via the `x < y` branch).
__device__ float swj(const int *ac, const float *av, int na, const int *bc,
                     const float *bv, int nb) {
  float num = 0.0f, den = 0.0f;
  int i = 0, j = 0;
  while (i < na || j < nb) {
    float x, y;
    if (j >= nb || (i < na && ac[i] < bc[j])) {
      x = av[i++];
      y = 0.0f;
    } else if (i >= na || bc[j] < ac[i]) {
      x = 0.0f;
      y = bv[j++];
    } else {
      x = av[i++];
      y = bv[j++];
    }
    if (x < y) {
      num = __fadd_rn(num, x);
      den = __fadd_rn(den, y);
    } else {
      num = __fadd_rn(num, y);
      den = __fadd_rn(den, x);
    }
  }
  return den == 0.0f ? 0.0f : __fdiv_rn(num, den);
}

// Centroid rows (capacity layout): row r of (rp, col) averages the feature
// rows t in row r (ascending t). One workgroup per row; a dense float
// accumulator and a bitmap per workgroup; t processed one after the other
// so every column's float32 sum has the reference's order.
__global__ __launch_bounds__(kCB) void centroid_rows(
    int R, const int *__restrict__ rp, const int *__restrict__ col,
    const int *__restrict__ frp, const int *__restrict__ fcol,
    const float *__restrict__ fval, int ncols, const int64_t *__restrict__ cap_off,
    int *__restrict__ out_col, float *__restrict__ out_val,
    int *__restrict__ out_cnt, float *__restrict__ acc_g,
    unsigned *__restrict__ bm_g, int *__restrict__ row_ctr) {
  __shared__ int s_row, s_ws[kCB / 64], s_base;
  const int tid = threadIdx.x;
  const int nwords = (ncols + 31) >> 5;
  float *acc = acc_g + (size_t)blockIdx.x * ncols;
  unsigned *bm = bm_g + (size_t)blockIdx.x * nwords;
  for (;;) {
    if (tid == 0) s_row = atomicAdd(row_ctr, 1);
    __syncthreads();
    const int r = s_row;
    if (r >= R) break;
    const int b = rp[r], e = rp[r + 1];
    for (int q = b; q < e; q++) {
      const int t = col[q];
      for (int z = frp[t] + tid; z < frp[t + 1]; z += kCB) {
        const int c = fcol[z];
        acc[c] = __fadd_rn(acc[c], fval[z]);
        atomicOr(&bm[c >> 5], 1u << (c & 31));
      }
      __syncthreads();
    }
    // sorted support from the bitmap, zeros dropped (.nonzero())
    const float len = (float)(e - b);
    int *oc = out_col + cap_off[r];
    float *ov = out_val + cap_off[r];
    if (tid == 0) s_base = 0;
    __syncthreads();
    for (int w0 = 0; w0 < nwords; w0 += kCB) {
      const int w = w0 + tid;
      unsigned bits = w < nwords ? bm[w] : 0u;
      // keep only columns whose mean is nonzero
      unsigned keep = 0u;
      for (unsigned x = bits; x; x &= x - 1) {
        const int c = (w << 5) + __ffs(x) - 1;
        if (__fdiv_rn(acc[c], len) != 0.0f) keep |= 1u << (c & 31);
      }
      const int cnt = __popc(keep);
      // block exclusive scan of cnt
      const int lane = tid & 63, wave = tid >> 6;
      int inc = cnt;
      for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(inc, off);
        if (lane >= off) inc += o;
      }
      if (lane == 63) s_ws[wave] = inc;
      __syncthreads();
      int before = s_base, tot = 0;
      for (int i = 0; i < kCB / 64; i++) {
        if (i < wave) before += s_ws[i];
        tot += s_ws[i];
      }
      int pos = before + inc - cnt;
      for (unsigned x = keep; x; x &= x - 1) {
        const int c = (w << 5) + __ffs(x) - 1;
        oc[pos] = c;
        ov[pos] = __fdiv_rn(acc[c], len);
        pos++;
      }
      for (unsigned x = bits; x; x &= x - 1) acc[(w << 5) + __ffs(x) - 1] = 0.0f;
      if (w < nwords) bm[w] = 0u;
      __syncthreads();
      if (tid == 0) s_base += tot;
      __syncthreads();
    }
    if (tid == 0) out_cnt[r] = s_base;
    __syncthreads();
  }
}

// per-row capacity = number of (t, feature) paths of the row
__global__ void centroid_caps(int R, const int *__restrict__ rp,
                              const int *__restrict__ col,
                              const int *__restrict__ frp, int64_t *__restrict__ cap) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R; r += gridDim.x * blockDim.x) {
    int64_t w = 0;
    for (int q = rp[r]; q < rp[r + 1]; q++) w += frp[col[q] + 1] - frp[col[q]];
    cap[r] = w;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) cap[R] = 0;
}

__global__ void compact_rows(int R, const int64_t *__restrict__ cap_off,
                             const int64_t *__restrict__ off,
                             const int *__restrict__ cnt,
                             const int *__restrict__ in_col,
                             const float *__restrict__ in_val,
                             int *__restrict__ out_col, float *__restrict__ out_val) {
  for (int r = blockIdx.x; r < R; r += gridDim.x) {
    const int n = cnt[r];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      out_col[off[r] + i] = in_col[cap_off[r] + i];
      out_val[off[r] + i] = in_val[cap_off[r] + i];
    }
  }
}

struct JacArgs {
  const int *rp_n, *col_n, *rp_e, *col_e;
  const float *fn, *fe;
  const int64_t *cn_p, *ce_p;
  const int *cn_j, *ce_j;
  const float *cn_v, *ce_v;
};

__device__ float jac_prob(const JacArgs &J, int kind, int a, int b) {
  if (kind == 0)
    return swj(J.col_n + J.rp_n[a], J.fn + J.rp_n[a], J.rp_n[a + 1] - J.rp_n[a],
               J.col_n + J.rp_n[b], J.fn + J.rp_n[b], J.rp_n[b + 1] - J.rp_n[b]);
  if (kind == 1)
    return swj(J.col_e + J.rp_e[a], J.fe + J.rp_e[a], J.rp_e[a + 1] - J.rp_e[a],
               J.col_e + J.rp_e[b], J.fe + J.rp_e[b], J.rp_e[b + 1] - J.rp_e[b]);
  const float pn = swj(J.col_n + J.rp_n[a], J.fn + J.rp_n[a],
                       J.rp_n[a + 1] - J.rp_n[a], J.ce_j + J.ce_p[b],
                       J.ce_v + J.ce_p[b], (int)(J.ce_p[b + 1] - J.ce_p[b]));
  const float pe = swj(J.col_e + J.rp_e[b], J.fe + J.rp_e[b],
                       J.rp_e[b + 1] - J.rp_e[b], J.cn_j + J.cn_p[a],
                       J.cn_v + J.cn_p[a], (int)(J.cn_p[a + 1] - J.cn_p[a]));
  return __fmul_rn(pn, pe);
}

// records [b, e) of the stream: kind 0 reads (ln, rn), 1 (le, re), 2 (ln, re)
__global__ void jac_fill(JacArgs J, int kind, int64_t b, int64_t e, int R,
                         const int *__restrict__ idx, float *__restrict__ tgt) {
  for (int64_t i = b + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < e;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int *r = idx + i * R;
    int x, y;
    if (kind == 0) { x = r[0] - 1; y = r[2] - 1; }
    else if (kind == 1) { x = r[1] - 1; y = r[3] - 1; }
    else { x = r[0] - 1; y = r[3] - 1; }
    tgt[i * 3 + kind] = jac_prob(J, kind, x, y);
  }
}

__global__ void jac_pairs(JacArgs J, int kind, int64_t n, const int *__restrict__ a,
                          const int *__restrict__ b, float *__restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = jac_prob(J, kind, a[i], b[i]);
}

int scan_i64(hgx_ctx *ctx, const int64_t *in, int64_t *out, int n, int64_t *total) {
  size_t tmp = 0;
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, in, out, n + 1,
                                                ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->s2, tmp + 16));
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(ctx->s2.p, tmp, in, out, n + 1,
                                                ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(total, out + n, sizeof(int64_t),
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

struct ToI64 {
  __host__ __device__ int64_t operator()(int x) const { return x; }
};

// Centroids of rows [0, R) of (rp, col) over features (frp, fcol, fval)
// (ncols feature columns) into p (R+1, int64), j, v.
int build_centroids(hgx_ctx *ctx, int R, const int *rp, const int *col,
                    const int *frp, const int *fcol, const float *fval, int ncols,
                    DevBuf &p, DevBuf &j, DevBuf &v, int64_t &nnz) {
  DevBuf cap, cap_off, cnt, tcol, tval;
  auto cleanup = [&]() {
    for (DevBuf *b : {&cap, &cap_off, &cnt, &tcol, &tval}) hgx_release(*b);
  };
  int rc = HGX_OK;
  int64_t total = 0;
  do {
    if ((rc = hgx_ensure(ctx, cap, sizeof(int64_t) * (R + 1)))) break;
    if ((rc = hgx_ensure(ctx, cap_off, sizeof(int64_t) * (R + 1)))) break;
    hipLaunchKernelGGL(centroid_caps, dim3(grid_for(R, 256)), dim3(256), 0,
                       ctx->stream, R, rp, col, frp, cap.as<int64_t>());
    if ((rc = scan_i64(ctx, cap.as<int64_t>(), cap_off.as<int64_t>(), R, &total))) break;
    if (total >= (int64_t)INT32_MAX * 2) {
      rc = hgx_fail(ctx, HGX_EUNSUP,
                    "weighted-Jaccard centroids need %lld candidate entries "
                    "(the 2-hop expansion of this graph is too large)",
                    (long long)total);
      break;
    }
    if ((rc = hgx_ensure(ctx, tcol, sizeof(int) * (total + 1)))) break;
    if ((rc = hgx_ensure(ctx, tval, sizeof(float) * (total + 1)))) break;
    if ((rc = hgx_ensure(ctx, cnt, sizeof(int) * (R + 1)))) break;
    const int nwords = (ncols + 31) / 32;
    int nwg = 1024;
    while (nwg > 32 && (double)nwg * ((double)ncols * 4 + nwords * 4) > 2e9) nwg /= 2;
    if ((rc = hgx_ensure(ctx, ctx->s3, sizeof(float) * (size_t)nwg * ncols + 16))) break;
    if ((rc = hgx_ensure(ctx, ctx->s4, sizeof(unsigned) * (size_t)nwg * nwords + 16))) break;
    if ((rc = hgx_ensure(ctx, ctx->s0, 16))) break;
    (void)hipMemsetAsync(ctx->s3.p, 0, sizeof(float) * (size_t)nwg * ncols, ctx->stream);
    (void)hipMemsetAsync(ctx->s4.p, 0, sizeof(unsigned) * (size_t)nwg * nwords, ctx->stream);
    (void)hipMemsetAsync(ctx->s0.p, 0, sizeof(int), ctx->stream);
    hipLaunchKernelGGL(centroid_rows, dim3(nwg), dim3(kCB), 0, ctx->stream, R,
                       rp, col, frp, fcol, fval, ncols, cap_off.as<int64_t>(),
                       tcol.as<int>(), tval.as<float>(), cnt.as<int>(),
                       ctx->s3.as<float>(), ctx->s4.as<unsigned>(), ctx->s0.as<int>());
    if ((rc = hgx_ensure(ctx, p, sizeof(int64_t) * (R + 1)))) break;
    {
      // exclusive scan of the row counts into p
      hipcub::TransformInputIterator<int64_t, ToI64, const int *> it(cnt.as<int>(), ToI64());
      size_t tmp = 0;
      (void)hipMemsetAsync(cnt.as<int>() + R, 0, sizeof(int), ctx->stream);
      HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, p.as<int64_t>(),
                                                    R + 1, ctx->stream));
      if ((rc = hgx_ensure(ctx, ctx->s2, tmp + 16))) break;
      HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(ctx->s2.p, tmp, it, p.as<int64_t>(),
                                                    R + 1, ctx->stream));
      HGX_HIP(ctx, hipMemcpyAsync(&nnz, p.as<int64_t>() + R, sizeof(int64_t),
                                  hipMemcpyDeviceToHost, ctx->stream));
      HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    if ((rc = hgx_ensure(ctx, j, sizeof(int) * (nnz + 1)))) break;
    if ((rc = hgx_ensure(ctx, v, sizeof(float) * (nnz + 1)))) break;
    hipLaunchKernelGGL(compact_rows, dim3(grid_for(R, 1, 65536)), dim3(64), 0,
                       ctx->stream, R, cap_off.as<int64_t>(), p.as<int64_t>(),
                       cnt.as<int>(), tcol.as<int>(), tval.as<float>(),
                       j.as<int>(), v.as<float>());
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  } while (0);
  cleanup();
  return rc;
}

JacArgs jac_args(hgx_ctx *ctx) {
  JacArgs J;
  J.rp_n = ctx->rp_n.as<int>();
  J.col_n = ctx->col_n.as<int>();
  J.rp_e = ctx->rp_e.as<int>();
  J.col_e = ctx->col_e.as<int>();
  J.fn = ctx->feat_n.as<float>();
  J.fe = ctx->feat_e.as<float>();
  J.cn_p = ctx->cn_p.as<int64_t>();
  J.cn_j = ctx->cn_j.as<int>();
  J.cn_v = ctx->cn_v.as<float>();
  J.ce_p = ctx->ce_p.as<int64_t>();
  J.ce_j = ctx->ce_j.as<int>();
  J.ce_v = ctx->ce_v.as<float>();
  return J;
}

int ensure_centroids(hgx_ctx *ctx) {
  if (ctx->centroids_ok) return HGX_OK;
  int64_t nnz = 0;
  // node centroid[v] = mean of edge2features rows of E(v): over nodes
  HGX_TRY(build_centroids(ctx, ctx->N, ctx->rp_n.as<int>(), ctx->col_n.as<int>(),
                          ctx->rp_e.as<int>(), ctx->col_e.as<int>(),
                          ctx->feat_e.as<float>(), ctx->N, ctx->cn_p, ctx->cn_j,
                          ctx->cn_v, nnz));
  ctx->cn_nnz = nnz;
  // edge centroid[e] = mean of node2features rows of N(e): over edges
  HGX_TRY(build_centroids(ctx, ctx->E, ctx->rp_e.as<int>(), ctx->col_e.as<int>(),
                          ctx->rp_n.as<int>(), ctx->col_n.as<int>(),
                          ctx->feat_n.as<float>(), ctx->E, ctx->ce_p, ctx->ce_j,
                          ctx->ce_v, nnz));
  ctx->ce_nnz = nnz;
  ctx->centroids_ok = true;
  return HGX_OK;
}

}  // namespace

// sampler building blocks shared with hgx_sample.hip
int hgx_sample_pairs4(hgx_ctx *ctx, uint64_t seed, int K, const int32_t *node_q,
                      const int32_t *edge_q, int64_t *o_ee, int64_t *o_ne,
                      int64_t *total);

extern "C" int hgx_features_set(hgx_ctx *ctx, const float *node_major,
                                const float *edge_major) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, node_major && edge_major, HGX_EINVAL, "null feature buffer");
  for (int64_t i = 0; i < ctx->nnz; i++)
    HGX_CHECK(ctx, node_major[i] >= 0.0f && edge_major[i] >= 0.0f, HGX_EINVAL,
              "negative feature value");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, ctx->feat_n, sizeof(float) * (ctx->nnz + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->feat_e, sizeof(float) * (ctx->nnz + 1)));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->feat_n.p, node_major, sizeof(float) * ctx->nnz,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->feat_e.p, edge_major, sizeof(float) * ctx->nnz,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->features_ok = true;
  ctx->centroids_ok = false;
  return HGX_OK;
}

extern "C" int hgx_jaccard_centroids(hgx_ctx *ctx, int which, int64_t *nnz,
                                     int64_t *rowptr, int32_t *col, float *val) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->features_ok, HGX_ESTATE, "hgx_features_set not called");
  HGX_CHECK(ctx, which == 0 || which == 1, HGX_EINVAL, "which must be 0 or 1");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(ensure_centroids(ctx));
  const int R = which == 0 ? ctx->N : ctx->E;
  const int64_t n = which == 0 ? ctx->cn_nnz : ctx->ce_nnz;
  DevBuf &p = which == 0 ? ctx->cn_p : ctx->ce_p;
  DevBuf &j = which == 0 ? ctx->cn_j : ctx->ce_j;
  DevBuf &v = which == 0 ? ctx->cn_v : ctx->ce_v;
  if (nnz) *nnz = n;
  if (rowptr)
    HGX_HIP(ctx, hipMemcpy(rowptr, p.p, sizeof(int64_t) * (R + 1), hipMemcpyDeviceToHost));
  if (col && n) HGX_HIP(ctx, hipMemcpy(col, j.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  if (val && n) HGX_HIP(ctx, hipMemcpy(val, v.p, sizeof(float) * n, hipMemcpyDeviceToHost));
  return HGX_OK;
}

extern "C" int hgx_jaccard_probs(hgx_ctx *ctx, int kind, int64_t n,
                                 const int32_t *a, const int32_t *b, float *out) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->features_ok, HGX_ESTATE, "hgx_features_set not called");
  HGX_CHECK(ctx, kind >= 0 && kind <= 2, HGX_EINVAL, "kind must be 0, 1 or 2");
  HGX_CHECK(ctx, n >= 0 && (n == 0 || (a && b && out)), HGX_EINVAL, "null pair buffer");
  const int na = kind == 1 ? ctx->E : ctx->N, nb = kind == 0 ? ctx->N : ctx->E;
  for (int64_t i = 0; i < n; i++)
    HGX_CHECK(ctx, a[i] >= 0 && a[i] < na && b[i] >= 0 && b[i] < nb, HGX_EINVAL,
              "pair %lld out of range", (long long)i);
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  if (kind == 2) HGX_TRY(ensure_centroids(ctx));
  if (n == 0) return HGX_OK;
  HGX_TRY(hgx_ensure(ctx, ctx->s1, sizeof(int) * 2 * n + sizeof(float) * n));
  int *da = ctx->s1.as<int>(), *db = da + n;
  float *dout = reinterpret_cast<float *>(db + n);
  HGX_HIP(ctx, hipMemcpyAsync(da, a, sizeof(int) * n, hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(db, b, sizeof(int) * n, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(jac_pairs, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream,
                     jac_args(ctx), kind, n, da, db, dout);
  HGX_LAUNCH_CHECK(ctx);
  HGX_HIP(ctx, hipMemcpyAsync(out, dout, sizeof(float) * n, hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

// the three kind blocks' probabilities of a pair stream on the context
// (records [0, o_ee) nn, [o_ee, o_ne) ee, [o_ne, total) node-edge): shared
// by hgx_sample_jaccard and the numpy-seeded sampler (hgx_mt.hip)
int hgx_jaccard_fill(hgx_ctx *ctx, int64_t o_ee, int64_t o_ne, int64_t total) {
  HGX_CHECK(ctx, ctx->features_ok, HGX_ESTATE, "hgx_features_set not called");
  HGX_TRY(ensure_centroids(ctx));
  const JacArgs J = jac_args(ctx);
  const int R = 4 + 2 * ctx->K;
  hipLaunchKernelGGL(jac_fill, dim3(grid_for(o_ee, 256)), dim3(256), 0, ctx->stream,
                     J, 0, (int64_t)0, o_ee, R, ctx->rec_idx.as<int>(),
                     ctx->rec_tgt.as<float>());
  hipLaunchKernelGGL(jac_fill, dim3(grid_for(o_ne - o_ee, 256)), dim3(256), 0,
                     ctx->stream, J, 1, o_ee, o_ne, R, ctx->rec_idx.as<int>(),
                     ctx->rec_tgt.as<float>());
  hipLaunchKernelGGL(jac_fill, dim3(grid_for(total - o_ne, 256)), dim3(256), 0,
                     ctx->stream, J, 2, o_ne, total, R, ctx->rec_idx.as<int>(),
                     ctx->rec_tgt.as<float>());
  HGX_LAUNCH_CHECK(ctx);
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_sample_jaccard(hgx_ctx *ctx, uint64_t seed, int K,
                                  const int32_t *node_quota,
                                  const int32_t *edge_quota, int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, ctx->features_ok, HGX_ESTATE, "hgx_features_set not called");
  HGX_CHECK(ctx, K >= 1 && K <= 16, HGX_EUNSUP, "num_neighbors %d outside [1,16]", K);
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(ensure_centroids(ctx));
  int64_t o_ee = 0, o_ne = 0, total = 0;
  HGX_TRY(hgx_sample_pairs4(ctx, seed, K, node_quota, edge_quota, &o_ee, &o_ne, &total));
  HGX_TRY(hgx_jaccard_fill(ctx, o_ee, o_ne, total));
  if (n_records) *n_records = total;
  return HGX_OK;
}
