// HOBE pair probabilities and per-incidence weights on MI355X.
//
// Reference: hg2v_sample.py:527-543 (_same_type_dist_calc): for a pair
// (i, j) of the same type, over the shared targets t (edges for node pairs,
// nodes for edge pairs), w_xt = (sqrt(k) - ||a_x - a_t||_2) / sqrt(k) in
// float32 and prob = max_t min(w_it, w_jt) (0 when nothing is shared);
// hg2v_sample.py:588-629 (DiffTypeDistanceSample): node-edge prob(v, e) =
// max over e' in E(v) of the edge-edge prob(e, e') (the node term at
// :607-616 is disabled).
// hg2v_weighting.py:195-198 (UniformWeight), 137-167 (WeightByNeighborhood).
//
// Bit-exactness with numpy: np.linalg.norm of a float32 vector of length
// k < 32 runs OpenBLAS sdot's tail loop -- float products accumulated in a
// DOUBLE, cast to float, then a float sqrt. The kernel does the same with
// explicitly rounded products (no contraction) and a correctly rounded
// sqrt and divide.
#include <algorithm>
#include <cmath>
#include <vector>

#include "hgx_internal.h"

namespace {

// a, b: coordinate rows in the [w, c_0..c_{k-1}, pad] layout.
__device__ __forceinline__ float dist_weight(const float *__restrict__ a,
                                             const float *__restrict__ b,
                                             int k) {
  double acc = 0.0;
  for (int d = 1; d <= k; d++) {
    const float df = __fsub_rn(a[d], b[d]);
    acc += (double)__fmul_rn(df, df);
  }
  const float nrm = (float)sqrt((double)(float)acc);
  const float md = (float)sqrt((double)k);
  return __fdiv_rn(__fsub_rn(md, nrm), md);
}

// max over t in row_i ∩ row_j of min(w(src_i, tgt_t), w(src_j, tgt_t))
__device__ float same_type_prob(const int *__restrict__ rp,
                                const int *__restrict__ col, int i, int j,
                                const float *__restrict__ src,
                                const float *__restrict__ tgt, int KS, int k) {
  int a = rp[i], ae = rp[i + 1], b = rp[j], be = rp[j + 1];
  const float *si = src + (size_t)i * KS, *sj = src + (size_t)j * KS;
  float prob = 0.f;
  while (a < ae && b < be) {
    const int ca = col[a], cb = col[b];
    if (ca < cb) {
      a++;
    } else if (ca > cb) {
      b++;
    } else {
      const float *tt = tgt + (size_t)ca * KS;
      const float wi = dist_weight(si, tt, k);
      const float wj = dist_weight(sj, tt, k);
      const float m = wj < wi ? wj : wi;
      if (m > prob) prob = m;
      a++;
      b++;
    }
  }
  return prob;
}

__global__ void hobe_probs_kernel(int kind, int64_t n, const int *__restrict__ pa,
                                  const int *__restrict__ pb,
                                  const int *__restrict__ rp_n,
                                  const int *__restrict__ col_n,
                                  const int *__restrict__ rp_e,
                                  const int *__restrict__ col_e,
                                  const float *__restrict__ X,
                                  const float *__restrict__ Y, int KS, int k,
                                  float *__restrict__ out) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int a = pa[q], b = pb[q];
    float p;
    if (kind == 0) {
      p = same_type_prob(rp_n, col_n, a, b, X, Y, KS, k);
    } else if (kind == 1) {
      p = same_type_prob(rp_e, col_e, a, b, Y, X, KS, k);
    } else {
      p = 0.f;
      for (int t = rp_n[a]; t < rp_n[a + 1]; t++) {
        const float pe = same_type_prob(rp_e, col_e, b, col_n[t], Y, X, KS, k);
        if (pe > p) p = pe;
      }
    }
    out[q] = p;
  }
}

// w for every incidence, in the order of the given CSR (rows of `rowtab`,
// columns of `coltab`).
__global__ void incidence_weight_kernel(int which, double alpha, int R,
                                        const int *__restrict__ rp,
                                        const int *__restrict__ col,
                                        const float *__restrict__ rowtab,
                                        const float *__restrict__ coltab,
                                        int KS, int k,
                                        const int *__restrict__ rp_other,
                                        int other_min, int other_max,
                                        float *__restrict__ out) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R;
       r += gridDim.x * blockDim.x) {
    for (int t = rp[r]; t < rp[r + 1]; t++) {
      const int c = col[t];
      float w;
      if (which == 0) {
        w = 1.0f;
      } else if (which == 1) {
        // weight of incidence (r, c) = neighbourhood factor of the COLUMN
        // entity: alpha + (1-alpha) * (1 - zero_one(|c|)), double math,
        // rounded to float once (DictToSparseRow stores float32).
        const int sz = rp_other[c + 1] - rp_other[c];
        double z = other_max == other_min
                       ? 1.0
                       : (double)(sz - other_min) / (double)(other_max - other_min);
        w = (float)(alpha + (1.0 - alpha) * (1.0 - z));
      } else {
        w = dist_weight(rowtab + (size_t)r * KS, coltab + (size_t)c * KS, k);
      }
      out[t] = w;
    }
  }
}

// HOBE targets for records [b, e) of one kind (ids in the records are +1)
__global__ void fill_probs_kernel(int kind, int64_t b, int64_t e, int R,
                                  const int *__restrict__ idx,
                                  float *__restrict__ tgt,
                                  const int *__restrict__ rp_n,
                                  const int *__restrict__ col_n,
                                  const int *__restrict__ rp_e,
                                  const int *__restrict__ col_e,
                                  const float *__restrict__ X,
                                  const float *__restrict__ Y, int KS, int k) {
  for (int64_t q = b + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < e;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int *ri = idx + q * R;
    float p;
    if (kind == 0) {
      p = same_type_prob(rp_n, col_n, ri[0] - 1, ri[2] - 1, X, Y, KS, k);
    } else if (kind == 1) {
      p = same_type_prob(rp_e, col_e, ri[1] - 1, ri[3] - 1, Y, X, KS, k);
    } else {
      const int v = ri[0] - 1, ed = ri[3] - 1;
      p = 0.f;
      for (int t = rp_n[v]; t < rp_n[v + 1]; t++) {
        const float pe = same_type_prob(rp_e, col_e, ed, col_n[t], Y, X, KS, k);
        if (pe > p) p = pe;
      }
    }
    tgt[q * 3 + kind] = p;
  }
}

int grid_for(int64_t work, int per_block) {
  int64_t g = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 4096));
}

}  // namespace

extern "C" int hgx_hobe_probs(hgx_ctx *ctx, int kind, int64_t n,
                              const int32_t *a, const int32_t *b, float *out) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE, "no alg coordinates on device");
  HGX_CHECK(ctx, kind >= 0 && kind <= 2, HGX_EINVAL, "kind must be 0, 1 or 2");
  HGX_CHECK(ctx, n >= 0, HGX_EINVAL, "negative pair count");
  if (n == 0) return HGX_OK;
  HGX_CHECK(ctx, a && b && out, HGX_EINVAL, "null pair buffer");
  const int32_t na = kind == 1 ? ctx->E : ctx->N;
  const int32_t nb = kind == 0 ? ctx->N : ctx->E;
  for (int64_t q = 0; q < n; q++)
    HGX_CHECK(ctx, a[q] >= 0 && a[q] < na && b[q] >= 0 && b[q] < nb,
              HGX_EINVAL, "pair %lld = (%d, %d) out of range", (long long)q,
              a[q], b[q]);
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(int32_t) * n));
  HGX_TRY(hgx_ensure(ctx, ctx->s3, sizeof(int32_t) * n));
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * n));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s2.p, a, sizeof(int32_t) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s3.p, b, sizeof(int32_t) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(hobe_probs_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     ctx->stream, kind, n, ctx->s2.as<int>(), ctx->s3.as<int>(),
                     ctx->rp_n.as<int>(), ctx->col_n.as<int>(),
                     ctx->rp_e.as<int>(), ctx->col_e.as<int>(),
                     ctx->X[ctx->xcur].as<float>(),
                     ctx->Y[ctx->ycur].as<float>(), ctx->ks, ctx->k,
                     ctx->s4.as<float>());
  HGX_LAUNCH_CHECK(ctx);
  HGX_HIP(ctx, hipMemcpyAsync(out, ctx->s4.p, sizeof(float) * n,
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_incidence_weights(hgx_ctx *ctx, int which, double alpha,
                                     float *node_major, float *edge_major) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, which >= 0 && which <= 2, HGX_EINVAL, "which must be 0..2");
  HGX_CHECK(ctx, alpha >= 0.0 && alpha <= 1.0, HGX_EINVAL,
            "alpha must be in [0,1] (hg2v_weighting.py:331-332)");
  HGX_CHECK(ctx, which != 2 || ctx->k > 0, HGX_ESTATE,
            "distance weights need alg coordinates on device");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * (ctx->nnz + 1)));
  // min/max of node degrees and edge sizes (host copies of row pointers
  // are not kept, so compute them on the host from a device copy once)
  int dmin = 0, dmax = 0, smin = 0, smax = 0;
  if (which == 1) {
    std::vector<int> rn(ctx->N + 1), re(ctx->E + 1);
    HGX_HIP(ctx, hipMemcpy(rn.data(), ctx->rp_n.p, sizeof(int) * (ctx->N + 1),
                           hipMemcpyDeviceToHost));
    HGX_HIP(ctx, hipMemcpy(re.data(), ctx->rp_e.p, sizeof(int) * (ctx->E + 1),
                           hipMemcpyDeviceToHost));
    dmin = smin = INT32_MAX;
    for (int i = 0; i < ctx->N; i++) {
      dmin = std::min(dmin, rn[i + 1] - rn[i]);
      dmax = std::max(dmax, rn[i + 1] - rn[i]);
    }
    for (int i = 0; i < ctx->E; i++) {
      smin = std::min(smin, re[i + 1] - re[i]);
      smax = std::max(smax, re[i + 1] - re[i]);
    }
  }
  const float *X = ctx->k ? ctx->X[ctx->xcur].as<float>() : nullptr;
  const float *Y = ctx->k ? ctx->Y[ctx->ycur].as<float>() : nullptr;
  for (int pass = 0; pass < 2; pass++) {
    float *host = pass == 0 ? node_major : edge_major;
    if (!host) continue;
    if (pass == 0)
      hipLaunchKernelGGL(incidence_weight_kernel, dim3(grid_for(ctx->N, 256)),
                         dim3(256), 0, ctx->stream, which, alpha,
                         ctx->N, ctx->rp_n.as<int>(), ctx->col_n.as<int>(), X,
                         Y, ctx->ks, ctx->k, ctx->rp_e.as<int>(), smin, smax,
                         ctx->s4.as<float>());
    else
      hipLaunchKernelGGL(incidence_weight_kernel, dim3(grid_for(ctx->E, 256)),
                         dim3(256), 0, ctx->stream, which, alpha,
                         ctx->E, ctx->rp_e.as<int>(), ctx->col_e.as<int>(), Y,
                         X, ctx->ks, ctx->k, ctx->rp_n.as<int>(), dmin, dmax,
                         ctx->s4.as<float>());
    HGX_LAUNCH_CHECK(ctx);
    HGX_HIP(ctx, hipMemcpyAsync(host, ctx->s4.p, sizeof(float) * ctx->nnz,
                                hipMemcpyDeviceToHost, ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return HGX_OK;
}

// Used by hgx_sample_hobe: fill the probability target of records [b, e).
int hgx_hobe_fill_probs(hgx_ctx *ctx, int kind, int64_t b, int64_t e) {
  if (e <= b) return HGX_OK;
  hipLaunchKernelGGL(fill_probs_kernel, dim3(grid_for(e - b, 256)), dim3(256),
                     0, ctx->stream, kind, b, e, 4 + 2 * ctx->K,
                     ctx->rec_idx.as<int>(), ctx->rec_tgt.as<float>(),
                     ctx->rp_n.as<int>(), ctx->col_n.as<int>(),
                     ctx->rp_e.as<int>(), ctx->col_e.as<int>(),
                     ctx->X[ctx->xcur].as<float>(),
                     ctx->Y[ctx->ycur].as<float>(), ctx->ks, ctx->k);
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}
