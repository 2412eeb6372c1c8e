// hg2v_weighting's distance and span weights on MI355X (SURVEY §8a A15 and
// the north star's "first/second-order pair weights").
//
// Reference (hypergraph_embedding/hg2v_weighting.py):
//   WeightByDistance 67-103     first order: per incidence (v, e) the norm of
//                               node_vec - edge_vec (float32 vectors), then
//                               ZeroOneScaleValues -> OneMinusValues ->
//                               AlphaScaleValues (301-333) over all
//                               incidences, stored in a float32 lil_matrix
//   WeightBySameTypeDistance 34-64
//                               second order: every pair of the A A^T (node)
//                               or A^T A (edge) pattern, diagonal included,
//                               norm of the difference, same scaling
//   ComputeSpans 207-293        per node: over its edges e and dimensions,
//                               max(0, max(e - v)) - min(0, min(e - v));
//                               per edge over its nodes
//   WeightByAlgebraicSpan 170-192
//                               spans zero-one / one-minus / alpha scaled,
//                               rounded to float32 (DictToSparseRow) and
//                               multiplied onto A (the edge's value) and A^T
//                               (the node's value)
//
// Bit-exactness. Every value is float32: WeightByDistance asks for float32
// vectors, and np.array(emb.values) / np.subtract(emb.values, ...) of
// protobuf's upb repeated-float containers (protobuf 7, the fixtures'
// version) are float32 arrays too, so the second-order norms and the spans
// are float32 as well. `norm` is np.linalg.norm: sqrt(x.dot(x)), OpenBLAS
// sdot through numpy's FLOAT_dot. The fixtures (tests/golden/
// make_golden_weights.py) were made with numpy's OpenBLAS 0.3.29, SkylakeX
// kernel; norm32 restates its arithmetic (probed against numpy on 3,000
// random vectors of 10-130 elements, no difference): the first k & ~31
// elements in 4 accumulators x 8 lanes (fused multiply-add; blocks of 64
// first go through 4 x 16 lanes folded lane l + l+8), accumulators summed
// ((a0 + a1) + a2) + a3, then lanes l + l+4, then (h0 + h1) + (h2 + h3); the
// rest added in DOUBLE as float products; the float of that, float sqrt.
// The scaling restates numpy 2's scalar rules on np.float32 values: float32
// arithmetic, alpha and 1 - alpha rounded to float32 as weak Python
// scalars. lil_matrix does not store zeros (the largest distance at alpha 0
// disappears): the host drops them too.
//
// Shapes are the reference's: the second-order pattern is materialised
// (that is what the function returns). Its expansion (sum over rows of the
// paths through their incidences) must stay below 2^31 paths; a power-law
// graph like C4 (hub edges of 1.7M nodes) is refused with HGX_EUNSUP -- the
// reference would build the same pattern as a Python dict.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "hgx_internal.h"

// No implicit contraction anywhere in this file: alpha + (1 - alpha) * v
// must stay two roundings (numpy's), and a float product added to a double
// must not become a double fma (hipcc contracts by default, through the
// __fadd_rn / __fmul_rn helpers too).
#pragma clang fp contract(off)

namespace {

// np.linalg.norm of the float32 vector a - b (see the header)
__device__ float norm32(const float *__restrict__ a, const float *__restrict__ b,
                        int k) {
  const int n1 = k & ~31, n64 = n1 & ~63;
  int i = 0;
  float tot = 0.f;
  if (n1) {
    float acc[32];
#pragma unroll
    for (int t = 0; t < 32; t++) acc[t] = 0.f;
    if (n64) {
      float a5[64];
#pragma unroll
      for (int t = 0; t < 64; t++) a5[t] = 0.f;
      for (; i < n64; i += 64) {
#pragma unroll
        for (int t = 0; t < 64; t++) {
          const float d = a[i + t] - b[i + t];
          a5[t] = __fmaf_rn(d, d, a5[t]);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int l = 0; l < 8; l++)
          acc[j * 8 + l] = a5[j * 16 + l] + a5[j * 16 + l + 8];
    }
    for (; i < n1; i += 32) {
#pragma unroll
      for (int t = 0; t < 32; t++) {
        const float d = a[i + t] - b[i + t];
        acc[t] = __fmaf_rn(d, d, acc[t]);
      }
    }
    float s[8];
#pragma unroll
    for (int l = 0; l < 8; l++)
      s[l] = ((acc[l] + acc[8 + l]) + acc[16 + l]) + acc[24 + l];
    float h[4];
#pragma unroll
    for (int l = 0; l < 4; l++) h[l] = s[l] + s[l + 4];
    tot = (h[0] + h[1]) + (h[2] + h[3]);
  }
  double dot = tot;
  for (; i < k; i++) {
    const float d = a[i] - b[i];
    const float p = d * d;
    dot = dot + (double)p;
  }
  // correctly rounded float sqrt (v_sqrt_f32 is not): through double
  return (float)sqrt((double)(float)dot);
}

// ord = inf: max |a_d - b_d| (exact in any order)
__device__ float ninf32(const float *a, const float *b, int k) {
  float m = 0.f;
  for (int i = 0; i < k; i++) m = fmaxf(m, fabsf(a[i] - b[i]));
  return m;
}

int grid_for(int64_t work, int per_block, int cap = 8192) {
  int64_t g = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// ---- first order: per-incidence distance -------------------------------
// Incidence t of the CSR (rp, col) over R rows; the node's row is `nodetab`
// row (node_is_row ? r : col[t]), the edge's the other. mm = {min bits, max
// bits} of the non-negative float values (uint order = float order).
__global__ void dist_incidence_kernel(int norm, int64_t nnz, int R,
                                      const int *__restrict__ rp,
                                      const int *__restrict__ col,
                                      const float *__restrict__ nodetab,
                                      const float *__restrict__ edgetab,
                                      bool node_is_row, int ks, int k,
                                      float *__restrict__ out,
                                      unsigned *__restrict__ mm) {
  for (int64_t b0 = blockIdx.x * (int64_t)blockDim.x; b0 < nnz;
       b0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = b0 + threadIdx.x;
    const bool act = t < nnz;
    float w = 0.f;
    if (act) {
      int lo = 0, hi = R - 1;
      while (lo < hi) {  // last row r with rp[r] <= t
        const int mid = (lo + hi + 1) >> 1;
        if (rp[mid] <= t) lo = mid;
        else hi = mid - 1;
      }
      const int c = col[t];
      const float *a = nodetab + (size_t)(node_is_row ? lo : c) * ks + 1;
      const float *b = edgetab + (size_t)(node_is_row ? c : lo) * ks + 1;
      w = norm == HGX_NORM_L2 ? norm32(a, b, k) : ninf32(a, b, k);
      out[t] = w;
    }
    if (mm) {
      const float mx = hgx::wave_max(act ? w : 0.f);
      const float mn = hgx::wave_min(act ? w : INFINITY);
      if ((threadIdx.x & 63) == 0) {
        atomicMax(&mm[1], __float_as_uint(mx));
        atomicMin(&mm[0], __float_as_uint(mn));
      }
    }
  }
}

// ZeroOneScaleValues -> OneMinusValues -> AlphaScaleValues on np.float32
// values: (v - min) / (max - min), 1 - z, a32 + b32 * o, all float32 (delta
// 0: every value 1 -> 0 -> alpha).
__global__ void scale_f32_kernel(int64_t n, float *__restrict__ v,
                                 const unsigned *__restrict__ mm, float a32,
                                 float b32) {
  const float mn = __uint_as_float(mm[0]);
  const float delta = __uint_as_float(mm[1]) - mn;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const float o = delta == 0.f ? 0.f : 1.f - __fdiv_rn(v[t] - mn, delta);
    const float p = b32 * o;  // two roundings: contraction is off
    v[t] = a32 + p;
  }
}

// ---- spans: one wave per row ---------------------------------------------
// row r of (rp, col): own coordinates `mine`, neighbours `other`; diff =
// other - mine (float32); span = max(0, max diff) - min(0, min diff).
__global__ __launch_bounds__(256) void span_kernel(
    int R, const int *__restrict__ rp, const int *__restrict__ col,
    const float *__restrict__ mine, const float *__restrict__ other, int ks,
    int k, float *__restrict__ span, unsigned *__restrict__ mm) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  float wlo = INFINITY, whi = 0.f;
  for (int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < R; r += nw) {
    const int b = rp[r], e = rp[r + 1];
    const float *m = mine + (size_t)r * ks + 1;
    float hi = 0.f, lo = 0.f;
    const int64_t work = (int64_t)(e - b) * k;
    for (int64_t w = lane; w < work; w += 64) {
      const int j = b + (int)(w / k), d = (int)(w % k);
      const float df = other[(size_t)col[j] * ks + 1 + d] - m[d];
      hi = fmaxf(hi, df);
      lo = fminf(lo, df);
    }
    hi = hgx::wave_max(hi);
    lo = hgx::wave_min(lo);
    // (+ 0: a zero span is +0, so the unsigned bit order of the min / max
    // atomics is the float order)
    const float s = (hi - lo) + 0.f;
    if (lane == 0) span[r] = s;
    wlo = fminf(wlo, s);
    whi = fmaxf(whi, s);
  }
  if (lane == 0 && whi >= wlo) {
    atomicMin(&mm[0], __float_as_uint(wlo));
    atomicMax(&mm[1], __float_as_uint(whi));
  }
}

// incidence t of (rp, col) gets the value of its column entity (A's node2
// weight[v, e] = w_edge[e]; A^T's edge2weight[e, v] = w_node[v])
__global__ void column_value_kernel(int64_t nnz, const int *__restrict__ col,
                                    const float *__restrict__ w,
                                    float *__restrict__ out) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nnz;
       t += (int64_t)gridDim.x * blockDim.x)
    out[t] = w[col[t]];
}

// ---- second order -----------------------------------------------------
// paths of row r of A A^T (through rp/col then rq/cq): sum of |e| over r's e
__global__ void path_count_kernel(int R, const int *__restrict__ rp,
                                  const int *__restrict__ col,
                                  const int *__restrict__ rq,
                                  long long *__restrict__ cnt) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R;
       r += gridDim.x * blockDim.x) {
    long long s = 0;
    for (int t = rp[r]; t < rp[r + 1]; t++) s += rq[col[t] + 1] - rq[col[t]];
    cnt[r] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[R] = 0;
}

// every path endpoint of row r at off[r]..: one wave per row
__global__ __launch_bounds__(256) void path_fill_kernel(
    int R, const int *__restrict__ rp, const int *__restrict__ col,
    const int *__restrict__ rq, const int *__restrict__ cq,
    const long long *__restrict__ off, int *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < R; r += nw) {
    long long o = off[r];
    for (int t = rp[r]; t < rp[r + 1]; t++) {
      const int e = col[t], b = rq[e], n = rq[e + 1] - b;
      for (int j = lane; j < n; j += 64) out[o + j] = cq[b + j];
      o += n;
    }
  }
}

// distinct columns per sorted row segment: one wave per row
__global__ __launch_bounds__(256) void unique_count_kernel(
    int R, const long long *__restrict__ off, const int *__restrict__ key,
    int *__restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  for (int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < R; r += nw) {
    const long long b = off[r], e = off[r + 1];
    int c = 0;
    for (long long i = b + lane; i < e; i += 64) c += (i == b || key[i] != key[i - 1]);
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) c += __shfl_xor(c, s);
    if (lane == 0) cnt[r] = c;
  }
}

// distinct columns written at outp[r].., with the norm of the two rows'
// difference (float32); min / max of the norms
__global__ __launch_bounds__(256) void pattern_norm_kernel(
    int norm, int R, const long long *__restrict__ off, const int *__restrict__ key,
    const long long *__restrict__ outp, int *__restrict__ ocol,
    float *__restrict__ oval, const float *__restrict__ tab, int ks, int k,
    unsigned *__restrict__ mm) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  float wlo = INFINITY, whi = 0.f;
  for (int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < R; r += nw) {
    const long long b = off[r], e = off[r + 1];
    long long o = outp[r];
    const float *mine = tab + (size_t)r * ks + 1;
    for (long long i0 = b; i0 < e; i0 += 64) {
      const long long i = i0 + lane;
      const bool first = i < e && (i == b || key[i] != key[i - 1]);
      const unsigned long long bal = __ballot(first);
      if (first) {
        const int pos = __popcll(bal & ((1ull << lane) - 1));
        const int c = key[i];
        const float *other = tab + (size_t)c * ks + 1;
        const float v = norm == HGX_NORM_L2 ? norm32(mine, other, k)
                                            : ninf32(mine, other, k);
        ocol[o + pos] = c;
        oval[o + pos] = v;
        wlo = fminf(wlo, v);
        whi = fmaxf(whi, v);
      }
      o += __popcll(bal);
    }
  }
  wlo = hgx::wave_min(wlo);
  whi = hgx::wave_max(whi);
  if (lane == 0 && whi >= wlo) {
    atomicMin(&mm[0], __float_as_uint(wlo));
    atomicMax(&mm[1], __float_as_uint(whi));
  }
}

struct ToI64 {
  __host__ __device__ long long operator()(int x) const { return x; }
};

int check_weights(hgx_ctx *ctx, int norm) {
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE,
            "no embedding on device (hgx_alg_set the reference embedding)");
  HGX_CHECK(ctx, norm == HGX_NORM_L2 || norm == HGX_NORM_INF, HGX_EINVAL,
            "norm must be HGX_NORM_L2 or HGX_NORM_INF");
  return HGX_OK;
}

int mm_init32(hgx_ctx *ctx, DevBuf &b) {
  HGX_TRY(hgx_ensure(ctx, b, 8));
  const unsigned init[2] = {0x7f800000u /* +inf */, 0u};
  HGX_HIP(ctx, hipMemcpyAsync(b.p, init, 8, hipMemcpyHostToDevice, ctx->stream));
  return HGX_OK;
}

}  // namespace

extern "C" int hgx_weight_distance(hgx_ctx *ctx, int norm, double alpha,
                                   float *node_major, float *edge_major) {
  if (!ctx) return HGX_EINVAL;
  HGX_TRY(check_weights(ctx, norm));
  HGX_CHECK(ctx, alpha >= 0.0 && alpha <= 1.0, HGX_EINVAL,
            "alpha must be in [0,1] (hg2v_weighting.py:331-332)");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int64_t nnz = ctx->nnz;
  if (nnz == 0) return HGX_OK;
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * nnz));
  HGX_TRY(hgx_ensure(ctx, ctx->s5, sizeof(float) * nnz));
  HGX_TRY(mm_init32(ctx, ctx->s0));
  const float *X = ctx->X[ctx->xcur].as<float>();
  const float *Y = ctx->Y[ctx->ycur].as<float>();
  unsigned *mm = ctx->s0.as<unsigned>();
  hipLaunchKernelGGL(dist_incidence_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0,
                     ctx->stream, norm, nnz, ctx->N, ctx->rp_n.as<int>(),
                     ctx->col_n.as<int>(), X, Y, true, ctx->ks, ctx->k,
                     ctx->s4.as<float>(), mm);
  HGX_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(dist_incidence_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0,
                     ctx->stream, norm, nnz, ctx->E, ctx->rp_e.as<int>(),
                     ctx->col_e.as<int>(), X, Y, false, ctx->ks, ctx->k,
                     ctx->s5.as<float>(), (unsigned *)nullptr);
  HGX_LAUNCH_CHECK(ctx);
  // AlphaScaleValues on np.float32 values: alpha and 1 - alpha are weak
  // Python scalars, cast to float32 (NEP 50)
  const float a32 = (float)alpha, b32 = (float)(1.0 - alpha);
  for (DevBuf *b : {&ctx->s4, &ctx->s5}) {
    hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0,
                       ctx->stream, nnz, b->as<float>(), mm, a32, b32);
    HGX_LAUNCH_CHECK(ctx);
  }
  if (node_major)
    HGX_HIP(ctx, hipMemcpyAsync(node_major, ctx->s4.p, sizeof(float) * nnz,
                                hipMemcpyDeviceToHost, ctx->stream));
  if (edge_major)
    HGX_HIP(ctx, hipMemcpyAsync(edge_major, ctx->s5.p, sizeof(float) * nnz,
                                hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_weight_span(hgx_ctx *ctx, double alpha, float *node_span,
                               float *edge_span, float *node_major,
                               float *edge_major) {
  if (!ctx) return HGX_EINVAL;
  HGX_TRY(check_weights(ctx, HGX_NORM_L2));
  HGX_CHECK(ctx, alpha >= 0.0 && alpha <= 1.0, HGX_EINVAL,
            "alpha must be in [0,1] (hg2v_weighting.py:331-332)");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int N = ctx->N, E = ctx->E;
  const int64_t nnz = ctx->nnz;
  // s1: spans (N + E floats), s2: their weights, s0: 2 x {min, max}
  HGX_TRY(hgx_ensure(ctx, ctx->s1, sizeof(float) * ((size_t)N + E)));
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(float) * ((size_t)N + E)));
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * (nnz + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->s0, 16));
  const unsigned init[4] = {0x7f800000u, 0u, 0x7f800000u, 0u};
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s0.p, init, 16, hipMemcpyHostToDevice,
                              ctx->stream));
  float *sn = ctx->s1.as<float>(), *se = sn + N;
  unsigned *mmn = ctx->s0.as<unsigned>(), *mme = mmn + 2;
  const float *X = ctx->X[ctx->xcur].as<float>();
  const float *Y = ctx->Y[ctx->ycur].as<float>();
  // node spans over their edges (diff = edge - node), edge spans over their
  // nodes (diff = node - edge): hg2v_weighting.py:226-232, 271-292
  hipLaunchKernelGGL(span_kernel, dim3(grid_for(N, 4)), dim3(256), 0, ctx->stream,
                     N, ctx->rp_n.as<int>(), ctx->col_n.as<int>(), X, Y, ctx->ks,
                     ctx->k, sn, mmn);
  HGX_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(span_kernel, dim3(grid_for(E, 4)), dim3(256), 0, ctx->stream,
                     E, ctx->rp_e.as<int>(), ctx->col_e.as<int>(), Y, X, ctx->ks,
                     ctx->k, se, mme);
  HGX_LAUNCH_CHECK(ctx);
  if (node_span)
    HGX_HIP(ctx, hipMemcpyAsync(node_span, sn, sizeof(float) * N,
                                hipMemcpyDeviceToHost, ctx->stream));
  if (edge_span)
    HGX_HIP(ctx, hipMemcpyAsync(edge_span, se, sizeof(float) * E,
                                hipMemcpyDeviceToHost, ctx->stream));
  // ZeroOneScaleValues -> OneMinusValues -> AlphaScaleValues per side on a
  // copy (DictToSparseRow keeps float32)
  float *wn = ctx->s2.as<float>(), *we = wn + N;
  HGX_HIP(ctx, hipMemcpyAsync(wn, sn, sizeof(float) * ((size_t)N + E),
                              hipMemcpyDeviceToDevice, ctx->stream));
  const float a32 = (float)alpha, b32 = (float)(1.0 - alpha);
  hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(N, 256)), dim3(256), 0,
                     ctx->stream, (int64_t)N, wn, mmn, a32, b32);
  hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(E, 256)), dim3(256), 0,
                     ctx->stream, (int64_t)E, we, mme, a32, b32);
  HGX_LAUNCH_CHECK(ctx);
  // node2weight = A * edge span weights, edge2weight = A^T * node ones
  for (int pass = 0; pass < 2; pass++) {
    float *host = pass == 0 ? node_major : edge_major;
    if (!host || nnz == 0) continue;
    hipLaunchKernelGGL(column_value_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0,
                       ctx->stream, nnz,
                       (pass == 0 ? ctx->col_n : ctx->col_e).as<int>(),
                       pass == 0 ? we : wn, ctx->s4.as<float>());
    HGX_LAUNCH_CHECK(ctx);
    HGX_HIP(ctx, hipMemcpyAsync(host, ctx->s4.p, sizeof(float) * nnz,
                                hipMemcpyDeviceToHost, ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_weight_same_type(hgx_ctx *ctx, int side, int norm,
                                    double alpha, int64_t *nnz_out,
                                    int64_t *rowptr, int32_t *col, float *val) {
  if (!ctx) return HGX_EINVAL;
  HGX_TRY(check_weights(ctx, norm));
  HGX_CHECK(ctx, side == 0 || side == 1, HGX_EINVAL, "side must be 0 or 1");
  HGX_CHECK(ctx, alpha >= 0.0 && alpha <= 1.0, HGX_EINVAL,
            "alpha must be in [0,1] (hg2v_weighting.py:331-332)");
  HGX_CHECK(ctx, nnz_out, HGX_EINVAL, "null nnz_out");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int R = side == 0 ? ctx->N : ctx->E;
  const int *rp = (side == 0 ? ctx->rp_n : ctx->rp_e).as<int>();
  const int *cl = (side == 0 ? ctx->col_n : ctx->col_e).as<int>();
  const int *rq = (side == 0 ? ctx->rp_e : ctx->rp_n).as<int>();
  const int *cq = (side == 0 ? ctx->col_e : ctx->col_n).as<int>();
  const float *tab = (side == 0 ? ctx->X[ctx->xcur] : ctx->Y[ctx->ycur]).as<float>();
  // path offsets (R + 1 int64) in s0
  HGX_TRY(hgx_ensure(ctx, ctx->s0, sizeof(long long) * ((size_t)R + 1)));
  long long *poff = ctx->s0.as<long long>();
  HGX_TRY(hgx_ensure(ctx, ctx->s6, sizeof(long long) * ((size_t)R + 1)));
  hipLaunchKernelGGL(path_count_kernel, dim3(grid_for(R, 256)), dim3(256), 0,
                     ctx->stream, R, rp, cl, rq, ctx->s6.as<long long>());
  HGX_LAUNCH_CHECK(ctx);
  size_t tb = 0;
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ctx->s6.as<long long>(),
                                                poff, R + 1, ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->s7, tb));
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(ctx->s7.p, tb, ctx->s6.as<long long>(),
                                                poff, R + 1, ctx->stream));
  long long P = 0;
  HGX_HIP(ctx, hipMemcpyAsync(&P, poff + R, sizeof(P), hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  HGX_CHECK(ctx, P < (long long)INT32_MAX, HGX_EUNSUP,
            "the second-order pattern expands to %lld paths (limit 2^31): "
            "too large to materialise", P);
  // path endpoints (s2), sorted per row (s3)
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(int) * (size_t)std::max(P, 1ll)));
  HGX_TRY(hgx_ensure(ctx, ctx->s3, sizeof(int) * (size_t)std::max(P, 1ll)));
  hipLaunchKernelGGL(path_fill_kernel, dim3(grid_for(R, 4)), dim3(256), 0,
                     ctx->stream, R, rp, cl, rq, cq, poff, ctx->s2.as<int>());
  HGX_LAUNCH_CHECK(ctx);
  int bits = 1;
  while (bits < 31 && (1ll << bits) < (side == 0 ? ctx->N : ctx->E)) bits++;
  tb = 0;
  HGX_HIP(ctx, hipcub::DeviceSegmentedRadixSort::SortKeys(
                   nullptr, tb, ctx->s2.as<int>(), ctx->s3.as<int>(), (int)P, R,
                   poff, poff + 1, 0, bits, ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->s7, tb));
  HGX_HIP(ctx, hipcub::DeviceSegmentedRadixSort::SortKeys(
                   ctx->s7.p, tb, ctx->s2.as<int>(), ctx->s3.as<int>(), (int)P, R,
                   poff, poff + 1, 0, bits, ctx->stream));
  // distinct columns per row (s6 as int counts), output row pointers (s1)
  int *ucnt = ctx->s6.as<int>();
  hipLaunchKernelGGL(unique_count_kernel, dim3(grid_for(R, 4)), dim3(256), 0,
                     ctx->stream, R, poff, ctx->s3.as<int>(), ucnt);
  HGX_LAUNCH_CHECK(ctx);
  HGX_HIP(ctx, hipMemsetAsync(ucnt + R, 0, sizeof(int), ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->s1, sizeof(long long) * ((size_t)R + 1) + 32));
  long long *optr = ctx->s1.as<long long>();
  hipcub::TransformInputIterator<long long, ToI64, const int *> it(ucnt, ToI64());
  tb = 0;
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, it, optr, R + 1,
                                                ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->s7, tb));
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(ctx->s7.p, tb, it, optr, R + 1,
                                                ctx->stream));
  long long nnz = 0;
  HGX_HIP(ctx, hipMemcpyAsync(&nnz, optr + R, sizeof(nnz), hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *nnz_out = nnz;
  if (rowptr)
    HGX_HIP(ctx, hipMemcpyAsync(rowptr, optr, sizeof(long long) * ((size_t)R + 1),
                                hipMemcpyDeviceToHost, ctx->stream));
  if (!col && !val) {
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return HGX_OK;
  }
  // columns (s2, reused) and norms (s5), scaled in place
  unsigned *mm = (unsigned *)(optr + R + 1);
  const unsigned init[2] = {0x7f800000u, 0u};
  HGX_HIP(ctx, hipMemcpyAsync(mm, init, 8, hipMemcpyHostToDevice, ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->s5, sizeof(float) * (size_t)std::max(nnz, 1ll)));
  hipLaunchKernelGGL(pattern_norm_kernel, dim3(grid_for(R, 4)), dim3(256), 0,
                     ctx->stream, norm, R, poff, ctx->s3.as<int>(), optr,
                     ctx->s2.as<int>(), ctx->s5.as<float>(), tab, ctx->ks, ctx->k,
                     mm);
  HGX_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(scale_f32_kernel, dim3(grid_for(nnz, 256)), dim3(256), 0,
                     ctx->stream, (int64_t)nnz, ctx->s5.as<float>(), mm,
                     (float)alpha, (float)(1.0 - alpha));
  HGX_LAUNCH_CHECK(ctx);
  if (col)
    HGX_HIP(ctx, hipMemcpyAsync(col, ctx->s2.p, sizeof(int) * nnz,
                                hipMemcpyDeviceToHost, ctx->stream));
  if (val)
    HGX_HIP(ctx, hipMemcpyAsync(val, ctx->s5.p, sizeof(float) * nnz,
                                hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}
