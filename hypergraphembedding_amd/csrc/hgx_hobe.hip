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
// DOUBLE, cast to float, then a float sqrt. The weight kernel does the same
// with explicitly rounded products (no contraction) and a correctly rounded
// sqrt and divide. w is symmetric bit for bit (the difference only changes
// sign), so one weight per incidence serves both orientations: `hw_n` in
// A's CSR order (node v, edge e), `hw_e` in A^T's (edge e, node u), and
// `hw_self[e]` = max_u w(e, u). Everything downstream is max / min of these
// values, so any evaluation order gives the reference's result exactly.
//
// Scale (power-law C4: edges of up to 1.7M members). The reference merges
// the two member lists of every edge pair. Here:
//   * nn(u, v): merge of the two (short) edge lists E(u), E(v), one lane
//     per pair;
//   * ee(e, f), one wave per pair: the SMALLER edge's members, each probed
//     for the other edge in its own sorted edge list (binary search over
//     ~deg entries), so the cost is min(|e|, |f|) probes, not |e| + |f|;
//     a member whose own weight w(s, u) cannot beat the running max is not
//     probed, ee(e, e) = hw_self[e], and ee(e, f) <= min(self[e], self[f])
//     ends the scan once reached;
//   * ne(v, e), one wave per pair: either (a) e's members u, each merged
//     against E(v) (cost |e| short merges), or (b) ee(e, e') for every
//     e' in E(v) (cost sum min(|e|, |e'|) probes), whichever is cheaper;
//     ne(v, e) <= self[e] ends either early.
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

// position of x in sorted col[b, e), or -1
__device__ __forceinline__ int find_sorted(const int *__restrict__ col, int b,
                                           int e, int x) {
  int lo = b, hi = e;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (col[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return (lo < e && col[lo] == x) ? lo : -1;
}

struct HobeW {
  const int *rp_n, *col_n, *rp_e, *col_e;
  const float *wn;    // w per incidence, A's CSR order
  const float *we;    // w per incidence, A^T's CSR order
  const float *self;  // per edge: max_u w(e, u)
};

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

// HOBE distance weights of one orientation, one lane per incidence (the
// row of incidence t found by binary search over the row pointers); for the
// edge-major pass also each edge's max weight (order-free atomicMax on the
// bits of non-negative floats; negative weights never win a max that
// starts at 0).
__global__ void hobe_weight_kernel(int64_t nnz, int R, const int *__restrict__ rp,
                                   const int *__restrict__ col,
                                   const float *__restrict__ rowtab,
                                   const float *__restrict__ coltab, int KS,
                                   int k, float *__restrict__ out,
                                   unsigned *__restrict__ rowmax) {
  // whole waves iterate together (the row max is reduced per wave first:
  // a power-law edge spans millions of incidences)
  for (int64_t b0 = blockIdx.x * (int64_t)blockDim.x; b0 < nnz;
       b0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = b0 + threadIdx.x;
    const bool act = t < nnz;
    int lo = 0;
    float w = 0.f;
    if (act) {
      int hi = R - 1;
      while (lo < hi) {  // last row r with rp[r] <= t
        const int mid = (lo + hi + 1) >> 1;
        if (rp[mid] <= t) lo = mid;
        else hi = mid - 1;
      }
      w = dist_weight(rowtab + (size_t)lo * KS, coltab + (size_t)col[t] * KS, k);
      out[t] = w;
    }
    if (!rowmax) continue;
    const int r0 = __builtin_amdgcn_readfirstlane(lo);
    if (__ballot(!act || lo != r0) == 0) {
      const float m = hgx::wave_max(w);
      if ((threadIdx.x & 63) == 0 && m > 0.f)
        atomicMax(&rowmax[r0], __float_as_uint(m));
    } else if (act && w > 0.f) {
      atomicMax(&rowmax[lo], __float_as_uint(w));
    }
  }
}

// ---- probabilities --------------------------------------------------------
// max(p, max_{t in row i ∩ row j} min(w[i,t], w[j,t])) over two sorted rows
// of one CSR with per-incidence weights w: merge, or probe the shorter row
// against the longer when they differ a lot.
__device__ float row_pair_prob(const int *__restrict__ rp,
                               const int *__restrict__ col,
                               const float *__restrict__ w, int i, int j) {
  int a = rp[i], ae = rp[i + 1], b = rp[j], be = rp[j + 1];
  float p = 0.f;
  if (ae - a > be - b) {
    const int t0 = a, t1 = ae;
    a = b;
    ae = be;
    b = t0;
    be = t1;
  }
  if (be - b > 16 * (ae - a)) {
    for (; a < ae; a++) {
      const int x = find_sorted(col, b, be, col[a]);
      if (x >= 0) p = fmaxf(p, fminf(w[a], w[x]));
    }
    return p;
  }
  while (a < ae && b < be) {
    const int ca = col[a], cb = col[b];
    if (ca < cb) {
      a++;
    } else if (ca > cb) {
      b++;
    } else {
      p = fmaxf(p, fminf(w[a], w[b]));
      a++;
      b++;
    }
  }
  return p;
}

__device__ __forceinline__ int esize(const HobeW &H, int e) {
  return H.rp_e[e + 1] - H.rp_e[e];
}

// One full wave: max(p, ee(e, f)), wave-uniform in and out. Each lane
// probes kEeWays members of the smaller edge at once (their binary searches
// in lockstep: independent load chains), kEeWays * 64 members per step.
constexpr int kEeWays = 4;
__device__ float wave_ee(const HobeW &H, int e, int f, float p, int lane) {
  if (e == f) return fmaxf(p, H.self[e]);
  const float bound = fminf(H.self[e], H.self[f]);
  if (bound <= p) return p;
  int s = e, b = f;
  if (esize(H, e) > esize(H, f)) {
    s = f;
    b = e;
  }
  const int se = H.rp_e[s + 1];
  float lp = p;
  for (int t0 = H.rp_e[s]; t0 < se; t0 += 64 * kEeWays) {
    float ws[kEeWays];
    int lo[kEeWays], hi[kEeWays], end[kEeWays];
#pragma unroll
    for (int k = 0; k < kEeWays; k++) {
      const int t = t0 + k * 64 + lane;
      ws[k] = t < se ? H.we[t] : 0.f;
      const int u = t < se && ws[k] > lp ? H.col_e[t] : -1;
      lo[k] = u >= 0 ? H.rp_n[u] : 0;
      end[k] = u >= 0 ? H.rp_n[u + 1] : 0;
      hi[k] = end[k];
    }
    while (true) {  // lower bound of b in each member's edge list
      bool live = false;
      int v[kEeWays];
#pragma unroll
      for (int k = 0; k < kEeWays; k++) {
        v[k] = lo[k] < hi[k] ? H.col_n[(lo[k] + hi[k]) >> 1] : 0;
        live |= lo[k] < hi[k];
      }
      if (!live) break;
#pragma unroll
      for (int k = 0; k < kEeWays; k++) {
        if (lo[k] < hi[k]) {
          const int mid = (lo[k] + hi[k]) >> 1;
          if (v[k] < b) lo[k] = mid + 1;
          else hi[k] = mid;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kEeWays; k++)
      if (lo[k] < end[k] && H.col_n[lo[k]] == b) lp = fmaxf(lp, fminf(ws[k], H.wn[lo[k]]));
    lp = hgx::wave_max(lp);
    if (lp >= bound) break;
  }
  return lp;
}

// A wave's LDS hash of E(v) (wave_ne's member walk)
constexpr int kNeBits = 9;
constexpr int kNeHash = 1 << kNeBits;
constexpr int kNeCap = kNeHash / 2;
constexpr int kNeRead = 8;
__device__ __forceinline__ unsigned ne_slot(int e) {
  return ((unsigned)e * 2654435761u) >> (32 - kNeBits);
}

#ifdef HGX_DEBUG_KNOBS
// wave_ne branch census (debug builds, hgx_hobe_diag): [branch] pairs,
// [4 + branch] s_memrealtime ticks; branch 0 bound 0, 1 LDS member walk,
// 2 merged member walk, 3 per-edge ee
__device__ unsigned long long g_ne_diag[8];
#endif

// One full wave: ne(v, e) = max over e' in E(v) of ee(e, e'). `ev`: the
// wave's kNeHash ints of LDS.
__device__ float wave_ne(const HobeW &H, int v, int e, int lane, int *ev, int &br) {
  const float bound = H.self[e];
  br = 0;
  if (bound <= 0.f) return 0.f;
  const int vb = H.rp_n[v], ve = H.rp_n[v + 1];
  const int eb = H.rp_e[e], eend = H.rp_e[e + 1], esz = eend - eb;
  long long cost_b = 0;  // probes of (b): sum over E(v) of min(|e|, |e'|)
  for (int t = vb + lane; t < ve; t += 64)
    cost_b += min(esz, esize(H, H.col_n[t]));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cost_b += __shfl_xor(cost_b, off);
  float p = 0.f;
  if ((long long)esz * 4 <= cost_b && ve - vb <= kNeCap) {
    br = 1;
    // (a) members u of e: max over e' in E(u) ∩ E(v) of min(w(e,u), w(u,e')),
    // E(v) in the wave's LDS hash, each member's edge list read straight
    // through (independent loads) instead of merged with E(v)
    for (int k = lane; k < kNeHash; k += 64) ev[k] = -1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int t = vb + lane; t < ve; t += 64) {
      const int f = H.col_n[t];
      unsigned sl = ne_slot(f);
      while (true) {
        const int old = atomicCAS(&ev[sl], -1, f);
        if (old == -1 || old == f) break;
        sl = (sl + 1) & (kNeHash - 1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int t0 = eb; t0 < eend; t0 += 64) {
      const int t = t0 + lane;
      if (t < eend) {
        const float weu = H.we[t];
        if (weu > p) {
          const int u = H.col_e[t];
          const int ae = H.rp_n[u + 1];
          // kNeRead edge ids per step, all loads issued before any probe
          for (int a0 = H.rp_n[u]; a0 < ae; a0 += kNeRead) {
            int f[kNeRead];
#pragma unroll
            for (int j = 0; j < kNeRead; j++) f[j] = a0 + j < ae ? H.col_n[a0 + j] : -1;
#pragma unroll
            for (int j = 0; j < kNeRead; j++) {
              if (f[j] < 0) continue;
              unsigned sl = ne_slot(f[j]);
              int k;
              while ((k = ev[sl]) >= 0 && k != f[j]) sl = (sl + 1) & (kNeHash - 1);
              if (k == f[j]) p = fmaxf(p, fminf(weu, H.wn[a0 + j]));
            }
          }
        }
      }
      p = hgx::wave_max(p);
      if (p >= bound) break;
    }
    // the next pair of this wave rewrites ev: every lane is done reading
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return p;
  }
  br = 3;
  if ((long long)esz * 4 <= cost_b) {
    br = 2;
    // (a) with a long E(v): each member's edge list merged with E(v)
    for (int t0 = eb; t0 < eend; t0 += 64) {
      const int t = t0 + lane;
      if (t < eend) {
        const float weu = H.we[t];
        if (weu > p) {
          const int u = H.col_e[t];
          int a = H.rp_n[u];
          const int ae = H.rp_n[u + 1];
          int b = vb;
          while (a < ae && b < ve) {
            const int ca = H.col_n[a], cb = H.col_n[b];
            if (ca < cb) {
              a++;
            } else if (ca > cb) {
              b++;
            } else {
              p = fmaxf(p, fminf(weu, H.wn[a]));
              a++;
              b++;
            }
          }
        }
      }
      p = hgx::wave_max(p);
      if (p >= bound) break;
    }
    return p;
  }
  // (b) ee(e, e') for every e' in E(v)
  for (int t = vb; t < ve; t++) {
    p = wave_ee(H, e, H.col_n[t], p, lane);
    if (p >= bound) break;
  }
  return p;
}

// Pairs: explicit (pa[q], pb[q]) or records (ids +1 in a record of R ints).
struct PairSrc {
  const int *pa, *pb;  // explicit pairs (nullptr -> records)
  const int *idx;      // records
  int R;
  int64_t base;        // first pair
  float *out;          // explicit: out[q]; records: tgt[(base + q) * 3 + kind]
};

__device__ __forceinline__ void get_pair(const PairSrc &P, int kind, int64_t q,
                                         int &a, int &b) {
  if (P.pa) {
    a = P.pa[q];
    b = P.pb[q];
    return;
  }
  const int *ri = P.idx + (P.base + q) * P.R;
  if (kind == 0) {
    a = ri[0] - 1;
    b = ri[2] - 1;
  } else if (kind == 1) {
    a = ri[1] - 1;
    b = ri[3] - 1;
  } else {
    a = ri[0] - 1;
    b = ri[3] - 1;
  }
}

__device__ __forceinline__ void put_prob(const PairSrc &P, int kind, int64_t q,
                                         float p) {
  if (P.pa) P.out[q] = p;
  else P.out[(P.base + q) * 3 + kind] = p;
}

// node-node: one lane per pair
__global__ void hobe_nn_kernel(HobeW H, PairSrc P, int64_t n) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    int a, b;
    get_pair(P, 0, q, a, b);
    put_prob(P, 0, q, row_pair_prob(H.rp_n, H.col_n, H.wn, a, b));
  }
}

// edge-edge (kind 1) / node-edge (kind 2): one wave per pair
__global__ __launch_bounds__(256) void hobe_wave_kernel(HobeW H, PairSrc P,
                                                        int kind, int64_t n) {
  __shared__ int s_ev[4][kNeHash];  // per wave: wave_ne's E(v) hash
  const int lane = threadIdx.x & 63;
  int *ev = s_ev[threadIdx.x >> 6];
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t q = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
       q < n; q += nw) {
    int a, b;
    get_pair(P, kind, q, a, b);
#ifdef HGX_DEBUG_KNOBS
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
    int br = 0;
    const float p = kind == 1 ? wave_ee(H, a, b, 0.f, lane) : wave_ne(H, a, b, lane, ev, br);
#ifdef HGX_DEBUG_KNOBS
    if (kind == 2 && lane == 0) {
      atomicAdd(&g_ne_diag[br], 1ull);
      atomicAdd(&g_ne_diag[4 + br], __builtin_amdgcn_s_memrealtime() - t0);
    }
#endif
    if (lane == 0) put_prob(P, kind, q, p);
  }
}

int grid_for(int64_t work, int per_block, int cap = 4096) {
  int64_t g = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

HobeW weights_of(hgx_ctx *ctx) {
  return HobeW{ctx->rp_n.as<int>(), ctx->col_n.as<int>(), ctx->rp_e.as<int>(),
               ctx->col_e.as<int>(), ctx->hw_n.as<float>(), ctx->hw_e.as<float>(),
               ctx->hw_self.as<float>()};
}

int launch_probs(hgx_ctx *ctx, int kind, const PairSrc &P, int64_t n) {
  if (n <= 0) return HGX_OK;
  const HobeW H = weights_of(ctx);
  if (kind == 0) {
    hipLaunchKernelGGL(hobe_nn_kernel, dim3(grid_for(n, 256, 16384)), dim3(256),
                       0, ctx->stream, H, P, n);
  } else {
    int dev = 0, ncu = 256;
    HGX_HIP(ctx, hipGetDevice(&dev));
    HGX_HIP(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    hipLaunchKernelGGL(hobe_wave_kernel, dim3(grid_for(n, 4, 8 * ncu)), dim3(256),
                       0, ctx->stream, H, P, kind, n);
  }
  HGX_LAUNCH_CHECK(ctx);
#ifdef HGX_DEBUG_KNOBS
  if (kind == 2 && hgx_debug_env("HGX_NE_DIAG", 0)) {
    unsigned long long d[8];
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    HGX_HIP(ctx, hipMemcpyFromSymbol(d, HIP_SYMBOL(g_ne_diag), sizeof(d)));
    fprintf(stderr, "ne_diag pairs %llu %llu %llu %llu wave_ms %.1f %.1f %.1f %.1f\n",
            d[0], d[1], d[2], d[3], d[4] / 1e5, d[5] / 1e5, d[6] / 1e5, d[7] / 1e5);
  }
#endif
  return HGX_OK;
}

}  // namespace

// Per-incidence HOBE weights of the current alg coords (both orientations)
// and each edge's max weight. Called before every probability pass.
int hgx_hobe_prepare(hgx_ctx *ctx) {
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE, "no alg coordinates on device");
  const int64_t nnz = ctx->nnz;
  HGX_TRY(hgx_ensure(ctx, ctx->hw_n, sizeof(float) * (nnz + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->hw_e, sizeof(float) * (nnz + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->hw_self, sizeof(float) * (ctx->E + 1)));
  HGX_HIP(ctx, hipMemsetAsync(ctx->hw_self.p, 0, sizeof(float) * (ctx->E + 1),
                              ctx->stream));
  if (nnz == 0) return HGX_OK;
  const float *X = ctx->X[ctx->xcur].as<float>();
  const float *Y = ctx->Y[ctx->ycur].as<float>();
  hipLaunchKernelGGL(hobe_weight_kernel, dim3(grid_for(nnz, 256, 65536)),
                     dim3(256), 0, ctx->stream, nnz, ctx->N, ctx->rp_n.as<int>(),
                     ctx->col_n.as<int>(), X, Y, ctx->ks, ctx->k,
                     ctx->hw_n.as<float>(), (unsigned *)nullptr);
  HGX_LAUNCH_CHECK(ctx);
  hipLaunchKernelGGL(hobe_weight_kernel, dim3(grid_for(nnz, 256, 65536)),
                     dim3(256), 0, ctx->stream, nnz, ctx->E, ctx->rp_e.as<int>(),
                     ctx->col_e.as<int>(), Y, X, ctx->ks, ctx->k,
                     ctx->hw_e.as<float>(), ctx->hw_self.as<unsigned>());
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

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
  HGX_TRY(hgx_hobe_prepare(ctx));
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(int32_t) * n));
  HGX_TRY(hgx_ensure(ctx, ctx->s3, sizeof(int32_t) * n));
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * n));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s2.p, a, sizeof(int32_t) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s3.p, b, sizeof(int32_t) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  PairSrc P{ctx->s2.as<int>(), ctx->s3.as<int>(), nullptr, 0, 0,
            ctx->s4.as<float>()};
  HGX_TRY(launch_probs(ctx, kind, P, n));
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
  if (which == 2) {
    HGX_TRY(hgx_hobe_prepare(ctx));
    if (node_major)
      HGX_HIP(ctx, hipMemcpyAsync(node_major, ctx->hw_n.p, sizeof(float) * ctx->nnz,
                                  hipMemcpyDeviceToHost, ctx->stream));
    if (edge_major)
      HGX_HIP(ctx, hipMemcpyAsync(edge_major, ctx->hw_e.p, sizeof(float) * ctx->nnz,
                                  hipMemcpyDeviceToHost, ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return HGX_OK;
  }
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
  for (int pass = 0; pass < 2; pass++) {
    float *host = pass == 0 ? node_major : edge_major;
    if (!host) continue;
    if (pass == 0)
      hipLaunchKernelGGL(incidence_weight_kernel, dim3(grid_for(ctx->N, 256)),
                         dim3(256), 0, ctx->stream, which, alpha,
                         ctx->N, ctx->rp_n.as<int>(), ctx->col_n.as<int>(),
                         nullptr, nullptr, 0, 0, ctx->rp_e.as<int>(), smin, smax,
                         ctx->s4.as<float>());
    else
      hipLaunchKernelGGL(incidence_weight_kernel, dim3(grid_for(ctx->E, 256)),
                         dim3(256), 0, ctx->stream, which, alpha,
                         ctx->E, ctx->rp_e.as<int>(), ctx->col_e.as<int>(),
                         nullptr, nullptr, 0, 0, ctx->rp_n.as<int>(), dmin, dmax,
                         ctx->s4.as<float>());
    HGX_LAUNCH_CHECK(ctx);
    HGX_HIP(ctx, hipMemcpyAsync(host, ctx->s4.p, sizeof(float) * ctx->nnz,
                                hipMemcpyDeviceToHost, ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return HGX_OK;
}

// Used by hgx_sample_hobe_rows (after hgx_hobe_prepare): the probability
// target of records [b, e) of one kind.
int hgx_hobe_fill_probs(hgx_ctx *ctx, int kind, int64_t b, int64_t e) {
  if (e <= b) return HGX_OK;
  PairSrc P{nullptr, nullptr, ctx->rec_idx.as<int>(), 4 + 2 * ctx->K, b,
            ctx->rec_tgt.as<float>()};
  return launch_probs(ctx, kind, P, e - b);
}
