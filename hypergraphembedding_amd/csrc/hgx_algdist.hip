// Algebraic-distance relaxation on MI355X.
//
// Reference: algebraic_distance.py:126-175 (driver), 34-51 (_update_alg_dist:
// weighted mean of neighbour coords, weight 1/deg(neighbour), averaged with
// self), 54-91 (node half, then edge half on the NEW node coords), 97-123
// (joint per-dim min-max rescale of nodes and edges to [0,1]).
//
// HBM layout: coordinates live in rows of KS = round_up(k+1, 4) fp32,
//   row = [w, c_0 .. c_{k-1}, pad]  with w = 1/len(own CSR row),
// so the gather of a source row brings its weight in the same 16-byte
// vectors (no separate random 4-byte load per incidence).
//
// Rescale fusion: iteration t writes RAW values and folds their per-dim
// min/max into mm[t] (order-preserving int32 atomicMax, one set of 2k
// atomics per workgroup). Iteration t+1 applies s_t(z) = (z - min_t) /
// (max_t - min_t) when it reads: self rows always; the node half's gathered
// edge rows as s_t(weighted mean) (the mean is affine); the edge half
// gathers the NEW node rows unscaled, exactly like the reference. A final
// pass applies the last affine in place.
//
// Sharded mode: rank g owns node rows [row0,row1). Per
// iteration: node half on own rows -> edge PARTIAL sums over own nodes
// (local edge sub-CSR, slot 0 = sum of weights) -> caller all-reduces the
// E x KS partial (SUM) -> edge FINAL on all edges -> caller all-reduces the
// 2*KS min/max words (MAX).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "hgx_internal.h"

using hgx::f2ord;
using hgx::ord2f;

namespace {

#ifndef HGX_ALG_BLOCK
#define HGX_ALG_BLOCK 256
#endif
constexpr int kBlock = HGX_ALG_BLOCK;
// min/max words are spread over kRep replicas (workgroup b adds to replica
// b % kRep): 2048 workgroups on one word serialise at the memory-side
// atomic unit (~90 us per sweep); 32 per word do not. Readers fold the
// replicas once per workgroup into LDS.
constexpr int kRep = 64;
enum { MODE_FULL = 0, MODE_PARTIAL = 1 };
// diagnostic ablation bits (HGX_ALG_ABLATE, timing experiments only):
// 1 = skip the min/max flush, 2 = skip the source gathers, 4 = flush
// without its global atomics
#ifdef HGX_DEBUG_KNOBS
__constant__ int g_ablate = 0;  // ablation bits (diagnostic builds only)
// source rows >= g_hot_lim gathered with non-temporal loads (experiment)
__constant__ int g_hot_lim = 0x7fffffff;
#else
static constexpr int g_ablate = 0;
static constexpr int g_hot_lim = 0x7fffffff;
#endif

__device__ __forceinline__ float4 f4fma(float w, float4 v, float4 a) {
  return make_float4(fmaf(w, v.x, a.x), fmaf(w, v.y, a.y), fmaf(w, v.z, a.z),
                     fmaf(w, v.w, a.w));
}
__device__ __forceinline__ float f4get(const float4 &v, int c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}
__device__ __forceinline__ void f4set(float4 &v, int c, float x) {
  if (c == 0) v.x = x;
  else if (c == 1) v.y = x;
  else if (c == 2) v.z = x;
  else v.w = x;
}

// Fold the kRep replicas of the previous iteration's min/max (layout
// [2*KS][kRep]) into s_m (min) and s_d (max - min) for slots 0..KS-1;
// identity when there is no previous iteration. Whole block, ends with a
// barrier.
// s_d = max - min, or 1 / (max - min) when `inverse` (narrow kernels).
__device__ void load_affine(const int *mm_prev, int KS, int k, float *s_m,
                            float *s_d, bool inverse = false) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  static_assert(kRep == 64, "one wave folds one slot");
  constexpr int W = kBlock / 64;
  constexpr int B = 8;  // slots per wave per batch: all loads issued first
  for (int i0 = wave; i0 < KS; i0 += W * B) {
    int mx[B], mn[B];
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int i = i0 + W * b;
      const bool live = mm_prev && i >= 1 && i <= k && i < KS;
      mx[b] = live ? mm_prev[(size_t)i * kRep + lane] : 0;
      mn[b] = live ? mm_prev[(size_t)(KS + i) * kRep + lane] : 0;
    }
#pragma unroll
    for (int b = 0; b < B; b++) {
      mx[b] = hgx::wave_max_i(mx[b]);
      mn[b] = hgx::wave_max_i(mn[b]);
    }
    if (lane == 0) {
#pragma unroll
      for (int b = 0; b < B; b++) {
        const int i = i0 + W * b;
        if (i < KS) {
          float m = 0.f, dl = 1.f;
          if (mm_prev && i >= 1 && i <= k) {
            m = ord2f(~mn[b]);
            dl = ord2f(mx[b]) - m;
          }
          s_m[i] = m;
          s_d[i] = inverse ? 1.0f / dl : dl;
        }
      }
    }
  }
  __syncthreads();
}

// Block-wide min/max of per-thread partials -> 2k atomics per workgroup.
// Whole-wave DPP reductions (hgx::wave_min/max: no LDS traffic; ds_bpermute
// shuffles queued on the LDS pipe at the tail). Measured on C3 (r01): LDS
// atomics instead of the wave reductions let every block reach its global
// atomics at the same moment and the burst on the replica lines cost more
// (12.5 vs 1.8 us per iteration).
template <int KS>
__device__ __forceinline__ void flush_minmax(const float (&lmn)[KS],
                                             const float (&lmx)[KS], int k,
                                             int *mm_cur) {
  __shared__ float s_red[2][kBlock / 64][KS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int i = 1; i < KS; i++) {
    float a = lmn[i], b = lmx[i];
    if (i <= k) {  // wave-uniform
      a = hgx::wave_min(a);
      b = hgx::wave_max(b);
    }
    if (lane == 0) {
      s_red[0][wave][i] = a;
      s_red[1][wave][i] = b;
    }
  }
  __syncthreads();
  if (tid >= 1 && tid <= k) {
    float a = INFINITY, b = -INFINITY;
#pragma unroll
    for (int w = 0; w < kBlock / 64; w++) {
      a = fminf(a, s_red[0][w][tid]);
      b = fmaxf(b, s_red[1][w][tid]);
    }
    if (b >= a && !(g_ablate & 4)) {
      const int r = blockIdx.x % kRep;
      atomicMax(&mm_cur[(size_t)tid * kRep + r], f2ord(b));
      atomicMax(&mm_cur[(size_t)(KS + tid) * kRep + r], ~f2ord(a));
    }
  }
}

// Sampled min/max (hgx_alg_run, every iteration but the last): the k
// argument carries kSampleFlush and only workgroups < kRep flush. The
// per-iteration rescale is a per-dimension increasing affine map applied
// to nodes and edges alike, and both half-updates (a normalised weighted
// mean averaged with self) commute with such maps, so any intermediate
// affine gives the same final, exactly normalised, coordinates up to
// rounding: the intermediate rescale only has to keep the values O(1),
// which a sample of rows does. The last iteration flushes every workgroup
// and final_affine applies its exact min/max (algebraic_distance.py:97-123).
constexpr int kSampleFlush = 1 << 24;
#define HGX_FLUSH_SEL(k)                                 \
  const bool fskip_ = ((k) & kSampleFlush) && blockIdx.x >= kRep; \
  (k) &= kSampleFlush - 1

// One CSR half-sweep over rows [row0, row0+R), narrow rows (KS <= 20):
// G lanes per destination row; each lane strides the row's incidences with
// two gathers in flight and keeps all KS accumulators in registers; an
// xor-shuffle reduction over the G lanes; lane 0 of the group writes.
//   MODE_FULL:    out[r] = [1/len, (s(self) + s?(sum w*src / sum w)) / 2]
//   MODE_PARTIAL: out[r] = [sum w, sum w*src]    (no self, no min/max)
template <int KS, int G, int MODE, int M>
__global__ __launch_bounds__(kBlock) void algdist_half_narrow(
    int row0, int R, const int *__restrict__ rp, const int *__restrict__ col,
    const float *__restrict__ self_in, const float *__restrict__ src,
    float *__restrict__ out, const int *__restrict__ mm_prev, int src_affine,
    int *__restrict__ mm_cur, int k, int long_thresh) {
  HGX_FLUSH_SEL(k);
  constexpr int NV = KS / 4;
  __shared__ float s_m[KS], s_d[KS];
  load_affine(mm_prev, KS, k, s_m, s_d, true);
  const int tid = threadIdx.x;
  const int lg = tid % G;
  constexpr int GPB = kBlock / G;
  const int ngroups = gridDim.x * GPB;
  float lmn[KS], lmx[KS];
#pragma unroll
  for (int i = 0; i < KS; i++) {
    lmn[i] = INFINITY;
    lmx[i] = -INFINITY;
  }
  const float4 *src4 = reinterpret_cast<const float4 *>(src);
  for (int rr = blockIdx.x * GPB + tid / G; rr < R; rr += ngroups) {
    const int r = row0 + rr;
    const int beg = rp[r], end = rp[r + 1];
    if (end - beg > long_thresh) continue;  // seg_partial + long_finish
    // own row early (MODE_FULL): its latency hides under the gathers
    // lane lg owns output vectors j = lg, lg + G, ...
    float4 self[NV];
    if (MODE == MODE_FULL) {
      const float4 *sp = reinterpret_cast<const float4 *>(self_in) + (size_t)r * NV;
#pragma unroll
      for (int j = 0; j < NV; j++)
        if (j % G == lg) self[j] = sp[j];
    }
    float4 acc[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    float wsum = 0.f;
    for (int base = beg + lg; base < end; base += G * M) {
      int c[M];
#pragma unroll
      for (int m = 0; m < M; m++) {
        const int t = base + G * m;
        c[m] = t < end ? ((g_ablate & 2) ? -2 : col[t]) : -1;
      }
      float4 v[M][NV];
#pragma unroll
      for (int m = 0; m < M; m++) {
        if (c[m] >= 0) {
#pragma unroll
          for (int j = 0; j < NV; j++) v[m][j] = src4[(size_t)c[m] * NV + j];
        }
      }
#pragma unroll
      for (int m = 0; m < M; m++) {
        if (c[m] >= 0) {
          const float w = v[m][0].x;
          wsum += w;
#pragma unroll
          for (int j = 0; j < NV; j++) acc[j] = f4fma(w, v[m][j], acc[j]);
        }
      }
    }
    wsum = hgx::group_allreduce_sum<G>(wsum);
#pragma unroll
    for (int j = 0; j < NV; j++) {
      acc[j].x = hgx::group_allreduce_sum<G>(acc[j].x);
      acc[j].y = hgx::group_allreduce_sum<G>(acc[j].y);
      acc[j].z = hgx::group_allreduce_sum<G>(acc[j].z);
      acc[j].w = hgx::group_allreduce_sum<G>(acc[j].w);
    }
    {
      float4 *op = reinterpret_cast<float4 *>(out) + (size_t)r * NV;
      if (MODE == MODE_PARTIAL) {
        acc[0].x = wsum;
#pragma unroll
        for (int j = 0; j < NV; j++)
          if (j % G == lg) op[j] = acc[j];
      } else {
        // one reciprocal per row; per-dim 1/(max-min) comes from LDS
        const float inv_w = 1.0f / wsum;
#pragma unroll
        for (int j = 0; j < NV; j++) {
          if (j % G != lg) continue;
          const float4 s = self[j];
          float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const int i = 4 * j + c;
            float v;
            if (i == 0) {
              v = 1.0f / (float)(end - beg);
            } else if (i <= k) {
              const float sv = (f4get(s, c) - s_m[i]) * s_d[i];
              float mv = f4get(acc[j], c) * inv_w;
              if (src_affine) mv = (mv - s_m[i]) * s_d[i];
              v = (sv + mv) * 0.5f;
              lmn[i] = fminf(lmn[i], v);
              lmx[i] = fmaxf(lmx[i], v);
            } else {
              v = 0.f;
            }
            f4set(o, c, v);
          }
          op[j] = o;
        }
      }
    }
  }
  if (MODE == MODE_FULL && !(g_ablate & 1) && !fskip_)
    flush_minmax<KS>(lmn, lmx, k, mm_cur);
}

// Same half-sweep with the source row split over a QUAD of lanes (KS <= 16):
// lane p of a quad gathers float4 p of the row (p < KS/4), so one load
// instruction touches 16 source rows as 1-2 whole 64-B sectors each instead
// of 64 rows x one 16-B piece per instruction (3 instructions per 48-B row in
// algdist_half_narrow). On an L2-resident source table (C3) the sweep is bound
// by L2 requests, and this cuts them from 3 to ~1.4 per incidence
// (tools/gather_tablesize.hip measures the 4-lane pattern). G = 4Q lanes per
// destination row: quad q of the group strides the row's incidences
// q, q + Q, ... with M in flight; the weight (vector 0, .x) is broadcast
// from lane 0 of the quad by DPP; the Q partial sums of each lane position
// are added by xor shuffles over lane offsets 4 .. G/2.
template <int G>
__device__ __forceinline__ float quad_stride_sum(float x) {
#pragma unroll
  for (int off = 4; off < G; off <<= 1) x += __shfl_xor(x, off);
  return x;
}

typedef float nt_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_load4(const float4 *p) {
  const nt_f4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f4 *>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// Push form of the edge half (tuning alg_push, single GPU): the node half
// (PM_PUSH) also writes every incidence's contribution row [w_v, w_v * x_v]
// (w_v = 1/deg v, x_v its NEW raw coords: what the edge half would gather)
// to contrib[tpos[t]], tpos = the incidence's position in the edge-major
// CSR; the edge half (PM_STREAM) then reads its rows' contributions
// sequentially in CSR order instead of gathering node rows (the gathers of
// the 480 MB node table hit L2 2.6% of the time at C4). Scattered stores do
// not stall the wave; the stream is coalesced.
enum { PM_GATHER = 0, PM_STREAM = 1, PM_PUSH = 2 };

template <int KS, int G, int MODE, int M, int PM = PM_GATHER>
__global__ __launch_bounds__(kBlock) void algdist_half_quad(
    int row0, int R, const int *__restrict__ rp, const int *__restrict__ col,
    const float *__restrict__ self_in, const float *__restrict__ src,
    float *__restrict__ out, const int *__restrict__ mm_prev, int src_affine,
    int *__restrict__ mm_cur, int k, int long_thresh,
    const int *__restrict__ tpos, float *__restrict__ contrib) {
  HGX_FLUSH_SEL(k);
  static_assert(PM == PM_GATHER || MODE == MODE_FULL, "push / stream: full rows");
  constexpr int NV = KS / 4, Q = G / 4;
  static_assert(NV >= 1 && NV <= 4 && G >= 4, "one float4 per lane");
  __shared__ float s_m[KS], s_d[KS];
  load_affine(mm_prev, KS, k, s_m, s_d, true);
  const int tid = threadIdx.x;
  const int lg = tid % G, p = lg & 3, qi = lg >> 2;
  const bool vl = p < NV;  // this lane carries vector p of a row
  constexpr int GPB = kBlock / G;
  const int ngroups = gridDim.x * GPB;
  float lmn[4], lmx[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    lmn[c] = INFINITY;
    lmx[c] = -INFINITY;
  }
  const float4 *src4 = reinterpret_cast<const float4 *>(src);
  for (int rr = blockIdx.x * GPB + tid / G; rr < R; rr += ngroups) {
    const int r = row0 + rr;
    const int beg = rp[r], end = rp[r + 1];
    if (end - beg > long_thresh) continue;  // seg_partial + long_finish
    float4 self = make_float4(0.f, 0.f, 0.f, 0.f);
    // push: every quad finishes the row (it writes a share of the
    // contributions); the same self row, from L2
    if (MODE == MODE_FULL && (qi == 0 || PM == PM_PUSH) && vl)
      self = reinterpret_cast<const float4 *>(self_in)[(size_t)r * NV + p];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float wsum = 0.f;
    for (int base = beg + qi; base < end; base += Q * M) {
      int c[M];
#pragma unroll
      for (int m = 0; m < M; m++) {
        const int t = base + Q * m;
        // stream: the source row is the incidence's own contribution row
        c[m] = t < end ? (PM == PM_STREAM ? t : (g_ablate & 2) ? -2 : col[t]) : -1;
      }
      float4 v[M];
#pragma unroll
      for (int m = 0; m < M; m++) {
        v[m] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c[m] >= 0 && vl) {
          if (c[m] < g_hot_lim) v[m] = src4[(size_t)c[m] * NV + p];
          else v[m] = nt_load4(&src4[(size_t)c[m] * NV + p]);
        }
      }
#pragma unroll
      for (int m = 0; m < M; m++) {
        // weight = vector 0 .x of the row, held by lane 0 of the quad
        const float w = hgx::dpp_f<0x00>(v[m].x);  // quad_perm [0,0,0,0]
        if (c[m] >= 0) {
          wsum += w;
          if (PM == PM_STREAM) {  // pre-multiplied [w, w*x]
            acc.x += v[m].x;
            acc.y += v[m].y;
            acc.z += v[m].z;
            acc.w += v[m].w;
          } else {
            acc = f4fma(w, v[m], acc);
          }
        }
      }
    }
    wsum = quad_stride_sum<G>(wsum);
    acc.x = quad_stride_sum<G>(acc.x);
    acc.y = quad_stride_sum<G>(acc.y);
    acc.z = quad_stride_sum<G>(acc.z);
    acc.w = quad_stride_sum<G>(acc.w);
    if ((qi == 0 || PM == PM_PUSH) && vl) {
      float4 *op = reinterpret_cast<float4 *>(out) + (size_t)r * NV + p;
      if (MODE == MODE_PARTIAL) {
        if (p == 0) acc.x = wsum;
        *op = acc;
      } else {
        const float inv_w = 1.0f / wsum;
        float4 o;
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const int i = 4 * p + c;
          float v;
          if (i == 0) {
            v = 1.0f / (float)(end - beg);
          } else if (i <= k) {
            const float sv = (f4get(self, c) - s_m[i]) * s_d[i];
            float mv = f4get(acc, c) * inv_w;
            if (src_affine) mv = (mv - s_m[i]) * s_d[i];
            v = (sv + mv) * 0.5f;
            lmn[c] = fminf(lmn[c], v);
            lmx[c] = fmaxf(lmx[c], v);
          } else {
            v = 0.f;
          }
          f4set(o, c, v);
        }
        if (qi == 0) *op = o;
        if (PM == PM_PUSH) {
          // contribution rows [w, w*x_1..k, 0] of this quad's incidences
          const float w = 1.0f / (float)(end - beg);
          float4 cv = make_float4(w * o.x, w * o.y, w * o.z, w * o.w);
          if (p == 0) cv.x = w;
          float4 *c4 = reinterpret_cast<float4 *>(contrib);
          for (int t = beg + qi; t < end; t += Q)
            c4[(size_t)tpos[t] * NV + p] = cv;
        }
      }
    }
  }
  if (MODE == MODE_FULL && !(g_ablate & 1) && !fskip_) {
    // lane position p holds components 4p .. 4p+3
    float mn[KS], mx[KS];
#pragma unroll
    for (int i = 0; i < KS; i++) {
      mn[i] = (i / 4 == p) ? lmn[i % 4] : INFINITY;
      mx[i] = (i / 4 == p) ? lmx[i % 4] : -INFINITY;
    }
    flush_minmax<KS>(mn, mx, k, mm_cur);
  }
}

// Long rows, step 1: one wave per piece of `T` incidences of a long row
// (LongRows): part[piece] = [sum w, sum w*src] over the piece, raw sums (the
// affine of a scaled source commutes with the weighted mean; long_finish
// applies it).
// PRE (push form): src holds the pre-multiplied contribution rows [w, w*x]
// in CSR order, read in sequence instead of gathered through col.
template <int KS, int M, bool PRE = false>
__global__ __launch_bounds__(kBlock) void algdist_seg_partial(
    int nseg, const int2 *__restrict__ seg, int T, const int *__restrict__ rp,
    const int *__restrict__ col, const float *__restrict__ src,
    float *__restrict__ part) {
  constexpr int NV = KS / 4;
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (kBlock / 64);
  const float4 *src4 = reinterpret_cast<const float4 *>(src);
  float4 *part4 = reinterpret_cast<float4 *>(part);
  for (int s = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); s < nseg; s += nw) {
    const int2 sg = seg[s];
    const int beg = rp[sg.x] + sg.y * T, end = min(rp[sg.x + 1], beg + T);
    float4 acc[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    float wsum = 0.f;
    for (int base = beg + lane; base < end; base += 64 * M) {
      int c[M];
#pragma unroll
      for (int m = 0; m < M; m++) {
        const int t = base + 64 * m;
        c[m] = t < end ? (PRE ? t : col[t]) : -1;
      }
      float4 v[M][NV];
#pragma unroll
      for (int m = 0; m < M; m++)
        if (c[m] >= 0) {
#pragma unroll
          for (int j = 0; j < NV; j++) v[m][j] = src4[(size_t)c[m] * NV + j];
        }
#pragma unroll
      for (int m = 0; m < M; m++)
        if (c[m] >= 0) {
          const float w = v[m][0].x;
          wsum += w;
#pragma unroll
          for (int j = 0; j < NV; j++) {
            if (PRE) {
              acc[j].x += v[m][j].x;
              acc[j].y += v[m][j].y;
              acc[j].z += v[m][j].z;
              acc[j].w += v[m][j].w;
            } else {
              acc[j] = f4fma(w, v[m][j], acc[j]);
            }
          }
        }
    }
    wsum = hgx::group_allreduce_sum<64>(wsum);
#pragma unroll
    for (int j = 0; j < NV; j++) {
      acc[j].x = hgx::group_allreduce_sum<64>(acc[j].x);
      acc[j].y = hgx::group_allreduce_sum<64>(acc[j].y);
      acc[j].z = hgx::group_allreduce_sum<64>(acc[j].z);
      acc[j].w = hgx::group_allreduce_sum<64>(acc[j].w);
    }
    acc[0].x = wsum;
#pragma unroll
    for (int j = 0; j < NV; j++)
      if (j == lane) part4[(size_t)s * NV + j] = acc[j];
  }
}

// Long rows, step 2: one wave per long row sums its pieces (lane-strided,
// then a fixed tree: deterministic) and writes the row like the narrow
// kernel's output stage (MODE_FULL, with min/max) or its partial
// (MODE_PARTIAL).
template <int KS, int MODE>
__global__ __launch_bounds__(kBlock) void algdist_long_finish(
    int nlong, const int *__restrict__ lrows, const int *__restrict__ loff,
    const float *__restrict__ part, const int *__restrict__ rp,
    const float *__restrict__ self_in, float *__restrict__ out,
    const int *__restrict__ mm_prev, int src_affine, int *__restrict__ mm_cur,
    int k) {
  HGX_FLUSH_SEL(k);
  constexpr int NV = KS / 4;
  __shared__ float s_m[KS], s_d[KS];
  load_affine(mm_prev, KS, k, s_m, s_d, true);
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (kBlock / 64);
  const float4 *part4 = reinterpret_cast<const float4 *>(part);
  float lmn[KS], lmx[KS];
#pragma unroll
  for (int i = 0; i < KS; i++) {
    lmn[i] = INFINITY;
    lmx[i] = -INFINITY;
  }
  for (int j = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); j < nlong; j += nw) {
    const int r = lrows[j], s0 = loff[j], s1 = loff[j + 1];
    float4 acc[NV];
#pragma unroll
    for (int q = 0; q < NV; q++) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = s0 + lane; s < s1; s += 64) {
#pragma unroll
      for (int q = 0; q < NV; q++) {
        const float4 p = part4[(size_t)s * NV + q];
        acc[q].x += p.x;
        acc[q].y += p.y;
        acc[q].z += p.z;
        acc[q].w += p.w;
      }
    }
#pragma unroll
    for (int q = 0; q < NV; q++) {
      acc[q].x = hgx::group_allreduce_sum<64>(acc[q].x);
      acc[q].y = hgx::group_allreduce_sum<64>(acc[q].y);
      acc[q].z = hgx::group_allreduce_sum<64>(acc[q].z);
      acc[q].w = hgx::group_allreduce_sum<64>(acc[q].w);
    }
    float4 *op = reinterpret_cast<float4 *>(out) + (size_t)r * NV;
    if (MODE == MODE_PARTIAL) {
#pragma unroll
      for (int q = 0; q < NV; q++)
        if (q == lane) op[q] = acc[q];
      continue;
    }
    const float inv_w = 1.0f / acc[0].x;
    const int len = rp[r + 1] - rp[r];
    const float4 *sp = reinterpret_cast<const float4 *>(self_in) + (size_t)r * NV;
#pragma unroll
    for (int q = 0; q < NV; q++) {
      if (q != lane) continue;
      const float4 sv4 = sp[q];
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int i = 4 * q + c;
        float v;
        if (i == 0) {
          v = 1.0f / (float)len;
        } else if (i <= k) {
          const float sv = (f4get(sv4, c) - s_m[i]) * s_d[i];
          float mv = f4get(acc[q], c) * inv_w;
          if (src_affine) mv = (mv - s_m[i]) * s_d[i];
          v = (sv + mv) * 0.5f;
          lmn[i] = fminf(lmn[i], v);
          lmx[i] = fmaxf(lmx[i], v);
        } else {
          v = 0.f;
        }
        f4set(o, c, v);
      }
      op[q] = o;
    }
  }
  if (MODE == MODE_FULL && !fskip_) flush_minmax<KS>(lmn, lmx, k, mm_cur);
}

// Incidence-parallel half-sweep for narrow rows (KS <= 20). Rows are cut
// into row-blocks (<= kBlkRows whole rows, <= kBlkNnz incidences; a longer
// row is a block by itself). One wave owns a block: its lanes take
// consecutive incidences (coalesced col loads, kFlatU windows of gathers in
// flight per lane), fold w*src into per-row LDS accumulators, then one lane
// per row finishes: MODE_FULL writes [1/len, (s(self) + s?(mean)) / 2] and
// tracks min/max; MODE_PARTIAL writes [sum w, sum w*src].
constexpr int kFlatU = 4;
constexpr int kBlkRows = 64;   // keep in sync with hgx_make_row_blocks
constexpr int kBlkNnz = 256;

template <int KS, int MODE>
__global__ __launch_bounds__(kBlock) void algdist_half_flat(
    int nblk, const int *__restrict__ blk, const int *__restrict__ rp,
    const int *__restrict__ col, const float *__restrict__ self_in,
    const float *__restrict__ src, float *__restrict__ out,
    const int *__restrict__ mm_prev, int src_affine, int *__restrict__ mm_cur,
    int k) {
  HGX_FLUSH_SEL(k);
  constexpr int NV = KS / 4;
  constexpr int W = kBlock / 64;
  constexpr int AS = KS + 1;  // odd stride: conflict-free per-row reads
  __shared__ float s_acc[W][kBlkRows * AS];
  __shared__ int s_rp[W][kBlkRows + 1];
  __shared__ float s_m[KS], s_d[KS];
  load_affine(mm_prev, KS, k, s_m, s_d, true);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float lmn[KS], lmx[KS];
#pragma unroll
  for (int i = 0; i < KS; i++) {
    lmn[i] = INFINITY;
    lmx[i] = -INFINITY;
  }
  const float4 *src4 = reinterpret_cast<const float4 *>(src);
  float *acc = s_acc[wv];
  int *srp = s_rp[wv];
  for (int b = blockIdx.x * W + wv; b < nblk; b += gridDim.x * W) {
    const int rA = blk[b], nr = blk[b + 1] - rA;
    for (int i = lane; i <= nr; i += 64) srp[i] = rp[rA + i];
    for (int i = lane; i < nr * AS; i += 64) acc[i] = 0.f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int tA = srp[0], tB = srp[nr];
    for (int base = tA; base < tB; base += 64 * kFlatU) {  // wave-uniform
      const int t0 = base + lane;
      int c[kFlatU];
#pragma unroll
      for (int u = 0; u < kFlatU; u++) {
        const int t = t0 + 64 * u;
        c[u] = t < tB ? ((g_ablate & 2) ? -2 : col[t]) : -1;
      }
      float4 v[kFlatU][NV];
#pragma unroll
      for (int u = 0; u < kFlatU; u++)
        if (c[u] >= 0) {
#pragma unroll
          for (int j = 0; j < NV; j++) v[u][j] = src4[(size_t)c[u] * NV + j];
        }
#pragma unroll
      for (int u = 0; u < kFlatU; u++) {
        const int t = t0 + 64 * u;
        // local row of incidence t: last i with srp[i] <= t (-1: no incidence)
        int rl = -1;
        if (c[u] >= 0) {
          int lo = 0, hi = nr - 1;
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (srp[mid] <= t) lo = mid;
            else hi = mid - 1;
          }
          rl = lo;
        }
        // segmented inclusive scan over the wave: a row's incidences are
        // consecutive lanes, so its sum lands in the row's last lane
        float val[KS];
        const float w = c[u] >= 0 ? v[u][0].x : 0.f;
        val[0] = w;
#pragma unroll
        for (int j = 0; j < NV; j++)
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int i = 4 * j + q;
            if (i >= 1) val[i] = (c[u] >= 0 && i <= k) ? w * f4get(v[u][j], q) : 0.f;
          }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int pr = __shfl_up(rl, d);
          const bool add = lane >= d && pr == rl;
#pragma unroll
          for (int i = 0; i < KS; i++) {
            const float o = __shfl_up(val[i], d);
            if (add) val[i] += o;
          }
        }
        const int nx = __shfl_down(rl, 1);
        if (rl >= 0 && (lane == 63 || nx != rl)) {
          float *ar = acc + rl * AS;
#pragma unroll
          for (int i = 0; i < KS; i++)
            if (i <= k) ar[i] += val[i];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int l = lane; l < nr; l += 64) {
      const int r = rA + l;
      const float *ar = acc + l * AS;
      float4 *op = reinterpret_cast<float4 *>(out) + (size_t)r * NV;
      if (MODE == MODE_PARTIAL) {
#pragma unroll
        for (int j = 0; j < NV; j++) {
          float4 o;
#pragma unroll
          for (int q = 0; q < 4; q++) f4set(o, q, ar[4 * j + q]);
          op[j] = o;
        }
      } else {
        const float4 *sp = reinterpret_cast<const float4 *>(self_in) + (size_t)r * NV;
        const float inv_w = 1.0f / ar[0];
#pragma unroll
        for (int j = 0; j < NV; j++) {
          const float4 sv4 = sp[j];
          float4 o;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int i = 4 * j + q;
            float v;
            if (i == 0) {
              v = 1.0f / (float)(srp[l + 1] - srp[l]);
            } else if (i <= k) {
              const float sv = (f4get(sv4, q) - s_m[i]) * s_d[i];
              float mv = ar[i] * inv_w;
              if (src_affine) mv = (mv - s_m[i]) * s_d[i];
              v = (sv + mv) * 0.5f;
              lmn[i] = fminf(lmn[i], v);
              lmx[i] = fmaxf(lmx[i], v);
            } else {
              v = 0.f;
            }
            f4set(o, q, v);
          }
          op[j] = o;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (MODE == MODE_FULL && !(g_ablate & 1) && !fskip_)
    flush_minmax<KS>(lmn, lmx, k, mm_cur);
}

// Wide rows (k > 19): one wave per destination row, the row's float4
// vectors spread over the lanes, incidences walked in order.
template <int MODE>
__global__ __launch_bounds__(kBlock) void algdist_half_wide(
    int row0, int R, int KS, const int *__restrict__ rp,
    const int *__restrict__ col, const float *__restrict__ self_in,
    const float *__restrict__ src, float *__restrict__ out,
    const int *__restrict__ mm_prev, int src_affine, int *__restrict__ mm_cur,
    int k) {
  HGX_FLUSH_SEL(k);
  const int NV = KS / 4;
  __shared__ float s_m[2048], s_d[2048];
  load_affine(mm_prev, KS, k, s_m, s_d);
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (kBlock / 64);
  constexpr int MAXV = 8;  // up to 64*8*4 = 2048 floats per row
  float lmn[MAXV * 4], lmx[MAXV * 4];
#pragma unroll
  for (int i = 0; i < MAXV * 4; i++) {
    lmn[i] = INFINITY;
    lmx[i] = -INFINITY;
  }
  const float4 *src4 = reinterpret_cast<const float4 *>(src);
  for (int rr = wid; rr < R; rr += nw) {
    const int r = row0 + rr;
    const int beg = rp[r], end = rp[r + 1];
    float4 acc[MAXV];
#pragma unroll
    for (int q = 0; q < MAXV; q++) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    float wsum = 0.f;
    constexpr int U = 8;  // incidences in flight per wave
    for (int t0 = beg; t0 < end; t0 += U) {
      int c[U];
      float w[U];
#pragma unroll
      for (int u = 0; u < U; u++) c[u] = t0 + u < end ? col[t0 + u] : -1;
#pragma unroll
      for (int u = 0; u < U; u++) w[u] = c[u] >= 0 ? src[(size_t)c[u] * KS] : 0.f;
#pragma unroll
      for (int q = 0; q < MAXV; q++) {
        const int j = lane + 64 * q;
        if (j < NV) {
          float4 v[U];
#pragma unroll
          for (int u = 0; u < U; u++)
            v[u] = c[u] >= 0 ? src4[(size_t)c[u] * NV + j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int u = 0; u < U; u++) acc[q] = f4fma(w[u], v[u], acc[q]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) wsum += w[u];
    }
    const float own_w = 1.0f / (float)(end - beg);
#pragma unroll
    for (int q = 0; q < MAXV; q++) {
      const int j = lane + 64 * q;
      if (j >= NV) continue;
      float4 o;
      if (MODE == MODE_PARTIAL) {
        o = acc[q];
        if (j == 0) o.x = wsum;
      } else {
        const float4 s = reinterpret_cast<const float4 *>(self_in)[(size_t)r * NV + j];
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const int i = 4 * j + c;
          float v = 0.f;
          if (i == 0) {
            v = own_w;
          } else if (i <= k) {
            const float m = s_m[i], dl = s_d[i];
            const float sv = (f4get(s, c) - m) / dl;
            float mv = f4get(acc[q], c) / wsum;
            if (src_affine) mv = (mv - m) / dl;
            v = (sv + mv) * 0.5f;
            lmn[4 * q + c] = fminf(lmn[4 * q + c], v);
            lmx[4 * q + c] = fmaxf(lmx[4 * q + c], v);
          }
          f4set(o, c, v);
        }
      }
      reinterpret_cast<float4 *>(out)[(size_t)r * NV + j] = o;
    }
  }
  if (MODE == MODE_PARTIAL || fskip_) return;
#pragma unroll
  for (int q = 0; q < MAXV; q++) {
    const int j = lane + 64 * q;
    if (j >= NV) continue;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int i = 4 * j + c;
      if (i >= 1 && i <= k && lmx[4 * q + c] >= lmn[4 * q + c]) {
        const int r = (int)((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) % kRep);
        atomicMax(&mm_cur[(size_t)i * kRep + r], f2ord(lmx[4 * q + c]));
        atomicMax(&mm_cur[(size_t)(KS + i) * kRep + r], ~f2ord(lmn[4 * q + c]));
      }
    }
  }
}

// Sharded edge half, after the caller's SUM all-reduce of the partials:
// y'_e = (s(y_e) + P[e][1..k] / P[e][0]) / 2, min/max into mm_cur.
__global__ __launch_bounds__(kBlock) void algdist_edge_final(
    int E, int KS, int k, const int *__restrict__ rp_e,
    const float *__restrict__ self_in, const float *__restrict__ part,
    float *__restrict__ out, const int *__restrict__ mm_prev,
    int *__restrict__ mm_cur) {
  __shared__ int s_mm[4096];  // 2 * KS, KS <= 2048
  __shared__ float s_m[2048], s_d[2048];
  for (int i = threadIdx.x; i < 2 * KS; i += blockDim.x) s_mm[i] = INT_MIN;
  load_affine(mm_prev, KS, k, s_m, s_d);
  const int64_t total = (int64_t)E * KS;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(q / KS), i = (int)(q % KS);
    float v = 0.f;
    if (i == 0) {
      v = 1.0f / (float)(rp_e[e + 1] - rp_e[e]);
    } else if (i <= k) {
      const float sv = (self_in[q] - s_m[i]) / s_d[i];
      const float mv = part[q] / part[(int64_t)e * KS];
      v = (sv + mv) * 0.5f;
      atomicMax(&s_mm[i], f2ord(v));
      atomicMax(&s_mm[KS + i], ~f2ord(v));
    }
    out[q] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * KS; i += blockDim.x) {
    const int s = i % KS;
    if (s >= 1 && s <= k && s_mm[i] != INT_MIN)
      atomicMax(&mm_cur[(size_t)i * kRep + blockIdx.x % kRep], s_mm[i]);
  }
}

// Compact exchange: the shared edges' partial rows [sum w, sum w x_1..k]
// (k + 1 floats, no padding slot) gathered onto the wire.
__global__ void algdist_wire_pack(int e0, int E, int KS, int k,
                                  const int *__restrict__ slot,
                                  const float *__restrict__ part,
                                  float *__restrict__ wire) {
  const int64_t total = (int64_t)E * (k + 1);
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int e = e0 + (int)(q / (k + 1)), i = (int)(q % (k + 1));
    const int s = slot[e];
    if (s >= 0) wire[(int64_t)s * (k + 1) + i] = part[(int64_t)e * KS + i];
  }
}

// algdist_edge_final over the compact exchange: shared edges read their
// reduced row from the wire, this rank's private edges their local partial,
// other ranks' private edges are skipped (never read by this rank's node
// rows; gathered once after the last iteration).
__global__ __launch_bounds__(kBlock) void algdist_edge_final_wire(
    int E, int KS, int k, const int *__restrict__ rp_e,
    const float *__restrict__ self_in, const float *__restrict__ part,
    const float *__restrict__ wire, const int *__restrict__ slot,
    float *__restrict__ out, const int *__restrict__ mm_prev,
    int *__restrict__ mm_cur) {
  __shared__ int s_mm[4096];
  __shared__ float s_m[2048], s_d[2048];
  for (int i = threadIdx.x; i < 2 * KS; i += blockDim.x) s_mm[i] = INT_MIN;
  load_affine(mm_prev, KS, k, s_m, s_d);
  const int64_t total = (int64_t)E * KS;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(q / KS), i = (int)(q % KS);
    const int sl = slot[e];
    if (sl == -2) continue;
    const float *P = sl >= 0 ? wire + (int64_t)sl * (k + 1) : part + (int64_t)e * KS;
    float v = 0.f;
    if (i == 0) {
      v = 1.0f / (float)(rp_e[e + 1] - rp_e[e]);
    } else if (i <= k) {
      const float sv = (self_in[q] - s_m[i]) / s_d[i];
      const float mv = P[i] / P[0];
      v = (sv + mv) * 0.5f;
      atomicMax(&s_mm[i], f2ord(v));
      atomicMax(&s_mm[KS + i], ~f2ord(v));
    }
    out[q] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * KS; i += blockDim.x) {
    const int s = i % KS;
    if (s >= 1 && s <= k && s_mm[i] != INT_MIN)
      atomicMax(&mm_cur[(size_t)i * kRep + blockIdx.x % kRep], s_mm[i]);
  }
}

// dense R x k  ->  rows [1/len, c_0..c_{k-1}, 0...] of KS floats
__global__ void pack_rows(int R, int k, int KS, const int *__restrict__ rp,
                          const float *__restrict__ dense,
                          float *__restrict__ rows) {
  const int64_t total = (int64_t)R * KS;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / KS), s = (int)(i % KS);
    float v = 0.f;
    if (s == 0) v = 1.0f / (float)(rp[r + 1] - rp[r]);
    else if (s <= k) v = dense[(int64_t)r * k + (s - 1)];
    rows[i] = v;
  }
}

// In place on rows [row0, row0+R): apply the affine of mm to slots 1..k.
__global__ __launch_bounds__(kBlock) void apply_affine(
    int row0, int R, int k, int KS, float *__restrict__ rows,
    const int *__restrict__ mm) {
  __shared__ float s_m[2048], s_d[2048];
  load_affine(mm, KS, k, s_m, s_d);
  const int64_t total = (int64_t)R * KS;
  float *base = rows + (int64_t)row0 * KS;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int s = (int)(i % KS);
    if (s >= 1 && s <= k) base[i] = (base[i] - s_m[s]) / s_d[s];
  }
}

__global__ void unpack_rows(int R, int k, int KS, const float *__restrict__ rows,
                            float *__restrict__ dense) {
  const int64_t total = (int64_t)R * k;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / k), s = (int)(i % k);
    dense[i] = rows[(int64_t)r * KS + 1 + s];
  }
}

__global__ void count_empty_rows(int R, const int *__restrict__ rp,
                                 int *__restrict__ out) {
  int bad = 0;
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R;
       r += gridDim.x * blockDim.x)
    bad |= (rp[r + 1] == rp[r]);
  if (bad) atomicOr(out, 1);
}

__global__ void fill_int(int *p, int64_t n, int v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

int grid_for(int64_t work, int per_block, int cap = 2048) {
  int64_t g = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// One resident round of workgroups: each amortises its prologue (the
// min/max replica fold) and its flush over many rows.
template <class F>
int resident_grid(F fn) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess ||
        cus <= 0)
      cus = 256;  // the grid size only: MI355X's CU count
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, 0) !=
          hipSuccess || per_cu <= 0)
    per_cu = 2;
  return cus * per_cu;
}

int pick_g(double avg) {
  static const int lpi = [] {  // incidences per lane targeted
    return hgx_debug_env("HGX_ALG_LPI", 4);
  }();
  int g = 1;
  while (g < 64 && g * lpi < avg) g *= 2;
  return g;
}

using HalfFn = void (*)(int, int, const int *, const int *, const float *,
                        const float *, float *, const int *, int, int *, int,
                        int);
using SegFn = void (*)(int, const int2 *, int, const int *, const int *,
                       const float *, float *);
using FinFn = void (*)(int, const int *, const int *, const float *,
                       const int *, const float *, float *, const int *, int,
                       int *, int);

template <int MODE, bool PRE = false>
bool long_fns(int ks, SegFn &seg, FinFn &fin) {
  switch (ks) {
#define HGX_LCASE(KSV)                                   \
    case KSV:                                            \
      seg = algdist_seg_partial<KSV, 4, PRE>;            \
      fin = algdist_long_finish<KSV, MODE>;              \
      return true;
    HGX_LCASE(4) HGX_LCASE(8) HGX_LCASE(12) HGX_LCASE(16) HGX_LCASE(20)
#undef HGX_LCASE
    default:
      return false;
  }
}
using FlatFn = void (*)(int, const int *, const int *, const int *,
                        const float *, const float *, float *, const int *, int,
                        int *, int);

template <int MODE>
FlatFn flat_fn(int ks) {
  switch (ks) {
    case 4: return algdist_half_flat<4, MODE>;
    case 8: return algdist_half_flat<8, MODE>;
    case 12: return algdist_half_flat<12, MODE>;
    case 16: return algdist_half_flat<16, MODE>;
    case 20: return algdist_half_flat<20, MODE>;
    default: return nullptr;
  }
}

// M = incidences in flight per lane
template <int KS, int MODE, int M>
HalfFn narrow_for_gm(int g) {
  switch (g) {
    case 1: return algdist_half_narrow<KS, 1, MODE, M>;
    case 2: return algdist_half_narrow<KS, 2, MODE, M>;
    case 4: return algdist_half_narrow<KS, 4, MODE, M>;
    case 8: return algdist_half_narrow<KS, 8, MODE, M>;
    case 16: return algdist_half_narrow<KS, 16, MODE, M>;
    case 32: return algdist_half_narrow<KS, 32, MODE, M>;
    default: return algdist_half_narrow<KS, 64, MODE, M>;
  }
}

template <int KS, int MODE>
HalfFn narrow_for_g(int g) {
  static const int m = [] {
    return hgx_debug_env("HGX_ALG_M", 2);
  }();
  return m >= 4 ? narrow_for_gm<KS, MODE, 4>(g)
                : m == 1 ? narrow_for_gm<KS, MODE, 1>(g)
                         : narrow_for_gm<KS, MODE, 2>(g);
}

using QuadFn = void (*)(int, int, const int *, const int *, const float *,
                        const float *, float *, const int *, int, int *, int,
                        int, const int *, float *);

template <int KS, int MODE, int M, int PM>
QuadFn quad_for_gm(int g) {
  switch (g) {
    case 4: return algdist_half_quad<KS, 4, MODE, M, PM>;
    case 8: return algdist_half_quad<KS, 8, MODE, M, PM>;
    case 16: return algdist_half_quad<KS, 16, MODE, M, PM>;
    case 32: return algdist_half_quad<KS, 32, MODE, M, PM>;
    default: return algdist_half_quad<KS, 64, MODE, M, PM>;
  }
}

// HGX_ALG_QM: incidences in flight per quad (2 or 4, default 4)
template <int KS, int MODE, int PM>
QuadFn quad_for_g(int g) {
  static const int m = [] {
    return hgx_debug_env("HGX_ALG_QM", 4);
  }();
  return m <= 2 ? quad_for_gm<KS, MODE, 2, PM>(g) : quad_for_gm<KS, MODE, 4, PM>(g);
}

// quad-split rows (algdist_half_quad) for KS <= 16; HGX_ALG_QUAD=0 selects
// algdist_half_narrow. G = 4 lanes per quad x Q quads, Q doubling while a
// quad would stride more than HGX_ALG_QLPI (default 8) incidences.
template <int MODE, int PM = PM_GATHER>
QuadFn quad_fn(int ks, double avg, int &g) {
  static const int on = [] {
    return hgx_debug_env("HGX_ALG_QUAD", 1);
  }();
  static const int qlpi = [] {
    return std::max(1, hgx_debug_env("HGX_ALG_QLPI", 8));
  }();
  if ((!on && PM == PM_GATHER) || ks > 16) return nullptr;
  int q = 1;
  while (q < 16 && q * qlpi < avg) q *= 2;
  g = 4 * q;
  switch (ks) {
    case 4: return quad_for_g<4, MODE, PM>(g);
    case 8: return quad_for_g<8, MODE, PM>(g);
    case 12: return quad_for_g<12, MODE, PM>(g);
    case 16: return quad_for_g<16, MODE, PM>(g);
    default: return nullptr;
  }
}

template <int MODE>
HalfFn narrow_fn(int ks, int g) {
  switch (ks) {
    case 4: return narrow_for_g<4, MODE>(g);
    case 8: return narrow_for_g<8, MODE>(g);
    case 12: return narrow_for_g<12, MODE>(g);
    case 16: return narrow_for_g<16, MODE>(g);
    case 20: return narrow_for_g<20, MODE>(g);
    default: return nullptr;
  }
}

// pm: PM_GATHER (every sharded / partial sweep), or the single-GPU push
// form: PM_PUSH for the node half (tpos, contrib written), PM_STREAM for the
// edge half (src = contrib). Push and stream need KS <= 16 (the quad kernel).
int launch_half(hgx_ctx *ctx, int mode, int row0, int R, const int *rp,
                const int *col, const float *self_in, const float *src,
                float *out, const int *mm_prev, int src_affine, int *mm_cur,
                double avg, const int *blk, int nblk, LongRows *lr,
                bool sample_flush = false, int pm = PM_GATHER,
                const int *tpos = nullptr, float *contrib = nullptr) {
  const int k = ctx->k | (sample_flush ? kSampleFlush : 0), KS = ctx->ks;
  if (R <= 0) return HGX_OK;
  if (pm != PM_GATHER) {
    HGX_CHECK(ctx, mode == MODE_FULL && KS <= 16, HGX_EUNSUP,
              "alg-dist push form needs full rows and k <= 15");
    HGX_CHECK(ctx, pm == PM_STREAM || !lr || lr->nlong == 0, HGX_EUNSUP,
              "alg-dist push form: node rows longer than the long-row "
              "threshold are not pushed");
    int thresh = INT_MAX;
    if (lr && lr->nlong > 0) {  // stream: long edge rows from contrib
      SegFn seg = nullptr;
      FinFn fin = nullptr;
      long_fns<MODE_FULL, true>(KS, seg, fin);
      thresh = lr->thresh;
      HGX_TRY(hgx_ensure(ctx, lr->part, sizeof(float) * (size_t)lr->nseg * KS));
      hipLaunchKernelGGL(seg, dim3(grid_for(lr->nseg, kBlock / 64, resident_grid(seg))),
                         dim3(kBlock), 0, ctx->stream, lr->nseg,
                         lr->seg.as<int2>(), lr->thresh, rp, col, src,
                         lr->part.as<float>());
      hipLaunchKernelGGL(fin, dim3(grid_for(lr->nlong, kBlock / 64, resident_grid(fin))),
                         dim3(kBlock), 0, ctx->stream, lr->nlong,
                         lr->rows.as<int>(), lr->off.as<int>(),
                         lr->part.as<float>(), rp, self_in, out, mm_prev,
                         src_affine, mm_cur, k);
    }
    int g = 0;
    QuadFn fn = pm == PM_PUSH ? quad_fn<MODE_FULL, PM_PUSH>(KS, avg, g)
                              : quad_fn<MODE_FULL, PM_STREAM>(KS, avg, g);
    hipLaunchKernelGGL(fn, dim3(grid_for(R, kBlock / g, resident_grid(fn))),
                       dim3(kBlock), 0, ctx->stream, row0, R, rp, col, self_in,
                       src, out, mm_prev, src_affine, mm_cur, k, thresh, tpos,
                       contrib);
    HGX_LAUNCH_CHECK(ctx);
    return HGX_OK;
  }
  static const bool flat_env = [] {
    return hgx_debug_env("HGX_ALG_FLAT", 0) == 1;
  }();
  if (KS <= 20 && flat_env) {
    FlatFn fn = mode == MODE_FULL ? flat_fn<MODE_FULL>(KS) : flat_fn<MODE_PARTIAL>(KS);
    hipLaunchKernelGGL(fn, dim3(grid_for(nblk, kBlock / 64, resident_grid(fn))),
                       dim3(kBlock), 0, ctx->stream, nblk, blk, rp, col,
                       self_in, src, out, mm_prev, src_affine, mm_cur, k);
  } else if (KS <= 20) {
    int thresh = INT_MAX;
    if (lr && lr->nlong > 0) {
      SegFn seg = nullptr;
      FinFn fin = nullptr;
      const bool ok = mode == MODE_FULL ? long_fns<MODE_FULL>(KS, seg, fin)
                                        : long_fns<MODE_PARTIAL>(KS, seg, fin);
      if (ok) {
        thresh = lr->thresh;
        HGX_TRY(hgx_ensure(ctx, lr->part, sizeof(float) * (size_t)lr->nseg * KS));
        hipLaunchKernelGGL(seg, dim3(grid_for(lr->nseg, kBlock / 64, resident_grid(seg))),
                           dim3(kBlock), 0, ctx->stream, lr->nseg,
                           lr->seg.as<int2>(), lr->thresh, rp, col, src,
                           lr->part.as<float>());
        hipLaunchKernelGGL(fin, dim3(grid_for(lr->nlong, kBlock / 64, resident_grid(fin))),
                           dim3(kBlock), 0, ctx->stream, lr->nlong,
                           lr->rows.as<int>(), lr->off.as<int>(),
                           lr->part.as<float>(), rp, self_in, out, mm_prev,
                           src_affine, mm_cur, k);
      }
    }
    int g = 0;
    QuadFn qf = mode == MODE_FULL ? quad_fn<MODE_FULL>(KS, avg, g)
                                  : quad_fn<MODE_PARTIAL>(KS, avg, g);
    if (qf) {
      hipLaunchKernelGGL(qf, dim3(grid_for(R, kBlock / g, resident_grid(qf))),
                         dim3(kBlock), 0, ctx->stream, row0, R, rp, col,
                         self_in, src, out, mm_prev, src_affine, mm_cur, k,
                         thresh, nullptr, nullptr);
    } else {
      g = pick_g(avg);
      HalfFn fn = mode == MODE_FULL ? narrow_fn<MODE_FULL>(KS, g)
                                    : narrow_fn<MODE_PARTIAL>(KS, g);
      hipLaunchKernelGGL(fn, dim3(grid_for(R, kBlock / g, resident_grid(fn))),
                         dim3(kBlock), 0,
                         ctx->stream, row0, R, rp, col, self_in, src, out,
                         mm_prev, src_affine, mm_cur, k, thresh);
    }
  } else {
    auto fn = mode == MODE_FULL ? algdist_half_wide<MODE_FULL>
                                : algdist_half_wide<MODE_PARTIAL>;
    hipLaunchKernelGGL(fn, dim3(grid_for(R, kBlock / 64, resident_grid(fn))),
                       dim3(kBlock), 0,
                       ctx->stream, row0, R, KS, rp, col, self_in, src, out,
                       mm_prev, src_affine, mm_cur, k);
  }
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

int check_nonempty(hgx_ctx *ctx) {
  HGX_TRY(hgx_ensure(ctx, ctx->s0, 16));
  int *flag = ctx->s0.as<int>();
  HGX_HIP(ctx, hipMemsetAsync(flag, 0, sizeof(int), ctx->stream));
  hipLaunchKernelGGL(count_empty_rows, dim3(grid_for(ctx->N, 256)), dim3(256),
                     0, ctx->stream, ctx->N, ctx->rp_n.as<int>(), flag);
  hipLaunchKernelGGL(count_empty_rows, dim3(grid_for(ctx->E, 256)), dim3(256),
                     0, ctx->stream, ctx->E, ctx->rp_e.as<int>(), flag);
  HGX_LAUNCH_CHECK(ctx);
  int h = 0;
  HGX_HIP(ctx, hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  HGX_CHECK(ctx, h == 0, HGX_EZERODIV,
            "isolated node or edge: 1/|row| weights divide by zero "
            "(algebraic_distance.py:49)");
  return HGX_OK;
}

int init_mm(hgx_ctx *ctx, int *mm, int64_t words) {
  hipLaunchKernelGGL(fill_int, dim3(grid_for(words, 256)), dim3(256), 0,
                     ctx->stream, mm, words, INT_MIN);
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

__global__ void iota_i32(int *p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (int)i;
}
__global__ void invert_perm(const int *perm, int *inv, int64_t n) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x)
    inv[perm[j]] = (int)j;
}

// tpos[t] = position of node-major incidence t in the edge-major CSR: a
// stable radix sort of the incidences by edge id keeps node order inside an
// edge, which is col_e's order (rows sorted by node id).
int build_tpos(hgx_ctx *ctx) {
  if (ctx->tpos_ok) return HGX_OK;
  const int64_t n = ctx->nnz;
  HGX_TRY(hgx_ensure(ctx, ctx->tpos, sizeof(int) * (size_t)(n + 1)));
  DevBuf k2, v1, v2, tmp;
  int rc = HGX_OK;
  do {
    if ((rc = hgx_ensure(ctx, k2, sizeof(int) * (size_t)(n + 1))) != HGX_OK) break;
    if ((rc = hgx_ensure(ctx, v1, sizeof(int) * (size_t)(n + 1))) != HGX_OK) break;
    if ((rc = hgx_ensure(ctx, v2, sizeof(int) * (size_t)(n + 1))) != HGX_OK) break;
    hipLaunchKernelGGL(iota_i32, dim3(grid_for(n, 256)), dim3(256), 0,
                       ctx->stream, v1.as<int>(), n);
    // keys: a copy of col_n (the sort ping-pongs its buffers)
    if (hipMemcpyAsync(ctx->tpos.p, ctx->col_n.p, sizeof(int) * (size_t)n,
                       hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess) {
      rc = hgx_fail(ctx, HGX_EHIP, "tpos key copy failed");
      break;
    }
    int bits = 1;
    while (bits < 31 && (1ll << bits) < ctx->E) bits++;
    hipcub::DoubleBuffer<int> keys(ctx->tpos.as<int>(), k2.as<int>());
    hipcub::DoubleBuffer<int> vals(v1.as<int>(), v2.as<int>());
    size_t tb = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, vals, (int)n, 0, bits,
                                           ctx->stream) != hipSuccess) {
      rc = hgx_fail(ctx, HGX_EHIP, "tpos radix sort sizing failed");
      break;
    }
    if ((rc = hgx_ensure(ctx, tmp, tb + 256)) != HGX_OK) break;
    if (hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, keys, vals, (int)n, 0, bits,
                                           ctx->stream) != hipSuccess) {
      rc = hgx_fail(ctx, HGX_EHIP, "tpos radix sort failed");
      break;
    }
    // vals.Current()[j] = node-major index of edge-major incidence j
    hipLaunchKernelGGL(invert_perm, dim3(grid_for(n, 256)), dim3(256), 0,
                       ctx->stream, vals.Current(), ctx->tpos.as<int>(), n);
    if (hipGetLastError() != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      rc = hgx_fail(ctx, HGX_EHIP, "tpos build failed");
  } while (0);
  hgx_release(k2);
  hgx_release(v1);
  hgx_release(v2);
  hgx_release(tmp);
  if (rc == HGX_OK) ctx->tpos_ok = true;
  return rc;
}

int final_affine(hgx_ctx *ctx, int node_row0, int node_rows, const int *last) {
  const int k = ctx->k, KS = ctx->ks;
  if (node_rows > 0)
    hipLaunchKernelGGL(apply_affine,
                       dim3(grid_for((int64_t)node_rows * KS, 256)), dim3(256),
                       0, ctx->stream, node_row0, node_rows, k, KS,
                       ctx->X[ctx->xcur].as<float>(), last);
  hipLaunchKernelGGL(apply_affine, dim3(grid_for((int64_t)ctx->E * KS, 256)),
                     dim3(256), 0, ctx->stream, 0, ctx->E, k, KS,
                     ctx->Y[ctx->ycur].as<float>(), last);
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

}  // namespace

extern "C" int hgx_alg_set(hgx_ctx *ctx, int k, const float *node_xy,
                           const float *edge_xy) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, k >= 1 && k <= 2046, HGX_EUNSUP, "k=%d outside [1,2046]", k);
  HGX_CHECK(ctx, node_xy && edge_xy, HGX_EINVAL, "null coordinate buffer");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(check_nonempty(ctx));
  int KS = ((k + 1) + 3) / 4 * 4;
  {
    // Rows of 12 floats (k = 8..11, HOBE's k = 10) straddle the 64-B memory
    // sectors: half of the random row gathers touch two. Where the tables
    // spill the 256 MiB Infinity Cache the gathers are served by HBM at the
    // random-sector rate, and 64-B rows read one sector each: C4 8.17 ->
    // 7.16 ms per iteration (tools/perf_alg_ks.py, profiles/r03/); C3's
    // cache-resident 48-B rows stay (0.0447 vs 0.0453 ms). The alg_ks
    // tuning overrides (12 keeps 48-B rows).
    const int want = ctx->tune.alg_ks;
    if (want == 0 && KS == 12 &&
        (int64_t)(ctx->N + (int64_t)ctx->E) * 64 > (int64_t)256 << 20)
      KS = 16;
    if (want > KS && want % 4 == 0 && want <= 20) KS = want;
  }
  ctx->k = k;
  ctx->ks = KS;
  for (int b = 0; b < 2; b++) {
    HGX_TRY(hgx_ensure(ctx, ctx->X[b], sizeof(float) * (size_t)ctx->N * KS));
    HGX_TRY(hgx_ensure(ctx, ctx->Y[b], sizeof(float) * (size_t)ctx->E * KS));
  }
  const size_t dn = sizeof(float) * (size_t)ctx->N * k;
  const size_t de = sizeof(float) * (size_t)ctx->E * k;
  HGX_TRY(hgx_ensure(ctx, ctx->s1, std::max(dn, de)));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s1.p, node_xy, dn, hipMemcpyHostToDevice,
                              ctx->stream));
  hipLaunchKernelGGL(pack_rows, dim3(grid_for((int64_t)ctx->N * KS, 256)),
                     dim3(256), 0, ctx->stream, ctx->N, k, KS,
                     ctx->rp_n.as<int>(), ctx->s1.as<float>(),
                     ctx->X[0].as<float>());
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s1.p, edge_xy, de, hipMemcpyHostToDevice,
                              ctx->stream));
  hipLaunchKernelGGL(pack_rows, dim3(grid_for((int64_t)ctx->E * KS, 256)),
                     dim3(256), 0, ctx->stream, ctx->E, k, KS,
                     ctx->rp_e.as<int>(), ctx->s1.as<float>(),
                     ctx->Y[0].as<float>());
  HGX_LAUNCH_CHECK(ctx);
  ctx->xcur = ctx->ycur = 0;
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_alg_run(hgx_ctx *ctx, int iters) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE, "hgx_alg_set not called");
  HGX_CHECK(ctx, iters >= 0, HGX_EINVAL, "iterations must be >= 0");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  if (iters == 0) return HGX_OK;
#ifdef HGX_DEBUG_KNOBS
  {
    const int v = hgx_debug_env("HGX_ALG_ABLATE", 0);
    HGX_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_ablate), &v, sizeof(int)));
  }
#endif
  const int KS = ctx->ks;
  const size_t slot = 2 * (size_t)KS * kRep;
  HGX_TRY(hgx_ensure(ctx, ctx->mm, sizeof(int) * slot * iters));
  int *mm = ctx->mm.as<int>();
  // push form where it applies (KS <= 16, no long node rows)
  const bool push = ctx->tune.alg_push && KS <= 16 && ctx->long_n.nlong == 0;
  if (push) {
    HGX_TRY(build_tpos(ctx));
    HGX_TRY(hgx_ensure(ctx, ctx->contrib, sizeof(float) * (size_t)ctx->nnz * KS));
  }
  HGX_TRY(init_mm(ctx, mm, (int64_t)slot * iters));
  HGX_HIP(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  static const bool sample_env = [] {
    return hgx_debug_env("HGX_ALG_SAMPLE_FLUSH", 1) != 0;
  }();
  for (int it = 0; it < iters; it++) {
    const int *prev = it ? mm + slot * (it - 1) : nullptr;
    int *cur = mm + slot * it;
    const bool sample = sample_env && it + 1 < iters;
    float *xc = ctx->X[ctx->xcur].as<float>(), *xn = ctx->X[ctx->xcur ^ 1].as<float>();
    float *yc = ctx->Y[ctx->ycur].as<float>(), *yn = ctx->Y[ctx->ycur ^ 1].as<float>();
#ifdef HGX_DEBUG_KNOBS
    {
      const int hn = hgx_debug_env("HGX_ALG_HOT", 0x7fffffff);
      hipMemcpyToSymbolAsync(HIP_SYMBOL(g_hot_lim), &hn, sizeof(int), 0,
                             hipMemcpyHostToDevice, ctx->stream);
    }
#endif
    // node half: self x (scaled), gathered y (scaled)
    HGX_TRY(launch_half(ctx, MODE_FULL, 0, ctx->N, ctx->rp_n.as<int>(),
                        ctx->col_n.as<int>(), xc, yc, xn, prev, prev != nullptr,
                        cur, ctx->avg_deg_n, ctx->blk_n.as<int>(), ctx->nblk_n,
                        &ctx->long_n, sample, push ? PM_PUSH : PM_GATHER,
                        ctx->tpos.as<int>(), ctx->contrib.as<float>()));
#ifdef HGX_DEBUG_KNOBS
    {
      const int he = hgx_debug_env("HGX_ALG_HOT_E", 0x7fffffff);
      hipMemcpyToSymbolAsync(HIP_SYMBOL(g_hot_lim), &he, sizeof(int), 0,
                             hipMemcpyHostToDevice, ctx->stream);
    }
#endif
    // edge half: self y (scaled), gathered NEW x (raw)
    HGX_TRY(launch_half(ctx, MODE_FULL, 0, ctx->E, ctx->rp_e.as<int>(),
                        ctx->col_e.as<int>(), yc,
                        push ? ctx->contrib.as<float>() : xn, yn, prev, 0, cur,
                        ctx->avg_deg_e, ctx->blk_e.as<int>(), ctx->nblk_e,
                        &ctx->long_e, sample, push ? PM_STREAM : PM_GATHER));
    ctx->xcur ^= 1;
    ctx->ycur ^= 1;
  }
  HGX_HIP(ctx, hipEventRecord(ctx->ev1, ctx->stream));
  HGX_TRY(final_affine(ctx, 0, ctx->N, mm + slot * (iters - 1)));
  HGX_HIP(ctx, hipEventSynchronize(ctx->ev1));
  float ms = 0.f;
  HGX_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->alg_ms = ms;
  ctx->alg_bytes = (double)iters * (8.0 * ctx->nnz +
                                    (8.0 + 12.0 * ctx->k) * (ctx->N + ctx->E));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_alg_get(hgx_ctx *ctx, float *node_xy, float *edge_xy) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE, "no alg coordinates on device");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int k = ctx->k, KS = ctx->ks;
  const size_t dn = sizeof(float) * (size_t)ctx->N * k;
  const size_t de = sizeof(float) * (size_t)ctx->E * k;
  HGX_TRY(hgx_ensure(ctx, ctx->s1, std::max(dn, de)));
  if (node_xy) {
    hipLaunchKernelGGL(unpack_rows, dim3(grid_for((int64_t)ctx->N * k, 256)),
                       dim3(256), 0, ctx->stream, ctx->N, k, KS,
                       ctx->X[ctx->xcur].as<float>(), ctx->s1.as<float>());
    HGX_LAUNCH_CHECK(ctx);
    HGX_HIP(ctx, hipMemcpyAsync(node_xy, ctx->s1.p, dn, hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  if (edge_xy) {
    hipLaunchKernelGGL(unpack_rows, dim3(grid_for((int64_t)ctx->E * k, 256)),
                       dim3(256), 0, ctx->stream, ctx->E, k, KS,
                       ctx->Y[ctx->ycur].as<float>(), ctx->s1.as<float>());
    HGX_LAUNCH_CHECK(ctx);
    HGX_HIP(ctx, hipMemcpyAsync(edge_xy, ctx->s1.p, de, hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return HGX_OK;
}

extern "C" int hgx_alg_dist(hgx_ctx *ctx, int k, int iters, float *node_xy,
                            float *edge_xy) {
  HGX_TRY(hgx_alg_set(ctx, k, node_xy, edge_xy));
  HGX_TRY(hgx_alg_run(ctx, iters));
  return hgx_alg_get(ctx, node_xy, edge_xy);
}

extern "C" int hgx_alg_last_stats(hgx_ctx *ctx, double *ms, double *bytes) {
  if (!ctx) return HGX_EINVAL;
  if (ms) *ms = ctx->alg_ms;
  if (bytes) *bytes = ctx->alg_bytes;
  return HGX_OK;
}

// ---------------------------------------------------------------------------
// Sharded relaxation: the caller (torch.distributed over RCCL, or gloo in
// tests) all-reduces `partial` (SUM, float32, E*KS) between edge_partial and
// edge_final, and mm slot `it` (MAX, int32, 2*KS) after edge_final.
// ---------------------------------------------------------------------------
extern "C" int hgx_alg_shard_begin(hgx_ctx *ctx, int32_t row0, int32_t row1,
                                   void *d_partial, void *d_mm, int iters,
                                   int *ks_out) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE, "hgx_alg_set not called");
  HGX_CHECK(ctx, 0 <= row0 && row0 <= row1 && row1 <= ctx->N, HGX_EINVAL,
            "node shard [%d,%d) outside [0,%d)", row0, row1, ctx->N);
  HGX_CHECK(ctx, d_partial && d_mm && iters > 0, HGX_EINVAL,
            "null exchange buffer or iters <= 0");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  // local edge sub-CSR: for every edge, the incidences with node in
  // [row0,row1) (edge rows are sorted, so they are contiguous).
  std::vector<int> rp(ctx->E + 1), col((size_t)ctx->nnz + 1), rpl(ctx->E + 1);
  HGX_HIP(ctx, hipMemcpy(rp.data(), ctx->rp_e.p, sizeof(int) * (ctx->E + 1),
                         hipMemcpyDeviceToHost));
  if (ctx->nnz)
    HGX_HIP(ctx, hipMemcpy(col.data(), ctx->col_e.p, sizeof(int) * ctx->nnz,
                           hipMemcpyDeviceToHost));
  std::vector<int> cl;
  cl.reserve((size_t)ctx->nnz / 2 + 1);
  rpl[0] = 0;
  for (int e = 0; e < ctx->E; e++) {
    auto b = col.begin() + rp[e], en = col.begin() + rp[e + 1];
    auto lo = std::lower_bound(b, en, row0), hi = std::lower_bound(b, en, row1);
    cl.insert(cl.end(), lo, hi);
    rpl[e + 1] = (int)cl.size();
  }
  HGX_TRY(hgx_ensure(ctx, ctx->rp_el, sizeof(int) * (ctx->E + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->col_el, sizeof(int) * (cl.size() + 1)));
  HGX_HIP(ctx, hipMemcpy(ctx->rp_el.p, rpl.data(), sizeof(int) * (ctx->E + 1),
                         hipMemcpyHostToDevice));
  if (!cl.empty())
    HGX_HIP(ctx, hipMemcpy(ctx->col_el.p, cl.data(), sizeof(int) * cl.size(),
                           hipMemcpyHostToDevice));
  {
    std::vector<int> rpn(ctx->N + 1);
    HGX_HIP(ctx, hipMemcpy(rpn.data(), ctx->rp_n.p, sizeof(int) * (ctx->N + 1),
                           hipMemcpyDeviceToHost));
    HGX_TRY(hgx_make_row_blocks(ctx, rpn.data(), row0, row1, ctx->blk_sn,
                                ctx->nblk_sn));
    HGX_TRY(hgx_make_row_blocks(ctx, rpl.data(), 0, ctx->E, ctx->blk_el,
                                ctx->nblk_el));
    HGX_TRY(hgx_make_long_rows(ctx, rpn.data(), row0, row1, ctx->long_sn));
    HGX_TRY(hgx_make_long_rows(ctx, rpl.data(), 0, ctx->E, ctx->long_el));
  }
  ctx->row0 = row0;
  ctx->row1 = row1;
  ctx->ext_wire = nullptr;
  ctx->n_wire = 0;
  ctx->ext_partial = (float *)d_partial;
  ctx->ext_mm = (int *)d_mm;
  ctx->ext_iters = iters;
  HGX_TRY(init_mm(ctx, ctx->ext_mm, (int64_t)2 * ctx->ks * kRep * iters));
  if (ks_out) *ks_out = ctx->ks;
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_alg_shard_node(hgx_ctx *ctx, int it) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->ext_mm && it >= 0 && it < ctx->ext_iters, HGX_ESTATE,
            "shard iteration %d out of order", it);
  const size_t slot = 2 * (size_t)ctx->ks * kRep;
  const int *prev = it ? ctx->ext_mm + slot * (it - 1) : nullptr;
  int *cur = ctx->ext_mm + slot * it;
  float *xc = ctx->X[ctx->xcur].as<float>(), *xn = ctx->X[ctx->xcur ^ 1].as<float>();
  float *yc = ctx->Y[ctx->ycur].as<float>();
  HGX_TRY(launch_half(ctx, MODE_FULL, ctx->row0, ctx->row1 - ctx->row0,
                      ctx->rp_n.as<int>(), ctx->col_n.as<int>(), xc, yc, xn,
                      prev, prev != nullptr, cur, ctx->avg_deg_n,
                      ctx->blk_sn.as<int>(), ctx->nblk_sn, &ctx->long_sn));
  return HGX_OK;
}

extern "C" int hgx_alg_shard_edge_partial(hgx_ctx *ctx, int it) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->ext_mm && it >= 0 && it < ctx->ext_iters, HGX_ESTATE,
            "shard iteration %d out of order", it);
  float *xn = ctx->X[ctx->xcur ^ 1].as<float>();
  const double avg = (double)std::max<int64_t>(1, ctx->nnz) / ctx->E;
  HGX_TRY(launch_half(ctx, MODE_PARTIAL, 0, ctx->E, ctx->rp_el.as<int>(),
                      ctx->col_el.as<int>(), nullptr, xn, ctx->ext_partial,
                      nullptr, 0, nullptr, avg, ctx->blk_el.as<int>(),
                      ctx->nblk_el, &ctx->long_el));
  if (ctx->ext_wire && ctx->n_wire > 0) {
    hipLaunchKernelGGL(algdist_wire_pack,
                       dim3(grid_for((int64_t)ctx->E * (ctx->k + 1), 256)),
                       dim3(256), 0, ctx->stream, 0, ctx->E, ctx->ks, ctx->k,
                       ctx->wire_slot.as<int>(), ctx->ext_partial, ctx->ext_wire);
    HGX_LAUNCH_CHECK(ctx);
  }
  return HGX_OK;
}

// Edge-range pipelining: the caller all-reduces the wire rows of range r
// while the partials of range r + 1 are computed (both ranges' rows are
// disjoint in `partial` and on the wire).
extern "C" int hgx_alg_shard_ranges(hgx_ctx *ctx, int n, int32_t *bounds) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->ext_mm, HGX_ESTATE, "hgx_alg_shard_begin not called");
  HGX_CHECK(ctx, n >= 1 && n <= hgx_ctx::kMaxEdgeRanges && bounds, HGX_EINVAL,
            "edge ranges %d outside [1,%d] or null bounds", n,
            hgx_ctx::kMaxEdgeRanges);
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  std::vector<int> rpl(ctx->E + 1), rpg(ctx->E + 1);
  HGX_HIP(ctx, hipMemcpy(rpl.data(), ctx->rp_el.p, sizeof(int) * (ctx->E + 1),
                         hipMemcpyDeviceToHost));
  HGX_HIP(ctx, hipMemcpy(rpg.data(), ctx->rp_e.p, sizeof(int) * (ctx->E + 1),
                         hipMemcpyDeviceToHost));
  // contiguous edge ranges balanced by ALL incidences (the global edge CSR),
  // so every rank gets the same split and the same wire slices
  const int64_t tot = rpg[ctx->E];
  ctx->elr_bound[0] = 0;
  for (int r = 1; r < n; r++) {
    const int64_t want = tot * r / n;
    int e = (int)(std::lower_bound(rpg.begin(), rpg.end(), (int)want) -
                  rpg.begin());
    ctx->elr_bound[r] = std::max(ctx->elr_bound[r - 1], std::min(e, ctx->E));
  }
  ctx->elr_bound[n] = ctx->E;
  for (int r = 0; r < n; r++)
    HGX_TRY(hgx_make_long_rows(ctx, rpl.data(), ctx->elr_bound[r],
                               ctx->elr_bound[r + 1], ctx->long_elr[r]));
  ctx->n_elr = n;
  for (int r = 0; r <= n; r++) bounds[r] = ctx->elr_bound[r];
  return HGX_OK;
}

extern "C" int hgx_alg_shard_edge_partial_range(hgx_ctx *ctx, int it, int r) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->ext_mm && it >= 0 && it < ctx->ext_iters, HGX_ESTATE,
            "shard iteration %d out of order", it);
  HGX_CHECK(ctx, r >= 0 && r < ctx->n_elr, HGX_EINVAL,
            "edge range %d outside [0,%d)", r, ctx->n_elr);
  const int e0 = ctx->elr_bound[r], e1 = ctx->elr_bound[r + 1];
  float *xn = ctx->X[ctx->xcur ^ 1].as<float>();
  const double avg = (double)std::max<int64_t>(1, ctx->nnz) / ctx->E;
  HGX_TRY(launch_half(ctx, MODE_PARTIAL, e0, e1 - e0, ctx->rp_el.as<int>(),
                      ctx->col_el.as<int>(), nullptr, xn, ctx->ext_partial,
                      nullptr, 0, nullptr, avg, ctx->blk_el.as<int>(),
                      ctx->nblk_el, &ctx->long_elr[r]));
  if (ctx->ext_wire && ctx->n_wire > 0 && e1 > e0) {
    hipLaunchKernelGGL(algdist_wire_pack,
                       dim3(grid_for((int64_t)(e1 - e0) * (ctx->k + 1), 256)),
                       dim3(256), 0, ctx->stream, e0, e1 - e0, ctx->ks, ctx->k,
                       ctx->wire_slot.as<int>(), ctx->ext_partial, ctx->ext_wire);
    HGX_LAUNCH_CHECK(ctx);
  }
  return HGX_OK;
}

extern "C" int hgx_alg_shard_wire(hgx_ctx *ctx, void *d_wire, int64_t n_shared,
                                  const int32_t *edge_slot) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->ext_mm, HGX_ESTATE, "hgx_alg_shard_begin not called");
  HGX_CHECK(ctx, edge_slot && n_shared >= 0 && (d_wire || n_shared == 0),
            HGX_EINVAL, "null wire or slot map");
  std::vector<char> seen((size_t)n_shared, 0);
  for (int e = 0; e < ctx->E; e++) {
    const int s = edge_slot[e];
    HGX_CHECK(ctx, s >= -2 && s < n_shared, HGX_EINVAL,
              "edge %d: slot %d outside [-2, %lld)", e, s, (long long)n_shared);
    if (s >= 0) {
      HGX_CHECK(ctx, !seen[s], HGX_EINVAL, "wire row %d given twice", s);
      seen[s] = 1;
    }
  }
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, ctx->wire_slot, sizeof(int) * (ctx->E + 1)));
  HGX_HIP(ctx, hipMemcpy(ctx->wire_slot.p, edge_slot, sizeof(int) * ctx->E,
                         hipMemcpyHostToDevice));
  ctx->ext_wire = (float *)d_wire;
  ctx->n_wire = n_shared;
  return HGX_OK;
}

extern "C" int hgx_alg_shard_edge_final(hgx_ctx *ctx, int it) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->ext_mm && it >= 0 && it < ctx->ext_iters, HGX_ESTATE,
            "shard iteration %d out of order", it);
  const size_t slot = 2 * (size_t)ctx->ks * kRep;
  const int *prev = it ? ctx->ext_mm + slot * (it - 1) : nullptr;
  int *cur = ctx->ext_mm + slot * it;
  float *yc = ctx->Y[ctx->ycur].as<float>(), *yn = ctx->Y[ctx->ycur ^ 1].as<float>();
  if (ctx->ext_wire)
    hipLaunchKernelGGL(algdist_edge_final_wire,
                       dim3(grid_for((int64_t)ctx->E * ctx->ks, 256)), dim3(256),
                       0, ctx->stream, ctx->E, ctx->ks, ctx->k,
                       ctx->rp_e.as<int>(), yc, ctx->ext_partial, ctx->ext_wire,
                       ctx->wire_slot.as<int>(), yn, prev, cur);
  else
    hipLaunchKernelGGL(algdist_edge_final,
                       dim3(grid_for((int64_t)ctx->E * ctx->ks, 256)), dim3(256),
                       0, ctx->stream, ctx->E, ctx->ks, ctx->k,
                       ctx->rp_e.as<int>(), yc, ctx->ext_partial, yn, prev, cur);
  HGX_LAUNCH_CHECK(ctx);
  ctx->xcur ^= 1;
  ctx->ycur ^= 1;
  return HGX_OK;
}

extern "C" int hgx_alg_shard_end(hgx_ctx *ctx) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->ext_mm, HGX_ESTATE, "hgx_alg_shard_begin not called");
  const size_t slot = 2 * (size_t)ctx->ks * kRep;
  HGX_TRY(final_affine(ctx, ctx->row0, ctx->row1 - ctx->row0,
                       ctx->ext_mm + slot * (ctx->ext_iters - 1)));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->ext_mm = nullptr;
  ctx->ext_partial = nullptr;
  ctx->ext_wire = nullptr;
  ctx->n_wire = 0;
  return HGX_OK;
}
