// Dense MLP engine: the Keras models behind the embedding combiners and the
// link-prediction classifier, trained with Keras 2.x fit semantics on one
// MI355X (gfx950).
//
// Reference models (restated, not translated):
//   HGX_MLP_LP_CLASSIFIER      evaluation_util.py:471-505
//       [node_emb | edge_emb] (2d) -> Dense(d, relu) -> Dense(1, sigmoid)
//       MSE, Adagrad, batch 256, 30 epochs, EarlyStopping(loss, 1e-3)
//   HGX_MLP_NE_SUPERVISED      combine_embeddings_util.py:80-174
//       per side (node / edge): Dropout(0.5) -> Dense(h, relu)
//       -> Dense(d, sigmoid) ["JointNode" / "JointEdge"], h = (in + d) / 2;
//       Concatenate -> Dense(d, relu) -> Dense(1, sigmoid); MSE, Adagrad,
//       batch 256, 100 epochs, EarlyStopping(loss)
//   HGX_MLP_NE_SEMI_SUPERVISED the same plus, per side, joint -> Dense(h,
//       relu) -> Dense(in, relu) ["Recovered*"] trained to reproduce the
//       undropped input; loss weights [4, 1, 1]
//
// Execution model. Keras batches are sequential (each batch's update feeds
// the next batch), so one batch is a short chain of grouped GEMM launches:
//   FWD  (per layer stage; both towers in one launch)  Y = act(A W + b)
//   HEAD (N = 1 label layer) y, loss, dz and the dX of its input, fused
//   BWD  (per layer stage) dZ_in = (sum_t dZ_t W_t^T) * act'(Y_in)
//   WGRAD (every layer, one launch) G = X^T dZ; Adagrad on W and b in the
//        epilogue (a += g^2; p -= lr g / (sqrt(a) + eps))
// Every GEMM tile is 32x32 on v_mfma_f32_32x32x2_f32 (exact f32 products,
// f32 accumulation), 4 waves per workgroup splitting each 64-long reduction
// chunk, operands staged through LDS in the MFMA's lane order (pair p of a
// chunk = one 64-float LDS row, lane l reads element l: conflict free),
// double buffered. The first layer gathers its input rows straight from the
// embedding tables through the sample's (node, edge) ids and applies the
// dropout mask on the fly: the concatenated sample matrix of the reference
// (6 nnz x 2 x in floats) is never materialised.
//
// Layout: every width is padded with zeros (activations and dZ to multiples
// of 64 columns, tables to multiples of 4); padded weight rows/columns start
// at 0 and stay 0 (their inputs or their dZ are exactly 0, so Adagrad's step
// is exactly 0), so padding changes no result.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hgx_internal.h"

// No implicit contraction: a + g*g must stay two roundings (hipcc fuses it
// into one fma by default, and the __fadd_rn/__fmul_rn helpers do not stop
// it: they are inlined with their header's contract setting); every fma of
// this file is written out, in the order the CPU restatement uses.
#pragma clang fp contract(off)

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kTile = 32;     // output tile edge
constexpr int kChunk = 64;    // reduction chunk staged in LDS
constexpr int kThreads = 256; // 4 waves
constexpr int kMaxJobs = 12;

// Diagnostic build only (HGX_MLP_DIAG_TIME=1, tools/build_variant.sh): thread
// 0 of every workgroup of the NCH-instantiated GEMM kernels stamps the 100 MHz
// real-time counter at phase boundaries (waiting for its own loads / stores at
// each one, which serialises what the product overlaps) and adds the phase
// times to per-kernel sums that hgx_mlp_fit prints to stderr.
#ifndef HGX_MLP_DIAG_TIME
#define HGX_MLP_DIAG_TIME 0
#endif
#if HGX_MLP_DIAG_TIME
__device__ unsigned long long g_mlp_t[8][12];
__device__ unsigned long long g_mlp_n[8];
#define TSTAMP(i)                                             \
  do {                                                        \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
    ts[i] = __builtin_amdgcn_s_memrealtime();                 \
  } while (0)
#define TDECL unsigned long long ts[12] = {}
#define HSTAMP(i)                                                  \
  do {                                                             \
    if (tsp) {                                                     \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  \
      tsp[i] = __builtin_amdgcn_s_memrealtime();                   \
    }                                                              \
  } while (0)
#define TFLUSH(kind, n)                                                   \
  do {                                                                    \
    if (threadIdx.x == 0) {                                               \
      for (int q = 1; q < (n); q++) atomicAdd(&g_mlp_t[kind][q], ts[q] - ts[0]); \
      atomicAdd(&g_mlp_n[kind], 1ull);                                    \
    }                                                                     \
  } while (0)
#else
#define TSTAMP(i) (void)0
#define HSTAMP(i) (void)0
#define TDECL (void)0
#define TFLUSH(kind, n) (void)0
#endif
constexpr int kMcap = 4096;   // activation rows (training uses the first 256)

// Global stores of the launches' outputs (activations, deltas, prefetched
// rows, weights and Adagrad state). HGX_MLP_WT=1: write-through (an
// agent-scope relaxed atomic store is `global_store ... sc1`), so the output
// leaves no dirty lines in the XCD's L2 for the kernel-end release to write
// back before the next, dependent launch (MI355X_MICROARCH "boundary":
// + bytes / 6 TB/s; "publish-large"); 0: plain stores (A/B builds). C5
// combiner, interleaved A/B (tools/r06_mlp_wt.sh, profiles/r06/mlp_wt/):
// 4.80 / 4.79M -> 4.94 / 4.95M samples/s, the MLP tests bit-exact.
#ifndef HGX_MLP_WT
#define HGX_MLP_WT 1
#endif
__device__ __forceinline__ void gst(float *p, float v) {
  if (HGX_MLP_WT)
    __hip_atomic_store(reinterpret_cast<unsigned *>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
__device__ __forceinline__ void gst4(float *p, float4 v) {
  if (HGX_MLP_WT) {
    unsigned long long *q = reinterpret_cast<unsigned long long *>(p);
    __hip_atomic_store(q, __builtin_bit_cast(unsigned long long, make_float2(v.x, v.y)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, __builtin_bit_cast(unsigned long long, make_float2(v.z, v.w)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *reinterpret_cast<float4 *>(p) = v;
  }
}

enum { ACT_SIGMOID = HGX_ACT_SIGMOID, ACT_RELU = HGX_ACT_RELU };

// exp for the sigmoid: Cephes expf's reduction and polynomial written as
// explicit fma steps (rint, fma and ldexp are exact operations), so the CPU
// restatement computes the same bits (oracle/mlpref.c).
__device__ __forceinline__ float mlp_exp(float x) {
  x = fminf(fmaxf(x, -87.0f), 88.0f);
  const float n = rintf(x * 1.44269504088896341f);
  float r = fmaf(-n, 0.693359375f, x);
  r = fmaf(-n, -2.12194440e-4f, r);
  float p = fmaf(1.9875691500e-4f, r, 1.3981999507e-3f);
  p = fmaf(p, r, 8.3334519073e-3f);
  p = fmaf(p, r, 4.1665795894e-2f);
  p = fmaf(p, r, 1.6666665459e-1f);
  p = fmaf(p, r, 5.0000001201e-1f);
  p = fmaf(p, r * r, r);
  return ldexpf(p + 1.0f, (int)n);
}
__device__ __forceinline__ float act_f(int act, float z) {
  return act == ACT_SIGMOID ? 1.0f / (1.0f + mlp_exp(-z)) : (z > 0.f ? z : 0.f);
}
// derivative from the activation's OUTPUT y
__device__ __forceinline__ float act_d(int act, float y) {
  return act == ACT_SIGMOID ? y * (1.0f - y) : (y > 0.f ? 1.0f : 0.0f);
}

// An [rows x width] operand: a dense activation buffer, or rows gathered
// from one or two embedding tables by the sample ids (columns [0, c1) from
// t0 row i0[p], [c1, width) from t1 row i1[p], p = pbase + m) with an
// optional dropout(0.5) mask (keep -> x2), keyed by (seed, stream, p, col).
struct Src {
  const float *x;
  int ldx;
  const float *t0, *t1;
  const int *i0, *i1;
  int ld0, ld1, c1;
  int width;
  int gather, drop;
  uint32_t dstream;
};

struct Ctx {
  int M;          // rows of this batch / chunk
  int grad_only;  // debug (HGX_MLP_GRAD_AT): store the gradient, no update
  int64_t pbase;  // position of row 0 in the epoch's sample order
  uint64_t dseed;
  float lr, eps;
};

// dropout bits of 4 consecutive columns k4..k4+3 (k4 % 4 == 0)
__device__ __forceinline__ unsigned drop_bits4(const Src &s, const Ctx &c,
                                               int64_t p, int k4) {
  const int w64 = (s.width + 63) >> 6;
  const uint64_t r =
      hgx::rand64(c.dseed, s.dstream, (uint64_t)p * (uint64_t)w64 + (k4 >> 6));
  return (unsigned)(r >> (k4 & 63)) & 0xFu;
}

__device__ __forceinline__ float4 src_load4(const Src &s, const Ctx &c, int m,
                                            int k4, bool use_drop) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (m >= c.M || k4 >= s.width) return v;
  if (!s.gather) {
    v = *reinterpret_cast<const float4 *>(s.x + (int64_t)m * s.ldx + k4);
  } else {
    const int64_t p = c.pbase + m;
    if (k4 < s.c1)
      v = *reinterpret_cast<const float4 *>(s.t0 + (int64_t)s.i0[p] * s.ld0 + k4);
    else
      v = *reinterpret_cast<const float4 *>(s.t1 + (int64_t)s.i1[p] * s.ld1 +
                                            (k4 - s.c1));
    if (use_drop && s.drop) {
      const unsigned b = drop_bits4(s, c, p, k4);
      v.x = (b & 1) ? v.x * 2.0f : 0.0f;
      v.y = (b & 2) ? v.y * 2.0f : 0.0f;
      v.z = (b & 4) ? v.z * 2.0f : 0.0f;
      v.w = (b & 8) ? v.w * 2.0f : 0.0f;
    }
  }
  return v;
}

// A source's fields read once into scalar registers (NCH-instantiated
// kernels). The asm pins keep them there: without them the compiler re-reads
// each field from the kernel-argument table inside every uniform branch that
// uses it, one scalar round trip per chunk (150+ s_load in mlp_fwd<8>).
template <class T> __device__ __forceinline__ T spin(T v) {
  asm volatile("" : "+s"(v));
  return v;
}
// pinned pointers are typed global (address space 1): a pointer through the
// asm would otherwise be generic and its loads flat_load
typedef const __attribute__((address_space(1))) float *gfp;
typedef const __attribute__((address_space(1))) int *gip;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) f4v *gf4p;
__device__ __forceinline__ float4 ldg4(gfp p) {
  const f4v v = *reinterpret_cast<gf4p>(p);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ gfp gpin(const float *p) {
  return (gfp)spin((uint64_t)p);
}
__device__ __forceinline__ gip gpin(const int *p) {
  return (gip)spin((uint64_t)p);
}
struct SrcK {
  gfp x, t0, t1, safe;  // t0 / t1: the tables of columns < c1 / >= c1
  gip j0, j1;           // their id arrays (a valid one either way)
  int ldx, l0, l1, c1, width, gather, drop, w64;
  uint64_t dkey;  // hgx::rand64_key(seed, dstream)
};
__device__ __forceinline__ SrcK src_k(const Src &s, const Ctx &c) {
  SrcK k;
  k.gather = spin(s.gather);
  k.drop = spin(s.drop);
  k.c1 = spin(s.c1);
  k.width = spin(s.width);
  k.ldx = spin(s.ldx);
  k.x = gpin(s.x);
  k.t0 = gpin(s.c1 > 0 ? s.t0 : s.t1);
  k.t1 = gpin(s.c1 < s.width ? s.t1 : s.t0);
  k.j0 = gpin(s.c1 > 0 ? s.i0 : s.i1);
  k.j1 = gpin(s.c1 < s.width ? s.i1 : s.i0);
  k.l0 = spin(s.c1 > 0 ? s.ld0 : s.ld1);
  k.l1 = spin(s.c1 < s.width ? s.ld1 : s.ld0);
  k.safe = s.gather ? k.t0 : k.x;
  k.w64 = (k.width + 63) >> 6;
  k.dkey = spin(hgx::rand64_key(c.dseed, s.dstream));
  return k;
}

// One operand row resolved once per kernel (the sample ids of a gathered
// source loaded up front), so the per-chunk loads of that row depend on no
// other load and several chunks can be in flight.
struct SrcRow {
  gfp p0, p1;  // dense row / table-0 row, table-1 row
  int64_t pos;
  bool ok;
};
// R rows of a tile: rows past M resolve to row 0 of the batch (never read:
// src_raw4 masks them). One uniform branch around all of them, and every id
// load unconditional inside it, so all ids share one round trip.
template <int R>
__device__ __forceinline__ void src_rows(const SrcK &s, const Ctx &c, const int (&m)[R],
                                         SrcRow (&r)[R]) {
#pragma unroll
  for (int i = 0; i < R; i++) {
    r[i].ok = m[i] < c.M;
    r[i].pos = c.pbase + m[i];
    r[i].p0 = r[i].p1 = nullptr;
  }
  if (!s.gather) {
#pragma unroll
    for (int i = 0; i < R; i++) r[i].p0 = s.x + (int64_t)(r[i].ok ? m[i] : 0) * s.ldx;
    return;
  }
  int a0[R], a1[R];
#pragma unroll
  for (int i = 0; i < R; i++) {
    const int64_t pa = r[i].ok ? r[i].pos : c.pbase;
    a0[i] = s.j0[pa];
    a1[i] = s.j1[pa];
  }
#pragma unroll
  for (int i = 0; i < R; i++) {
    r[i].p0 = s.t0 + (int64_t)a0[i] * s.l0;
    r[i].p1 = s.t1 + (int64_t)a1[i] * s.l1;
  }
}
// src_load4 of a resolved row in two steps, so that no lane-divergent
// branch separates a load from its use (a join over loaded registers makes
// the compiler wait for them): src_raw4 issues one unconditional load (a
// valid dummy row when the element is outside the operand), src_fix4 zeroes
// and applies the dropout mask when the chunk is consumed. Same values as
// src_load4.
__device__ __forceinline__ float4 src_raw4(const SrcK &s, const SrcRow &r, int k4) {
  const bool in = r.ok && k4 < s.width;
  gfp a = s.gather ? (k4 < s.c1 ? r.p0 + k4 : r.p1 + (k4 - s.c1)) : r.p0 + k4;
  return ldg4(in ? a : s.safe);
}
__device__ __forceinline__ float4 src_fix4(const SrcK &s, const SrcRow &r, int k4,
                                           float4 v, bool use_drop) {
  if (!(r.ok && k4 < s.width)) return make_float4(0.f, 0.f, 0.f, 0.f);
  if (s.gather && use_drop && s.drop) {
    // drop_bits4 with rand64's invariant part precomputed (same bits)
    const uint64_t q = (uint64_t)r.pos * (uint64_t)s.w64 + (k4 >> 6);
    const unsigned b = (unsigned)(hgx::mix64(s.dkey + q) >> (k4 & 63)) & 0xFu;
    v.x = (b & 1) ? v.x * 2.0f : 0.0f;
    v.y = (b & 2) ? v.y * 2.0f : 0.0f;
    v.z = (b & 4) ? v.z * 2.0f : 0.0f;
    v.w = (b & 8) ? v.w * 2.0f : 0.0f;
  }
  return v;
}

__device__ __forceinline__ float src_at(const Src &s, const Ctx &c, int m,
                                        int k) {
  if (m >= c.M || k >= s.width) return 0.f;
  if (!s.gather) return s.x[(int64_t)m * s.ldx + k];
  const int64_t p = c.pbase + m;
  return k < s.c1 ? s.t0[(int64_t)s.i0[p] * s.ld0 + k]
                  : s.t1[(int64_t)s.i1[p] * s.ld1 + (k - s.c1)];
}

// LDS operand image of one chunk: pair p (reduction indices 2p, 2p+1) is a
// 64-float row, element (i, r) at (r>>1)*64 + (r&1)*32 + i: exactly the
// lane order of v_mfma_f32_32x32x2_f32 (lane = 32*(r&1) + i).
__device__ __forceinline__ int lds_at(int i, int r) {
  return (r >> 1) * 64 + (r & 1) * 32 + i;
}

// wave w consumes pairs 8w..8w+7 of the chunk
__device__ __forceinline__ void mma_chunk(const float *As, const float *Bs,
                                          f32x16 &acc, int w, int lane) {
#pragma unroll
  for (int s = 0; s < 8; s++) {
    const int q = (w * 8 + s) * 64 + lane;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[q], Bs[q], acc, 0, 0, 0);
  }
}

// Sum the 4 waves' partial tiles (fixed order) and hand each thread the 4
// results it owns: column j = lane & 31, rows i0..i0+3 (i0 = 8g + 4(lane>>5)).
__device__ __forceinline__ void reduce_tile(float *lds, const f32x16 &acc,
                                            float out[4], int &i0, int &j) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  __syncthreads();  // every wave is done with the operand buffers
#pragma unroll
  for (int r = 0; r < 16; r++) lds[(w * 16 + r) * 64 + lane] = acc[r];
  __syncthreads();
  const int g = w;  // register group of this thread
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int r = 4 * g + e;
    out[e] = lds[(0 * 16 + r) * 64 + lane] + lds[(1 * 16 + r) * 64 + lane];
    out[e] += lds[(2 * 16 + r) * 64 + lane];
    out[e] += lds[(3 * 16 + r) * 64 + lane];
  }
  i0 = 8 * g + 4 * (lane >> 5);
  j = lane & 31;
}

// ---- operand loaders: one chunk = 2 float4 per thread per operand ----
// pattern R (rows along the tile index, 4 values along the reduction index):
//   thread t: tile rows (t>>4) and (t>>4)+16, reduction r4 = 4*(t&15)
// pattern C (rows along the reduction index, 4 values along the tile index):
//   thread t: reduction rows (t>>3) and (t>>3)+32, tile cols 4*(t&7)
__device__ __forceinline__ void store_R1(float *S, float4 v, int i, int r4) {
  S[lds_at(i, r4 + 0)] = v.x;
  S[lds_at(i, r4 + 1)] = v.y;
  S[lds_at(i, r4 + 2)] = v.z;
  S[lds_at(i, r4 + 3)] = v.w;
}
__device__ __forceinline__ void store_R(float *S, float4 v0, float4 v1) {
  const int t = threadIdx.x, r4 = 4 * (t & 15);
  store_R1(S, v0, t >> 4, r4);
  store_R1(S, v1, (t >> 4) + 16, r4);
}
// pattern R2 (the NCH-instantiated kernels): thread t holds tile row
// i = t & 31 at reduction r4 = 4*(t>>5) and r4 + 32, so one ds_write_b32 of
// a wave spans all 32 rows (2-way bank conflicts instead of pattern R's
// 16-way); the LDS image is the same
__device__ __forceinline__ void store_R2(float *S, float4 v0, float4 v1) {
  const int t = threadIdx.x, i = t & 31, r4 = 4 * (t >> 5);
  store_R1(S, v0, i, r4);
  store_R1(S, v1, i, r4 + 32);
}
__device__ __forceinline__ void store_C(float *S, float4 v0, float4 v1) {
  const int t = threadIdx.x, j4 = 4 * (t & 7);
  *reinterpret_cast<float4 *>(S + lds_at(j4, t >> 3)) = v0;
  *reinterpret_cast<float4 *>(S + lds_at(j4, (t >> 3) + 32)) = v1;
}

// ============================ FWD ==========================================
struct FwdJob {
  Src a;
  int K;              // reduction length (multiple of 64)
  const float *W;     // [K][ldw]
  const float *b;
  int ldw, tiles_n, Nreal, act;
  float *Y;
  int ldy;
  // reconstruction loss epilogue (semi-supervised combiner): target = the
  // undropped input `tgt`, weight lw, mean over Nreal columns and M rows
  int loss;
  float lw;
  Src tgt;
  float *dZ;
  int lddz;
  float *part;        // one loss partial per tile
  // prefetch job (pf = 1, no GEMM; combiner training): the next batch's
  // rows of the gathered, dropped-out input `a` -- sample positions pfbase ..
  // pfbase + pfM, the kPfRows rows zero past pfM -- into pfX (row stride
  // pfld), which that batch's first layer and its weight gradient then read
  // as a dense operand: the same values in the same places as the gather
  int pf, pfM, pfld;
  int64_t pfbase;
  float *pfX;
};
constexpr int kPfRows = 256;             // rows of a prefetch buffer (max batch)
constexpr int kPfItems = 4 * kThreads;   // float4 items per prefetch workgroup
template <class J> struct Jobs {
  int n;
  int start[kMaxJobs + 1];
  J j[kMaxJobs];
};

// the job of workgroup bid: start[] is read whole and unconditionally (one
// scalar round trip, not one per job as a search loop's dependent loads)
__device__ __forceinline__ int find_job(const int *start, int n, int bid) {
  int q = 0;
#pragma unroll
  for (int i = 1; i < kMaxJobs; i++) q += (int)((bid >= start[i]) & (i < n));
  return q;
}

// One workgroup of a prefetch job: items tile * kPfItems + t + 256 i of the
// (row, float4 column) space, every id load and then every row load issued
// before the first store.
__device__ __forceinline__ void fwd_prefetch(const FwdJob &J, const Ctx &c, int tile) {
  Ctx cn = c;
  cn.pbase = J.pfbase;
  cn.M = J.pfM;
  const SrcK sa = src_k(J.a, cn);
  const int w4 = J.pfld >> 2;
  int m[4], k4[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int idx = tile * kPfItems + threadIdx.x + kThreads * i;
    m[i] = idx / w4;
    k4[i] = (idx - m[i] * w4) * 4;
  }
  SrcRow r[4];
  src_rows(sa, cn, m, r);
  float4 v[4];
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = src_raw4(sa, r[i], k4[i]);
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (m[i] < kPfRows)
      gst4(J.pfX + (int64_t)m[i] * J.pfld + k4[i], src_fix4(sa, r[i], k4[i], v[i], true));
}

// NCH > 0: exactly NCH reduction chunks, every chunk's operands loaded up
// front (straight-line code: no load waits on another, the wait before chunk
// ch is for chunk ch's loads only); NCH = 0: any K, one chunk ahead.
template <int NCH>
__global__ __launch_bounds__(kThreads) void mlp_fwd(Jobs<FwdJob> js, Ctx c) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][32 * 64];
  const int qj = find_job(js.start, js.n, blockIdx.x);
  const FwdJob &J = js.j[qj];
  const int tile = blockIdx.x - js.start[qj];
  if (J.pf) {
    fwd_prefetch(J, c, tile);
    return;
  }
  const int m0 = (tile / J.tiles_n) * kTile, n0 = (tile % J.tiles_n) * kTile;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  TDECL;
  TSTAMP(0);
  // the epilogue's bias, loaded before the GEMM (reduce_tile's column j)
  const float bias = J.b[n0 + (lane & 31)];
  f32x16 acc = {};
  if constexpr (NCH > 0) {
    const SrcK sa = src_k(J.a, c);
    SrcRow rr[1];
    src_rows(sa, c, {m0 + (t & 31)}, rr);
    const SrcRow &row0 = rr[0];
    TSTAMP(1);
    const int q4 = 4 * (t >> 5);  // pattern R2
    float4 ra0[NCH], ra1[NCH], rb0[NCH], rb1[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      const int r0 = ch * kChunk;
      ra0[ch] = src_raw4(sa, row0, r0 + q4);
      ra1[ch] = src_raw4(sa, row0, r0 + q4 + 32);
      const float *wp = J.W + (int64_t)(r0 + (t >> 3)) * J.ldw + n0 + 4 * (t & 7);
      rb0[ch] = *reinterpret_cast<const float4 *>(wp);
      rb1[ch] = *reinterpret_cast<const float4 *>(wp + (int64_t)32 * J.ldw);
    }
    TSTAMP(2);
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      float *As = lds[ch & 1][0], *Bs = lds[ch & 1][1];
      const int k4 = ch * kChunk + q4;
      store_R2(As, src_fix4(sa, row0, k4, ra0[ch], true),
               src_fix4(sa, row0, k4 + 32, ra1[ch], true));
      store_C(Bs, rb0[ch], rb1[ch]);
      __syncthreads();
      mma_chunk(As, Bs, acc, w, lane);
    }
  } else {
    const int nch = J.K / kChunk;
    float4 ra0, ra1, rb0, rb1;
    auto load = [&](int ch) {
      const int r0 = ch * kChunk;
      ra0 = src_load4(J.a, c, m0 + (t >> 4), r0 + 4 * (t & 15), true);
      ra1 = src_load4(J.a, c, m0 + (t >> 4) + 16, r0 + 4 * (t & 15), true);
      const float *wp = J.W + (int64_t)(r0 + (t >> 3)) * J.ldw + n0 + 4 * (t & 7);
      rb0 = *reinterpret_cast<const float4 *>(wp);
      rb1 = *reinterpret_cast<const float4 *>(wp + (int64_t)32 * J.ldw);
    };
    load(0);
    for (int ch = 0; ch < nch; ch++) {
      float *As = lds[ch & 1][0], *Bs = lds[ch & 1][1];
      store_R(As, ra0, ra1);
      store_C(Bs, rb0, rb1);
      __syncthreads();
      if (ch + 1 < nch) load(ch + 1);
      mma_chunk(As, Bs, acc, w, lane);
    }
  }
  float v[4];
  int i0, j;
  TSTAMP(3);
  reduce_tile(&lds[0][0][0], acc, v, i0, j);
  TSTAMP(4);
  const int n = n0 + j;
  float lsum = 0.f;
  // the four outputs first, with the activation chosen once per workgroup
  // (straight-line, so the four sigmoids and divisions interleave), then
  // the stores
  float ya[4];
  if (J.act == ACT_SIGMOID) {
#pragma unroll
    for (int e = 0; e < 4; e++) ya[e] = act_f(ACT_SIGMOID, v[e] + bias);
  } else {
#pragma unroll
    for (int e = 0; e < 4; e++) ya[e] = act_f(ACT_RELU, v[e] + bias);
  }
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int m = m0 + i0 + e;
    const bool valid = m < c.M && n < J.Nreal;
    const float y = valid ? ya[e] : 0.f;
    gst(&J.Y[(int64_t)m * J.ldy + n], y);
    if (J.loss) {
      float dz = 0.f;
      if (valid) {
        const float diff = y - src_at(J.tgt, c, m, n);
        lsum += diff * diff;
        dz = J.lw * 2.0f * diff / ((float)J.Nreal * (float)c.M) * act_d(J.act, y);
      }
      gst(&J.dZ[(int64_t)m * J.lddz + n], dz);
    }
  }
  if (J.loss) {
    // workgroup sum of the squared errors -> one partial per tile
    lsum = hgx::group_allreduce_sum<64>(lsum);
    __shared__ float wsum[4];
    if (lane == 0) wsum[w] = lsum;
    __syncthreads();
    if (t == 0)
      J.part[tile] = J.lw * (((wsum[0] + wsum[1]) + wsum[2]) + wsum[3]) /
                     ((float)J.Nreal * (float)c.M);
  }
  if constexpr (NCH > 0) {
    TSTAMP(5);
    TFLUSH(NCH == 8 ? (J.a.gather ? 0 : 2) : (NCH == 6 ? 1 : 6), 6);
  }
}

// ============================ HEAD =========================================
// The N = 1 label layer: y = act(H w + b); with a loss: MSE against the
// label, dz = lw 2 (y - t) / M act'(y) (stored in column 0 of dz4 for the
// weight gradient) and dZprev = dz w^T * act_prev'(H). One wave per 8 rows.
struct HeadJob {
  const float *H;
  int ldh, K;
  const float *W;  // column 0 of [K][ldw]
  int ldw;
  const float *b;
  int act, act_prev, loss;
  float lw;
  const float *label;  // indexed by pbase + m
  float *dZprev;
  int ldp;
  float *dz4;
  int ld4;
  float *y;            // optional output (predict)
  float *part;         // one partial per workgroup
};

// HEAD_KH: inputs of up to 64 * HEAD_KH columns are kept in registers
constexpr int kHeadKH = 8;

// One wave's 8 rows mb .. mb + 7 of the head. gstore: y, dz4 and dZprev to
// global memory; S (optional): dZprev also into LDS rows mb - m0 of S (row
// stride sld floats), every column k < K (rows past M zero). lsum: lane 0's
// sum of the squared errors of the wave's valid rows, in row order.
// ACT / ACTP >= 0: the head's / the previous layer's activation known at
// compile time (straight-line code the scheduler can interleave across the
// 8 rows: with one wave per SIMD a per-row activation branch left every
// dependent VALU step exposed); -1: read from h.
template <int ACT = -1, int ACTP = -1, int KH = kHeadKH>
__device__ __forceinline__ void head_wave_t(const HeadJob &h, const Ctx &c, int mb,
                                            int lane, bool gstore, float *S, int srow,
                                            int sld, float &lsum,
                                            unsigned long long *tsp = nullptr) {
  const int act = ACT >= 0 ? ACT : h.act, act_prev = ACTP >= 0 ? ACTP : h.act_prev;
  // Every load is issued, and consumed, before the first store: on this
  // architecture the vector-memory counter also counts stores, so a load
  // waited for after a store waits for that store too. The same arithmetic
  // in the same order per row as one row at a time: each row's fma chain in
  // k order, the loss summed over the wave's rows in order. Rows past M read
  // the batch's last row (their sums are never used).
  float lab[8];
#pragma unroll
  for (int s = 0; s < 8; s++)
    lab[s] = h.loss ? h.label[c.pbase + min(mb + s, c.M - 1)] : 0.f;
  const float bias = h.b[0];
  const bool regs = h.K <= 64 * KH;
  float zs[8], wv[KH], hv[KH][8];
#pragma unroll
  for (int s = 0; s < 8; s++) zs[s] = 0.f;
  if (regs) {
#pragma unroll
    for (int kk = 0; kk < KH; kk++) {
      const int k = min(lane + 64 * kk, h.K - 1);
      wv[kk] = h.W[(int64_t)k * h.ldw];
#pragma unroll
      for (int s = 0; s < 8; s++)
        hv[kk][s] = h.H[(int64_t)min(mb + s, c.M - 1) * h.ldh + k];
    }
#pragma unroll
    for (int kk = 0; kk < KH; kk++) {
      const bool in = lane + 64 * kk < h.K;
#pragma unroll
      for (int s = 0; s < 8; s++)
        zs[s] = in ? fmaf(hv[kk][s], wv[kk], zs[s]) : zs[s];
    }
  } else {
    for (int k = lane; k < h.K; k += 64) {
      const float wk = h.W[(int64_t)k * h.ldw];
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const int m = min(mb + s, c.M - 1);
        zs[s] = fmaf(h.H[(int64_t)m * h.ldh + k], wk, zs[s]);
      }
    }
  }
  HSTAMP(8);
  // the 8 rows' wave sums interleaved (group_allreduce_sum<64>'s bits)
  hgx::wave_allreduce_sum_n<8>(zs);
  HSTAMP(9);
  // Row s's output, error and delta computed by lanes s, s + 8, ... at once
  // and read back per row: eight rows one after another left every step of
  // the sigmoid and of two IEEE divisions exposed (the divisions' VCC
  // hand-off keeps them from interleaving). The same arithmetic per row.
  float ys[8], dzs[8];
  const bool loss = h.loss;
  {
    const int sr = lane & 7;
    float zr = zs[0], lr = lab[0];
#pragma unroll
    for (int s = 1; s < 8; s++) {
      zr = sr == s ? zs[s] : zr;
      lr = sr == s ? lab[s] : lr;
    }
    const bool validr = mb + sr < c.M;
    const float yr = act_f(act, (validr ? zr : 0.f) + bias);
    const float diffr = yr - lr;
    const float dzr =
        loss && validr ? h.lw * 2.0f * diffr / (float)c.M * act_d(act, yr) : 0.f;
#pragma unroll
    for (int s = 0; s < 8; s++) {
      ys[s] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(yr), s));
      dzs[s] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dzr), s));
      const float diff = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(diffr), s));
      const bool on = loss && mb + s < c.M;
      lsum = (on && lane == 0) ? lsum + diff * diff : lsum;
    }
  }
  HSTAMP(10);
  // stores
  if (gstore) {
#pragma unroll
    for (int s = 0; s < 8; s++) {
      const int m = mb + s;
      if (m < c.M && h.y && lane == 0) gst(&h.y[m], ys[s]);
      if (h.loss && lane == 0) gst(&h.dz4[(int64_t)m * h.ld4], dzs[s]);
    }
  }
  if (!h.loss) return;
  if (regs) {
    // every value first, then the LDS rows, then (one tile per row block)
    // the global copy: no store waits behind a per-element branch
    float dv[KH][8];
#pragma unroll
    for (int kk = 0; kk < KH; kk++)
#pragma unroll
      for (int s = 0; s < 8; s++)
        dv[kk][s] = mb + s < c.M ? dzs[s] * wv[kk] * act_d(act_prev, hv[kk][s]) : 0.f;
    if (S) {
#pragma unroll
      for (int kk = 0; kk < KH; kk++)
        if (lane + 64 * kk < h.K)
#pragma unroll
          for (int s = 0; s < 8; s++) S[(srow + s) * sld + lane + 64 * kk] = dv[kk][s];
    }
    if (gstore) {
#pragma unroll
      for (int kk = 0; kk < KH; kk++)
        if (lane + 64 * kk < h.K)
#pragma unroll
          for (int s = 0; s < 8; s++)
            gst(&h.dZprev[(int64_t)(mb + s) * h.ldp + lane + 64 * kk], dv[kk][s]);
    }
  } else {
    for (int k = lane; k < h.K; k += 64) {
      const float wk = h.W[(int64_t)k * h.ldw];
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const int m = mb + s;
        const bool valid = m < c.M;
        const float hvv = h.H[(int64_t)min(m, c.M - 1) * h.ldh + k];
        const float v = valid ? dzs[s] * wk * act_d(act_prev, hvv) : 0.f;
        if (gstore) gst(&h.dZprev[(int64_t)m * h.ldp + k], v);
        if (S) S[(srow + s) * sld + k] = v;
      }
    }
  }
}

// head_wave_t with the combiners' and the classifier's (sigmoid head over a
// relu layer) activations compiled in and the input's 64-column groups
// counted exactly (KH = 2 / 4: no clamped duplicate loads taking
// vector-memory counter slots), any other case read at run time
__device__ __forceinline__ void head_wave(const HeadJob &h, const Ctx &c, int mb, int lane,
                                          bool gstore, float *S, int srow, int sld,
                                          float &lsum, unsigned long long *tsp = nullptr) {
  if (h.act == ACT_SIGMOID && h.act_prev == ACT_RELU) {
    if (h.K <= 128)
      head_wave_t<ACT_SIGMOID, ACT_RELU, 2>(h, c, mb, lane, gstore, S, srow, sld, lsum, tsp);
    else if (h.K <= 256)
      head_wave_t<ACT_SIGMOID, ACT_RELU, 4>(h, c, mb, lane, gstore, S, srow, sld, lsum, tsp);
    else
      head_wave_t<ACT_SIGMOID, ACT_RELU>(h, c, mb, lane, gstore, S, srow, sld, lsum, tsp);
  } else {
    head_wave_t<>(h, c, mb, lane, gstore, S, srow, sld, lsum, tsp);
  }
}

// the workgroup's loss partial: the 4 waves' sums in wave order
__device__ __forceinline__ void head_partial(const HeadJob &h, const Ctx &c, int slot,
                                             float lsum) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  __shared__ float wsum[4];
  if (lane == 0) wsum[w] = lsum;
  __syncthreads();
  if (t == 0)
    h.part[slot] = h.lw * (((wsum[0] + wsum[1]) + wsum[2]) + wsum[3]) / (float)c.M;
}

__global__ __launch_bounds__(kThreads) void mlp_head(HeadJob h, Ctx c) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  float lsum = 0.f;
  head_wave(h, c, blockIdx.x * 32 + w * 8, lane, true, nullptr, 0, 0, lsum);
  if (h.loss) head_partial(h, c, blockIdx.x, lsum);
}

// ============================ BWD ==========================================
struct BwdTerm {
  const float *dz;  // [M][lddz]
  int lddz;
  const float *W;   // rows k of W_t (this input's rows), [.][ldw]
  int ldw, R;       // reduction length (multiple of 64)
};
struct BwdJob {
  BwdTerm tm[2];
  int nt;
  int act;           // activation of the layer that produced Y
  const float *Y;
  int ldy;
  float *dZ;         // output [M][ldo]
  int ldo, Kreal, tiles_n;
};

// FH (fused head, combiner training): term 0's delta rows are the label
// head's dZprev for rows m0 .. m0 + 31, computed here by head_wave exactly
// as mlp_head computes them (same arithmetic, same order) into LDS instead of
// being read from global memory; the first job's k0 = 0 tile of each row
// block also stores the head's outputs (dZprev, dz4, loss partial) for the
// weight gradients. Every tile of the row block recomputes the head for its
// 32 rows: it reads 32 hidden rows instead of 32 delta rows, and the head's
// own launch goes away.
constexpr int kHdLd = 256 + 4;  // LDS row stride of the fused head's rows

template <int NCH, bool FH = false>
__global__ __launch_bounds__(kThreads) void mlp_bwd(Jobs<BwdJob> js, Ctx c, HeadJob hj) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][32 * 64];
  __shared__ __attribute__((aligned(16))) float s_hd[FH ? 32 * kHdLd : 4];
  const int qj = find_job(js.start, js.n, blockIdx.x);
  const BwdJob &J = js.j[qj];
  const int tile = blockIdx.x - js.start[qj];
  const int m0 = (tile / J.tiles_n) * kTile, k0 = (tile % J.tiles_n) * kTile;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int nch0 = J.tm[0].R / kChunk;
  TDECL;
  TSTAMP(0);
  // the epilogue's activations, loaded before the GEMM (reduce_tile's
  // rows i0 .. i0 + 3 of column j; clamped, used only where in range)
  float ypre[4];
  {
    const int i0p = 8 * w + 4 * (lane >> 5), kp = min(k0 + (lane & 31), J.Kreal - 1);
#pragma unroll
    for (int e = 0; e < 4; e++)
      ypre[e] = J.Y[(int64_t)min(m0 + i0p + e, c.M - 1) * J.ldy + kp];
  }
  f32x16 acc = {};
  if constexpr (NCH > 0) {
    // all NCH chunks' loads up front, unconditional (rows past M read row 0
    // and are zeroed when stored)
    // pattern R2 for both operands: row i = t & 31, reduction r4, r4 + 32
    const int row = t & 31, ma = m0 + row, q4 = 4 * (t >> 5);
    const bool oka = ma < c.M;
    float4 ra0[NCH], ra1[NCH], rb0[NCH], rb1[NCH];
    // both terms' fields pinned in scalar registers (see SrcK)
    const gfp dzt[2] = {gpin(J.tm[0].dz), gpin(J.tm[1].dz)};
    const gfp Wt[2] = {gpin(J.tm[0].W), gpin(J.tm[1].W)};
    const int lddzt[2] = {spin(J.tm[0].lddz), spin(J.tm[1].lddz)};
    const int ldwt[2] = {spin(J.tm[0].ldw), spin(J.tm[1].ldw)};
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      const bool first = ch < nch0;
      const gfp dz = first ? dzt[0] : dzt[1];
      const gfp W = first ? Wt[0] : Wt[1];
      const int lddz = first ? lddzt[0] : lddzt[1];
      const int ldw = first ? ldwt[0] : ldwt[1];
      const int r4 = (first ? ch : ch - nch0) * kChunk + q4;
      const gfp dr = dz + (int64_t)(oka ? ma : 0) * lddz + r4;
      const gfp wr = W + (int64_t)(k0 + row) * ldw + r4;
      if (!(FH && first)) {
        ra0[ch] = ldg4(dr);
        ra1[ch] = ldg4(dr + 32);
      }
      rb0[ch] = ldg4(wr);
      rb1[ch] = ldg4(wr + 32);
    }
    TSTAMP(1);
    if constexpr (FH) {
      float lsum = 0.f;
      const bool gst = qj == 0 && k0 == 0;
#if HGX_MLP_DIAG_TIME
      head_wave(hj, c, m0 + w * 8, lane, gst, s_hd, w * 8, kHdLd, lsum, ts);
#else
      head_wave(hj, c, m0 + w * 8, lane, gst, s_hd, w * 8, kHdLd, lsum);
#endif
      TSTAMP(6);
      if (gst) head_partial(hj, c, m0 / kTile, lsum);
      __syncthreads();
      TSTAMP(7);
#pragma unroll
      for (int ch = 0; ch < NCH; ch++) {
        if (ch < nch0) {
          const float *sr = s_hd + row * kHdLd + ch * kChunk + q4;
          ra0[ch] = *reinterpret_cast<const float4 *>(sr);
          ra1[ch] = *reinterpret_cast<const float4 *>(sr + 32);
        }
      }
    }
    TSTAMP(2);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      float *As = lds[ch & 1][0], *Bs = lds[ch & 1][1];
      store_R2(As, oka ? ra0[ch] : z4, oka ? ra1[ch] : z4);
      store_R2(Bs, rb0[ch], rb1[ch]);
      __syncthreads();
      mma_chunk(As, Bs, acc, w, lane);
    }
  } else {
    const int nch = nch0 + (J.nt > 1 ? J.tm[1].R / kChunk : 0);
    float4 ra0, ra1, rb0, rb1;
    auto load = [&](int ch) {
      const BwdTerm &T = ch < nch0 ? J.tm[0] : J.tm[1];
      const int r0 = (ch < nch0 ? ch : ch - nch0) * kChunk;
      const int r4 = r0 + 4 * (t & 15);
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      const int row = t >> 4, m = m0 + row;
      ra0 = z4;
      ra1 = z4;
      if (m < c.M) ra0 = *reinterpret_cast<const float4 *>(T.dz + (int64_t)m * T.lddz + r4);
      if (m + 16 < c.M)
        ra1 = *reinterpret_cast<const float4 *>(T.dz + (int64_t)(m + 16) * T.lddz + r4);
      rb0 = *reinterpret_cast<const float4 *>(T.W + (int64_t)(k0 + row) * T.ldw + r4);
      rb1 = *reinterpret_cast<const float4 *>(T.W + (int64_t)(k0 + row + 16) * T.ldw + r4);
    };
    load(0);
    for (int ch = 0; ch < nch; ch++) {
      float *As = lds[ch & 1][0], *Bs = lds[ch & 1][1];
      store_R(As, ra0, ra1);
      store_R(Bs, rb0, rb1);
      __syncthreads();
      if (ch + 1 < nch) load(ch + 1);
      mma_chunk(As, Bs, acc, w, lane);
    }
  }
  float v[4];
  int i0, j;
  TSTAMP(3);
  reduce_tile(&lds[0][0][0], acc, v, i0, j);
  TSTAMP(4);
  const int k = k0 + j;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int m = m0 + i0 + e;
    const float d = (m < c.M && k < J.Kreal) ? v[e] * act_d(J.act, ypre[e]) : 0.f;
    gst(&J.dZ[(int64_t)m * J.ldo + k], d);
  }
  if constexpr (NCH > 0) {
    TSTAMP(5);
    TFLUSH(FH ? 3 : 4, FH ? 11 : 6);
  }
}

// ============================ WGRAD ========================================
struct WgJob {
  Src a;              // the layer's input (same gather / dropout as FWD)
  const float *dZ;
  int lddz;
  float *W, *aW, *b, *ab;
  int ldw, tiles_n;
  int gemm_tiles;     // tiles past these are the bias's (one per column tile)
};

// A bias workgroup of WGRAD: column sums of dZ over the batch rows for columns
// n0 .. n0 + 31 (8 row groups per column, each summed in row order, then the
// groups in order) and the bias's Adagrad step. Its own workgroups, run beside
// the GEMM tiles, with every load issued up front: appended to the k0 = 0 GEMM
// tiles (before r04) its dependent load rounds were the launch's tail.
__device__ __forceinline__ void wgrad_bias(const WgJob &J, const Ctx &c, int n0, float *bs) {
  const int t = threadIdx.x, col = t & 31, grp = t >> 5;
  float bb = 0.f, ba = 0.f;
  if (t < 32) {
    bb = J.b[n0 + t];
    ba = J.ab[n0 + t];
  }
  float dv[32];
#pragma unroll
  for (int i = 0; i < 32; i++)
    dv[i] = J.dZ[(int64_t)min(grp + 8 * i, c.M - 1) * J.lddz + n0 + col];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 32; i++)
    if (grp + 8 * i < c.M) s += dv[i];
  for (int m = grp + 256; m < c.M; m += 8) s += J.dZ[(int64_t)m * J.lddz + n0 + col];
  bs[grp * 32 + col] = s;
  __syncthreads();
  if (t < 32) {
    float g = 0.f;
#pragma unroll
    for (int q = 0; q < 8; q++) g += bs[q * 32 + t];
    const int nn = n0 + t;
    if (c.grad_only) {
      gst(&J.b[nn], g);
      return;
    }
    const float na = ba + g * g;
    gst(&J.ab[nn], na);
    gst(&J.b[nn], bb - (c.lr * g) / (sqrtf(na) + c.eps));
  }
}

template <int NCH>
__global__ __launch_bounds__(kThreads) void mlp_wgrad(Jobs<WgJob> js, Ctx c) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][32 * 64];
  const int qj = find_job(js.start, js.n, blockIdx.x);
  const WgJob &J = js.j[qj];
  const int tile = blockIdx.x - js.start[qj];
  if (tile >= J.gemm_tiles) {
    wgrad_bias(J, c, (tile - J.gemm_tiles) * kTile, &lds[0][0][0]);
    return;
  }
  const int k0 = (tile / J.tiles_n) * kTile, n0 = (tile % J.tiles_n) * kTile;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  // the Adagrad operands of the 4 elements this thread updates (reduce_tile's
  // mapping), loaded before the GEMM so the update needs no further round trip
  float pW[4], pA[4];
  {
    const int e0 = 8 * w + 4 * (lane >> 5), jn = n0 + (lane & 31);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t q = (int64_t)(k0 + e0 + e) * J.ldw + jn;
      pW[e] = J.W[q];
      pA[e] = J.aW[q];
    }
  }
  f32x16 acc = {};
  TDECL;
  TSTAMP(0);
  if constexpr (NCH > 0) {
    // the reduction runs over the batch rows: every chunk's input rows
    // resolved (ids in one round trip), then all chunks' loads up front
    const SrcK sa = src_k(J.a, c);
    int mr[2 * NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      mr[2 * ch] = ch * kChunk + (t >> 3);
      mr[2 * ch + 1] = ch * kChunk + (t >> 3) + 32;
    }
    SrcRow rows[2 * NCH];
    src_rows(sa, c, mr, rows);
    TSTAMP(1);
    const int kk = k0 + 4 * (t & 7);
    float4 xa0[NCH], xa1[NCH], d0[NCH], d1[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      const int m = ch * kChunk + (t >> 3);
      xa0[ch] = src_raw4(sa, rows[2 * ch], kk);
      xa1[ch] = src_raw4(sa, rows[2 * ch + 1], kk);
      const float *dp = J.dZ + n0 + 4 * (t & 7);
      d0[ch] = *reinterpret_cast<const float4 *>(dp + (int64_t)(m < c.M ? m : 0) * J.lddz);
      d1[ch] = *reinterpret_cast<const float4 *>(dp + (int64_t)(m + 32 < c.M ? m + 32 : 0) * J.lddz);
    }
    TSTAMP(2);
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      const int m = ch * kChunk + (t >> 3);
      float *As = lds[ch & 1][0], *Bs = lds[ch & 1][1];
      store_C(As, src_fix4(sa, rows[2 * ch], kk, xa0[ch], true),
              src_fix4(sa, rows[2 * ch + 1], kk, xa1[ch], true));
      store_C(Bs, m < c.M ? d0[ch] : z4, m + 32 < c.M ? d1[ch] : z4);
      __syncthreads();
      mma_chunk(As, Bs, acc, w, lane);
    }
  } else {
    const int nch = (c.M + kChunk - 1) / kChunk;
    float4 ra0, ra1, rb0, rb1;
    auto load = [&](int ch) {
      const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
      const int m = ch * kChunk + (t >> 3);
      ra0 = src_load4(J.a, c, m, k0 + 4 * (t & 7), true);
      ra1 = src_load4(J.a, c, m + 32, k0 + 4 * (t & 7), true);
      const float *dp = J.dZ + (int64_t)m * J.lddz + n0 + 4 * (t & 7);
      rb0 = z4;
      rb1 = z4;
      if (m < c.M) rb0 = *reinterpret_cast<const float4 *>(dp);
      if (m + 32 < c.M) rb1 = *reinterpret_cast<const float4 *>(dp + (int64_t)32 * J.lddz);
    };
    load(0);
    for (int ch = 0; ch < nch; ch++) {
      float *As = lds[ch & 1][0], *Bs = lds[ch & 1][1];
      store_C(As, ra0, ra1);
      store_C(Bs, rb0, rb1);
      __syncthreads();
      if (ch + 1 < nch) load(ch + 1);
      mma_chunk(As, Bs, acc, w, lane);
    }
  }
  float v[4];
  int i0, j;
  TSTAMP(3);
  reduce_tile(&lds[0][0][0], acc, v, i0, j);
  TSTAMP(4);
  const int n = n0 + j;
  if (c.grad_only) {
#pragma unroll
    for (int e = 0; e < 4; e++) gst(&J.W[(int64_t)(k0 + i0 + e) * J.ldw + n], v[e]);
  } else {
    // the four Adagrad steps first (their square roots and divisions
    // interleave), then the stores. Plain sqrtf is correctly rounded on
    // gfx950 (__fsqrt_rn is not: 15% of 1M inputs off by an ulp,
    // tools/fp_check.hip), as the CPU side's is
    float na[4], nw[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const float g = v[e];
      na[e] = pA[e] + g * g;
      nw[e] = pW[e] - (c.lr * g) / (sqrtf(na[e]) + c.eps);
    }
#ifndef HGX_MLP_PROBE_ST
#define HGX_MLP_PROBE_ST 0
#endif
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int64_t q = (int64_t)(k0 + i0 + e) * J.ldw + n;
      // probe builds only (results wrong): 1 no accumulator stores, 2 no
      // weight-gradient tile stores at all
      if (HGX_MLP_PROBE_ST == 0) gst(&J.aW[q], na[e]);
      if (HGX_MLP_PROBE_ST < 2) gst(&J.W[q], nw[e]);
    }
  }
  if constexpr (NCH > 0) {
    TSTAMP(5);
    TFLUSH(5, 6);
  }
}

// ============================ epoch plumbing ===============================
__global__ void mlp_shuffle_keys(uint64_t seed, int epoch, int64_t n,
                                 unsigned long long *keys, int *vals) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = hgx::rand64(seed, 0x4d4c5053ull + epoch, (uint64_t)i);
    vals[i] = (int)i;
  }
}

__global__ void mlp_permute(const int *perm, int64_t n, const int *nr,
                            const int *er, const float *lab, int *pn, int *pe,
                            float *pl) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int s = perm[i];
    pn[i] = nr[s];
    pe[i] = er[s];
    pl[i] = lab[s];
  }
}

// per batch: sum of its loss partials in slot order
__global__ void mlp_loss_reduce(const float *part, int nslot, int nb,
                                double *out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  double s = 0.0;
  for (int q = 0; q < nslot; q++) s += (double)part[(int64_t)b * nslot + q];
  out[b] = s;
}

int round_up(int x, int a) { return (x + a - 1) / a * a; }
unsigned grid_for(int64_t n, int tb) {
  return (unsigned)std::min<int64_t>((n + tb - 1) / tb, 4096);
}

}  // namespace

// ============================ host plan ====================================
struct MlpLayer {
  int Kext, N;          // Keras kernel shape
  int Kp, Np;           // internal (padded) shape
  int act;
  // external input row e -> internal row: e < seg ? e : off + (e - seg)
  int seg, off;
  DevBuf W, b, aW, ab;
};

struct hgx_mlp {
  hgx_ctx *ctx = nullptr;
  int kind = 0, in = 0, out = 0, hid = 0;
  std::vector<MlpLayer> L;
  // layer indices (Keras creation order; -1 = absent)
  int pre_n = -1, pre_e = -1, joint_n = -1, joint_e = -1, post_n = -1,
      post_e = -1, rec_n = -1, rec_e = -1, hidden = -1, label = -1;
  // tables (row stride ldt, zero padded) and samples
  DevBuf tn, te;
  int ldt = 0, twidth = 0;
  int64_t tn_rows = 0, te_rows = 0;
  DevBuf s_node, s_edge, s_label;
  int64_t ns = 0;
  // activations [kMcap][*] and deltas [256][*]
  DevBuf A_hn, A_he, A_j, A_hm, A_pn, A_pe, A_rn, A_re, A_y;
  DevBuf D_hn, D_he, D_jn, D_je, D_hm, D_4, D_pn, D_pe, D_rn, D_re;
  int ldJ = 0;
  // epoch scratch
  DevBuf perm, p_node, p_edge, p_label, keys, part, bloss, sort_tmp, idx_a, idx_b;
  DevBuf xpf[2];  // prefetched input rows, alternating by batch (run_batch)
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double ms = 0, flops = 0;
  int64_t samples = 0, batches = 0;
};

namespace {

int new_layer(hgx_mlp *m, int Kext, int N, int Kp, int act, int seg, int off) {
  MlpLayer l;
  l.Kext = Kext;
  l.N = N;
  l.Kp = Kp;
  l.Np = round_up(N, 64);
  l.act = act;
  l.seg = seg;
  l.off = off;
  m->L.push_back(l);
  return (int)m->L.size() - 1;
}

int alloc_zero(hgx_ctx *ctx, DevBuf &b, size_t bytes) {
  HGX_TRY(hgx_ensure(ctx, b, bytes));
  HGX_HIP(ctx, hipMemsetAsync(b.p, 0, bytes, ctx->stream));
  return HGX_OK;
}

Src dense(const DevBuf &b, int ld, int width, int coloff = 0) {
  Src s{};
  s.x = b.as<float>() + coloff;
  s.ldx = ld;
  s.width = width;
  return s;
}

// the first layer's input: kind 0 = [node_tab row | edge_tab row] (no
// dropout); kinds 1/2 = one table row with dropout (tower 0 node, 1 edge)
Src gather_src(const hgx_mlp *m, int tower, const int *pn, const int *pe,
               uint32_t dstream, bool drop) {
  Src s{};
  s.gather = 1;
  if (m->kind == HGX_MLP_LP_CLASSIFIER) {
    s.t0 = m->tn.as<float>();
    s.i0 = pn;
    s.ld0 = m->ldt;
    s.t1 = m->te.as<float>();
    s.i1 = pe;
    s.ld1 = m->ldt;
    s.c1 = m->ldt;
    s.width = 2 * m->ldt;
  } else {
    s.t0 = tower == 0 ? m->tn.as<float>() : m->te.as<float>();
    s.i0 = tower == 0 ? pn : pe;
    s.ld0 = m->ldt;
    s.c1 = m->ldt;
    s.t1 = s.t0;
    s.i1 = s.i0;
    s.ld1 = m->ldt;
    s.width = m->ldt;
    s.drop = drop ? 1 : 0;
    s.dstream = dstream + (uint32_t)tower;
  }
  return s;
}

template <class J>
int launch_jobs(hgx_ctx *ctx, void (*kern)(Jobs<J>, Ctx), const J *jobs,
                const int *tiles, int n, const Ctx &c) {
  Jobs<J> js{};
  js.n = n;
  int tot = 0;
  for (int q = 0; q < n; q++) {
    js.start[q] = tot;
    js.j[q] = jobs[q];
    tot += tiles[q];
  }
  js.start[n] = tot;
  if (tot == 0) return HGX_OK;
  hipLaunchKernelGGL(kern, dim3(tot), dim3(kThreads), 0, ctx->stream, js, c);
  return HGX_OK;
}

// FWD launch: the all-chunks-in-flight instantiation when every job of the
// launch has the same K of 2..8 chunks, else the generic one (same results:
// identical chunk order and wave split)
int launch_fwd(hgx_ctx *ctx, const FwdJob *jobs, const int *tiles, int n,
               const Ctx &c) {
  int nch = n > 0 ? jobs[0].K / kChunk : 0;
  for (int q = 1; q < n; q++)
    if (!jobs[q].pf && jobs[q].K != jobs[0].K) nch = 0;
  switch (nch) {
    case 2: return launch_jobs(ctx, mlp_fwd<2>, jobs, tiles, n, c);
    case 3: return launch_jobs(ctx, mlp_fwd<3>, jobs, tiles, n, c);
    case 4: return launch_jobs(ctx, mlp_fwd<4>, jobs, tiles, n, c);
    case 5: return launch_jobs(ctx, mlp_fwd<5>, jobs, tiles, n, c);
    case 6: return launch_jobs(ctx, mlp_fwd<6>, jobs, tiles, n, c);
    case 7: return launch_jobs(ctx, mlp_fwd<7>, jobs, tiles, n, c);
    case 8: return launch_jobs(ctx, mlp_fwd<8>, jobs, tiles, n, c);
    default: return launch_jobs(ctx, mlp_fwd<0>, jobs, tiles, n, c);
  }
}

// BWD: every job of the launch with the same total chunk count (2..8); hj:
// the label head fused into this launch (fused_head_ok), else null
bool fused_head_ok(const HeadJob &h, const BwdJob *jobs, int n) {
  if (h.K > 256 || h.K % kChunk) return false;
  for (int q = 0; q < n; q++)
    if (jobs[q].tm[0].R != h.K) return false;
  return true;
}

int launch_bwd(hgx_ctx *ctx, const BwdJob *jobs, const int *tiles, int n,
               const Ctx &c, const HeadJob *hj = nullptr) {
  auto chunks = [](const BwdJob &j) {
    return j.tm[0].R / kChunk + (j.nt > 1 ? j.tm[1].R / kChunk : 0);
  };
  int nch = n > 0 ? chunks(jobs[0]) : 0;
  for (int q = 1; q < n; q++)
    if (chunks(jobs[q]) != nch) nch = 0;
  const HeadJob h = hj ? *hj : HeadJob{};
  auto go = [&](auto kern) {
    Jobs<BwdJob> js{};
    js.n = n;
    int tot = 0;
    for (int q = 0; q < n; q++) {
      js.start[q] = tot;
      js.j[q] = jobs[q];
      tot += tiles[q];
    }
    js.start[n] = tot;
    if (tot == 0) return HGX_OK;
    hipLaunchKernelGGL(kern, dim3(tot), dim3(kThreads), 0, ctx->stream, js, c, h);
    return HGX_OK;
  };
  if (hj) {
    HGX_CHECK(ctx, nch >= 1 && nch <= 8 && fused_head_ok(h, jobs, n), HGX_EINVAL,
              "fused head: unsupported layer shape");
    switch (nch) {
      case 1: return go(mlp_bwd<1, true>);
      case 2: return go(mlp_bwd<2, true>);
      case 3: return go(mlp_bwd<3, true>);
      case 4: return go(mlp_bwd<4, true>);
      case 5: return go(mlp_bwd<5, true>);
      case 6: return go(mlp_bwd<6, true>);
      case 7: return go(mlp_bwd<7, true>);
      default: return go(mlp_bwd<8, true>);
    }
  }
  switch (nch) {
    case 2: return go(mlp_bwd<2>);
    case 3: return go(mlp_bwd<3>);
    case 4: return go(mlp_bwd<4>);
    case 5: return go(mlp_bwd<5>);
    case 6: return go(mlp_bwd<6>);
    case 7: return go(mlp_bwd<7>);
    case 8: return go(mlp_bwd<8>);
    default: return go(mlp_bwd<0>);
  }
}

// WGRAD: the reduction is the batch (M rows): 1..4 chunks at batch <= 256
int launch_wgrad(hgx_ctx *ctx, const WgJob *jobs, const int *tiles, int n,
                 const Ctx &c) {
  switch ((c.M + kChunk - 1) / kChunk) {
    case 1: return launch_jobs(ctx, mlp_wgrad<1>, jobs, tiles, n, c);
    case 2: return launch_jobs(ctx, mlp_wgrad<2>, jobs, tiles, n, c);
    case 3: return launch_jobs(ctx, mlp_wgrad<3>, jobs, tiles, n, c);
    case 4: return launch_jobs(ctx, mlp_wgrad<4>, jobs, tiles, n, c);
    default: return launch_jobs(ctx, mlp_wgrad<0>, jobs, tiles, n, c);
  }
}

FwdJob fwd_job(const hgx_mlp *m, int li, const Src &a, float *Y, int ldy) {
  const MlpLayer &l = m->L[li];
  FwdJob j{};
  j.a = a;
  j.K = l.Kp;
  j.W = l.W.as<float>();
  j.b = l.b.as<float>();
  j.ldw = l.Np;
  j.tiles_n = l.Np / kTile;
  j.Nreal = l.N;
  j.act = l.act;
  j.Y = Y;
  j.ldy = ldy;
  return j;
}

WgJob wg_job(const hgx_mlp *m, int li, const Src &a, const DevBuf &dz, int lddz) {
  const MlpLayer &l = m->L[li];
  WgJob j{};
  j.a = a;
  j.dZ = dz.as<float>();
  j.lddz = lddz;
  j.W = l.W.as<float>();
  j.aW = l.aW.as<float>();
  j.b = l.b.as<float>();
  j.ab = l.ab.as<float>();
  j.ldw = l.Np;
  j.tiles_n = l.Np / kTile;
  j.gemm_tiles = (l.Kp / kTile) * j.tiles_n;
  return j;
}

BwdTerm term(const hgx_mlp *m, int li, const DevBuf &dz, int row0) {
  const MlpLayer &l = m->L[li];
  BwdTerm t{};
  t.dz = dz.as<float>();
  t.lddz = l.Np;
  t.W = l.W.as<float>() + (int64_t)row0 * l.Np;
  t.ldw = l.Np;
  t.R = l.Np;
  return t;
}

double layer_flops(const MlpLayer &l, int M, bool dx) {
  return 2.0 * M * l.Kext * l.N * (dx ? 3.0 : 2.0);
}

// Launches of one batch (training) or one chunk (predict, train = false).
// pn/pe: sample ids by position; slot: this batch's loss partials.
// Prefetch (combiner training): xin, when set, holds this batch's dropped-out
// input rows ([node | edge] blocks of kPfRows rows, stride ldt), written by the
// previous batch; xout, when set, receives the rows of the batch at position
// next_pbase (next_M samples) from this batch's hidden-layer launch.
int run_batch(hgx_mlp *m, const Ctx &c, const int *pn, const int *pe,
              const float *plab, uint32_t dstream, bool train, int upto,
              float *slot, float *yout, float *xin = nullptr, float *xout = nullptr,
              int64_t next_pbase = 0, int next_M = 0) {
  hgx_ctx *ctx = m->ctx;
  const int tm = (c.M + kTile - 1) / kTile;
  std::vector<MlpLayer> &L = m->L;
  auto tiles = [&](int li) { return tm * (L[li].Np / kTile); };
  if (m->kind == HGX_MLP_LP_CLASSIFIER) {
    const int l1 = m->pre_n, l2 = m->label;
    const Src in = gather_src(m, 0, pn, pe, dstream, false);
    FwdJob f = fwd_job(m, l1, in, m->A_hn.as<float>(), L[l1].Np);
    int tl = tiles(l1);
    HGX_TRY(launch_fwd(ctx, &f, &tl, 1, c));
    HeadJob h{};
    h.H = m->A_hn.as<float>();
    h.ldh = L[l1].Np;
    h.K = L[l2].Kp;
    h.W = L[l2].W.as<float>();
    h.ldw = L[l2].Np;
    h.b = L[l2].b.as<float>();
    h.act = L[l2].act;
    h.act_prev = L[l1].act;
    h.loss = train;
    h.lw = 1.0f;
    h.label = plab;
    h.dZprev = m->D_hn.as<float>();
    h.ldp = L[l1].Np;
    h.dz4 = m->D_4.as<float>();
    h.ld4 = L[l2].Np;
    h.y = yout;
    h.part = slot;
    hipLaunchKernelGGL(mlp_head, dim3(tm), dim3(kThreads), 0, ctx->stream, h, c);
    if (!train) return HGX_OK;
    WgJob wj[2] = {wg_job(m, l1, in, m->D_hn, L[l1].Np),
                   wg_job(m, l2, dense(m->A_hn, L[l1].Np, L[l1].Np), m->D_4, L[l2].Np)};
    int wt[2] = {wj[0].gemm_tiles + wj[0].tiles_n, wj[1].gemm_tiles + wj[1].tiles_n};
    return launch_wgrad(ctx, wj, wt, 2, c);
  }
  // combiners
  const bool ae = m->kind == HGX_MLP_NE_SEMI_SUPERVISED && train;
  const int a = m->pre_n, b = m->pre_e, jn = m->joint_n, je = m->joint_e,
            hd = m->hidden, lb = m->label;
  const int NpJ = L[jn].Np;  // J = [J_n | J_e], each NpJ wide
  Src in_n = gather_src(m, 0, pn, pe, dstream, train);
  Src in_e = gather_src(m, 1, pn, pe, dstream, train);
  if (xin) {
    const int64_t side = (int64_t)kPfRows * m->ldt;
    in_n = Src{};
    in_n.x = xin;
    in_e = Src{};
    in_e.x = xin + side;
    in_n.ldx = in_e.ldx = m->ldt;
    in_n.width = in_e.width = m->ldt;
  }
  // the next batch's input rows, on the CUs a launch leaves idle (tuning
  // mlp_prefetch: 1 the hidden layer's launch, 2 the joint layers')
  auto add_prefetch = [&](FwdJob *f, int *tl, int &n) {
    for (int q = 0; q < 2; q++) {
      FwdJob p{};
      p.pf = 1;
      p.K = f[0].K;
      p.a = gather_src(m, q, pn, pe, dstream, true);
      p.pfX = xout + (int64_t)q * kPfRows * m->ldt;
      p.pfld = m->ldt;
      p.pfbase = next_pbase;
      p.pfM = next_M;
      f[n] = p;
      tl[n++] = (kPfRows * (m->ldt / 4) + kPfItems - 1) / kPfItems;
    }
  };
  {  // stage 1: pre layers
    const int which = upto;  // predict: 1 = node side only, 2 = edge only
    FwdJob f[4];
    int tl[4], n = 0;
    if (which != 2) {
      f[n] = fwd_job(m, a, in_n, m->A_hn.as<float>(), L[a].Np);
      tl[n++] = tiles(a);
    }
    if (which != 1) {
      f[n] = fwd_job(m, b, in_e, m->A_he.as<float>(), L[b].Np);
      tl[n++] = tiles(b);
    }
    HGX_TRY(launch_fwd(ctx, f, tl, n, c));
    n = 0;
    if (which != 2) {
      f[n] = fwd_job(m, jn, dense(m->A_hn, L[a].Np, L[a].Np), m->A_j.as<float>(), m->ldJ);
      tl[n++] = tiles(jn);
    }
    if (which != 1) {
      f[n] = fwd_job(m, je, dense(m->A_he, L[b].Np, L[b].Np), m->A_j.as<float>() + NpJ,
                     m->ldJ);
      tl[n++] = tiles(je);
    }
    if (xout && ctx->tune.mlp_prefetch == 2) add_prefetch(f, tl, n);
    HGX_TRY(launch_fwd(ctx, f, tl, n, c));
    if (which == 1 || which == 2) return HGX_OK;
  }
  {  // stage 3: merged hidden (+ post layers)
    FwdJob f[5];
    int tl[5], n = 0;
    f[n] = fwd_job(m, hd, dense(m->A_j, m->ldJ, 2 * NpJ), m->A_hm.as<float>(), L[hd].Np);
    tl[n++] = tiles(hd);
    if (xout && ctx->tune.mlp_prefetch == 1) add_prefetch(f, tl, n);
    if (ae) {
      f[n] = fwd_job(m, m->post_n, dense(m->A_j, m->ldJ, NpJ), m->A_pn.as<float>(),
                     L[m->post_n].Np);
      tl[n++] = tiles(m->post_n);
      f[n] = fwd_job(m, m->post_e, dense(m->A_j, m->ldJ, NpJ, NpJ), m->A_pe.as<float>(),
                     L[m->post_e].Np);
      tl[n++] = tiles(m->post_e);
    }
    HGX_TRY(launch_fwd(ctx, f, tl, n, c));
  }
  HeadJob h{};
  h.H = m->A_hm.as<float>();
  h.ldh = L[hd].Np;
  h.K = L[lb].Kp;
  h.W = L[lb].W.as<float>();
  h.ldw = L[lb].Np;
  h.b = L[lb].b.as<float>();
  h.act = L[lb].act;
  h.act_prev = L[hd].act;
  h.loss = train;
  h.lw = m->kind == HGX_MLP_NE_SEMI_SUPERVISED ? 4.0f : 1.0f;
  h.label = plab;
  h.dZprev = m->D_hm.as<float>();
  h.ldp = L[hd].Np;
  h.dz4 = m->D_4.as<float>();
  h.ld4 = L[lb].Np;
  h.y = yout;
  h.part = slot;
  // training: the head rides in the joint layers' delta launch below when
  // its shape allows (tuning mlp_fuse_head)
  const int nchj = L[hd].Np / kChunk + (ae ? L[m->post_n].Np / kChunk : 0);
  const bool fuse = train && ctx->tune.mlp_fuse_head && L[lb].Kp <= 256 &&
                    L[hd].Np == L[lb].Kp && nchj <= 8;
  if (!fuse)
    hipLaunchKernelGGL(mlp_head, dim3(tm), dim3(kThreads), 0, ctx->stream, h, c);
  if (!train) return HGX_OK;
  if (ae) {  // reconstruction layers with the loss epilogue
    const int rn = m->rec_n, re = m->rec_e;
    FwdJob f[2] = {fwd_job(m, rn, dense(m->A_pn, L[m->post_n].Np, L[m->post_n].Np),
                           m->A_rn.as<float>(), L[rn].Np),
                   fwd_job(m, re, dense(m->A_pe, L[m->post_e].Np, L[m->post_e].Np),
                           m->A_re.as<float>(), L[re].Np)};
    const DevBuf *dzb[2] = {&m->D_rn, &m->D_re};
    for (int q = 0; q < 2; q++) {
      f[q].loss = 1;
      f[q].lw = 1.0f;
      f[q].tgt = gather_src(m, q, pn, pe, dstream, false);
      f[q].dZ = dzb[q]->as<float>();
      f[q].lddz = L[q ? re : rn].Np;
    }
    f[0].part = slot + 8;
    f[1].part = slot + 8 + tiles(rn);
    int tl[2] = {tiles(rn), tiles(re)};
    HGX_TRY(launch_fwd(ctx, f, tl, 2, c));
    // dZ of the post layers
    BwdJob bj[2] = {};
    const int po[2] = {m->post_n, m->post_e};
    const DevBuf *pa[2] = {&m->A_pn, &m->A_pe}, *pd[2] = {&m->D_pn, &m->D_pe};
    int bt[2];
    for (int q = 0; q < 2; q++) {
      bj[q].tm[0] = term(m, q ? re : rn, *dzb[q], 0);
      bj[q].nt = 1;
      bj[q].act = L[po[q]].act;
      bj[q].Y = pa[q]->as<float>();
      bj[q].ldy = L[po[q]].Np;
      bj[q].dZ = pd[q]->as<float>();
      bj[q].ldo = L[po[q]].Np;
      bj[q].Kreal = L[po[q]].N;
      bj[q].tiles_n = L[po[q]].Np / kTile;
      bt[q] = tiles(po[q]);
    }
    HGX_TRY(launch_bwd(ctx, bj, bt, 2, c));
  }
  {  // dZ of the joint layers: from the merged hidden layer (+ post layers)
    BwdJob bj[2] = {};
    const int jl[2] = {jn, je};
    const DevBuf *jd[2] = {&m->D_jn, &m->D_je};
    int bt[2];
    for (int q = 0; q < 2; q++) {
      bj[q].tm[0] = term(m, hd, m->D_hm, q * NpJ);
      bj[q].nt = 1;
      if (ae) {
        bj[q].tm[1] = term(m, q ? m->post_e : m->post_n, q ? m->D_pe : m->D_pn, 0);
        bj[q].nt = 2;
      }
      bj[q].act = L[jl[q]].act;
      bj[q].Y = m->A_j.as<float>() + q * NpJ;
      bj[q].ldy = m->ldJ;
      bj[q].dZ = jd[q]->as<float>();
      bj[q].ldo = NpJ;
      bj[q].Kreal = L[jl[q]].N;
      bj[q].tiles_n = NpJ / kTile;
      bt[q] = tiles(jl[q]);
    }
    HGX_TRY(launch_bwd(ctx, bj, bt, 2, c, fuse ? &h : nullptr));
  }
  {  // dZ of the pre layers
    BwdJob bj[2] = {};
    const int pl[2] = {a, b}, jl[2] = {jn, je};
    const DevBuf *ya[2] = {&m->A_hn, &m->A_he}, *yd[2] = {&m->D_hn, &m->D_he},
                 *jd[2] = {&m->D_jn, &m->D_je};
    int bt[2];
    for (int q = 0; q < 2; q++) {
      bj[q].tm[0] = term(m, jl[q], *jd[q], 0);
      bj[q].nt = 1;
      bj[q].act = L[pl[q]].act;
      bj[q].Y = ya[q]->as<float>();
      bj[q].ldy = L[pl[q]].Np;
      bj[q].dZ = yd[q]->as<float>();
      bj[q].ldo = L[pl[q]].Np;
      bj[q].Kreal = L[pl[q]].N;
      bj[q].tiles_n = L[pl[q]].Np / kTile;
      bt[q] = tiles(pl[q]);
    }
    HGX_TRY(launch_bwd(ctx, bj, bt, 2, c));
  }
  // every weight gradient + Adagrad
  std::vector<WgJob> wj;
  std::vector<int> wt;
  auto add = [&](int li, const Src &x, const DevBuf &dz) {
    wj.push_back(wg_job(m, li, x, dz, L[li].Np));
    wt.push_back(wj.back().gemm_tiles + wj.back().tiles_n);
  };
  add(a, in_n, m->D_hn);
  add(b, in_e, m->D_he);
  add(jn, dense(m->A_hn, L[a].Np, L[a].Np), m->D_jn);
  add(je, dense(m->A_he, L[b].Np, L[b].Np), m->D_je);
  if (ae) {
    add(m->post_n, dense(m->A_j, m->ldJ, NpJ), m->D_pn);
    add(m->post_e, dense(m->A_j, m->ldJ, NpJ, NpJ), m->D_pe);
    add(m->rec_n, dense(m->A_pn, L[m->post_n].Np, L[m->post_n].Np), m->D_rn);
    add(m->rec_e, dense(m->A_pe, L[m->post_e].Np, L[m->post_e].Np), m->D_re);
  }
  add(hd, dense(m->A_j, m->ldJ, 2 * NpJ), m->D_hm);
  add(lb, dense(m->A_hm, L[hd].Np, L[hd].Np), m->D_4);
  if (ctx->tune.mlp_wgrad_split == 1) {
    // the layers after the pre layers first, then the pre layers (same
    // arithmetic per weight; only the launch grouping differs)
    HGX_TRY(launch_wgrad(ctx, wj.data() + 2, wt.data() + 2, (int)wj.size() - 2, c));
    return launch_wgrad(ctx, wj.data(), wt.data(), 2, c);
  }
  return launch_wgrad(ctx, wj.data(), wt.data(), (int)wj.size(), c);
}

int loss_slots(const hgx_mlp *m) {
  int s = 8;
  if (m->kind == HGX_MLP_NE_SEMI_SUPERVISED)
    s += 2 * 8 * (m->L[m->rec_n].Np / kTile);
  return s;
}

double batch_flops(const hgx_mlp *m, int M) {
  double f = 0;
  for (size_t q = 0; q < m->L.size(); q++) {
    const bool first = (int)q == m->pre_n || (int)q == m->pre_e;
    f += layer_flops(m->L[q], M, !first);
  }
  return f;
}

}  // namespace

// ============================ C ABI ========================================
extern "C" {

int hgx_mlp_create(hgx_ctx *ctx, int kind, int in_dim, int out_dim,
                   hgx_mlp **out) {
  if (!ctx || !out) return HGX_EINVAL;
  *out = nullptr;
  HGX_CHECK(ctx, kind >= 0 && kind <= 2, HGX_EINVAL, "unknown MLP kind %d", kind);
  HGX_CHECK(ctx, in_dim > 0, HGX_EINVAL, "input dimension must be positive");
  HGX_CHECK(ctx, kind == HGX_MLP_LP_CLASSIFIER || out_dim > 0, HGX_EINVAL,
            "desired_dim > 0");  // combine_embeddings_util.py:83
  HGX_CHECK(ctx, in_dim <= 16384 && out_dim <= 16384, HGX_EUNSUP,
            "MLP widths above 16384 are not supported");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  hgx_mlp *m = new hgx_mlp();
  m->ctx = ctx;
  m->kind = kind;
  m->in = in_dim;
  m->out = out_dim;
  m->ldt = round_up(in_dim, 4);
  m->twidth = in_dim;
  if (kind == HGX_MLP_LP_CLASSIFIER) {
    // [node | edge] (2 in) -> Dense(in, relu) -> Dense(1, sigmoid)
    m->hid = in_dim;
    m->pre_n = new_layer(m, 2 * in_dim, in_dim, round_up(2 * m->ldt, 64), ACT_RELU,
                         in_dim, m->ldt);
    m->label = new_layer(m, in_dim, 1, round_up(in_dim, 64), ACT_SIGMOID, in_dim, 0);
  } else {
    const int h = (in_dim + out_dim) / 2;  // combine_embeddings_util.py:91
    m->hid = h;
    const int Kin = round_up(m->ldt, 64), Kh = round_up(h, 64), Kd = round_up(out_dim, 64);
    m->pre_n = new_layer(m, in_dim, h, Kin, ACT_RELU, in_dim, 0);
    m->pre_e = new_layer(m, in_dim, h, Kin, ACT_RELU, in_dim, 0);
    m->joint_n = new_layer(m, h, out_dim, Kh, ACT_SIGMOID, h, 0);
    m->joint_e = new_layer(m, h, out_dim, Kh, ACT_SIGMOID, h, 0);
    if (kind == HGX_MLP_NE_SEMI_SUPERVISED) {
      m->post_n = new_layer(m, out_dim, h, Kd, ACT_RELU, out_dim, 0);
      m->post_e = new_layer(m, out_dim, h, Kd, ACT_RELU, out_dim, 0);
      m->rec_n = new_layer(m, h, in_dim, Kh, ACT_RELU, h, 0);
      m->rec_e = new_layer(m, h, in_dim, Kh, ACT_RELU, h, 0);
    }
    // Concatenate([joint_n, joint_e]) -> Dense(d, relu): J_e rows start at Kd
    m->hidden = new_layer(m, 2 * out_dim, out_dim, 2 * Kd, ACT_RELU, out_dim, Kd);
    m->label = new_layer(m, out_dim, 1, Kd, ACT_SIGMOID, out_dim, 0);
    m->ldJ = 2 * Kd;
  }
  int rc = HGX_OK;
  for (auto &l : m->L) {
    const size_t wb = sizeof(float) * (size_t)l.Kp * l.Np, bb = sizeof(float) * l.Np;
    if ((rc = alloc_zero(ctx, l.W, wb)) || (rc = alloc_zero(ctx, l.aW, wb)) ||
        (rc = alloc_zero(ctx, l.b, bb)) || (rc = alloc_zero(ctx, l.ab, bb)))
      break;
  }
  auto act = [&](DevBuf &b, int li) {
    return rc ? rc : (rc = alloc_zero(ctx, b, sizeof(float) * (size_t)kMcap * m->L[li].Np));
  };
  auto del = [&](DevBuf &b, int width) {
    return rc ? rc : (rc = alloc_zero(ctx, b, sizeof(float) * (size_t)256 * width));
  };
  act(m->A_hn, m->pre_n);
  del(m->D_hn, m->L[m->pre_n].Np);
  del(m->D_4, 64);
  if (kind != HGX_MLP_LP_CLASSIFIER) {
    act(m->A_he, m->pre_e);
    if (!rc) rc = alloc_zero(ctx, m->A_j, sizeof(float) * (size_t)kMcap * m->ldJ);
    act(m->A_hm, m->hidden);
    del(m->D_he, m->L[m->pre_e].Np);
    del(m->D_jn, m->L[m->joint_n].Np);
    del(m->D_je, m->L[m->joint_e].Np);
    del(m->D_hm, m->L[m->hidden].Np);
    if (kind == HGX_MLP_NE_SEMI_SUPERVISED) {
      act(m->A_pn, m->post_n);
      act(m->A_pe, m->post_e);
      act(m->A_rn, m->rec_n);
      act(m->A_re, m->rec_e);
      del(m->D_pn, m->L[m->post_n].Np);
      del(m->D_pe, m->L[m->post_e].Np);
      del(m->D_rn, m->L[m->rec_n].Np);
      del(m->D_re, m->L[m->rec_e].Np);
    }
  }
  if (!rc) rc = alloc_zero(ctx, m->A_y, sizeof(float) * kMcap);
  if (!rc && hipEventCreate(&m->e0) != hipSuccess) rc = hgx_fail(ctx, HGX_EHIP, "event");
  if (!rc && hipEventCreate(&m->e1) != hipSuccess) rc = hgx_fail(ctx, HGX_EHIP, "event");
  if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess)
    rc = hgx_fail(ctx, HGX_EHIP, "stream synchronize failed");
  if (rc) {
    hgx_mlp_destroy(m);
    return rc;
  }
  *out = m;
  return HGX_OK;
}

int hgx_mlp_destroy(hgx_mlp *m) {
  if (!m) return HGX_OK;
  if (m->ctx) hipStreamSynchronize(m->ctx->stream);
  for (auto &l : m->L) {
    hgx_release(l.W);
    hgx_release(l.b);
    hgx_release(l.aW);
    hgx_release(l.ab);
  }
  DevBuf *bufs[] = {&m->tn, &m->te, &m->s_node, &m->s_edge, &m->s_label, &m->A_hn,
                    &m->A_he, &m->A_j, &m->A_hm, &m->A_pn, &m->A_pe, &m->A_rn,
                    &m->A_re, &m->A_y, &m->D_hn, &m->D_he, &m->D_jn, &m->D_je,
                    &m->D_hm, &m->D_4, &m->D_pn, &m->D_pe, &m->D_rn, &m->D_re,
                    &m->perm, &m->p_node, &m->p_edge, &m->p_label, &m->keys,
                    &m->part, &m->bloss, &m->sort_tmp, &m->idx_a, &m->idx_b,
                    &m->xpf[0], &m->xpf[1]};
  for (DevBuf *b : bufs) hgx_release(*b);
  if (m->e0) hipEventDestroy(m->e0);
  if (m->e1) hipEventDestroy(m->e1);
  delete m;
  return HGX_OK;
}

int hgx_mlp_layers(const hgx_mlp *m, int *n_layers, int32_t *shapes) {
  if (!m || !n_layers) return HGX_EINVAL;
  *n_layers = (int)m->L.size();
  if (shapes)
    for (size_t q = 0; q < m->L.size(); q++) {
      shapes[2 * q] = m->L[q].Kext;
      shapes[2 * q + 1] = m->L[q].N;
    }
  return HGX_OK;
}

// flat = per layer (creation order): kernel Kext x N row-major, then bias N
static int mlp_weights_io(hgx_mlp *m, float *flat, bool set) {
  hgx_ctx *ctx = m->ctx;
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  int64_t off = 0;
  for (auto &l : m->L) {
    std::vector<float> W((size_t)l.Kp * l.Np, 0.f), b(l.Np, 0.f);
    if (!set) {
      HGX_HIP(ctx, hipMemcpyAsync(W.data(), l.W.p, sizeof(float) * W.size(),
                                  hipMemcpyDeviceToHost, ctx->stream));
      HGX_HIP(ctx, hipMemcpyAsync(b.data(), l.b.p, sizeof(float) * b.size(),
                                  hipMemcpyDeviceToHost, ctx->stream));
      HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    for (int e = 0; e < l.Kext; e++) {
      const int r = e < l.seg ? e : l.off + (e - l.seg);
      for (int n = 0; n < l.N; n++) {
        float &dst = W[(size_t)r * l.Np + n];
        if (set) dst = flat[off + (int64_t)e * l.N + n];
        else flat[off + (int64_t)e * l.N + n] = dst;
      }
    }
    off += (int64_t)l.Kext * l.N;
    for (int n = 0; n < l.N; n++) {
      if (set) b[n] = flat[off + n];
      else flat[off + n] = b[n];
    }
    off += l.N;
    if (set) {
      HGX_HIP(ctx, hipMemcpyAsync(l.W.p, W.data(), sizeof(float) * W.size(),
                                  hipMemcpyHostToDevice, ctx->stream));
      HGX_HIP(ctx, hipMemcpyAsync(l.b.p, b.data(), sizeof(float) * b.size(),
                                  hipMemcpyHostToDevice, ctx->stream));
      // a fresh set of weights starts Adagrad from zero accumulators
      HGX_HIP(ctx, hipMemsetAsync(l.aW.p, 0, l.aW.bytes, ctx->stream));
      HGX_HIP(ctx, hipMemsetAsync(l.ab.p, 0, l.ab.bytes, ctx->stream));
      HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
  }
  return HGX_OK;
}

int hgx_mlp_set_weights(hgx_mlp *m, const float *flat) {
  if (!m || !flat) return HGX_EINVAL;
  return mlp_weights_io(m, const_cast<float *>(flat), true);
}

int hgx_mlp_get_weights(hgx_mlp *m, float *flat) {
  if (!m || !flat) return HGX_EINVAL;
  return mlp_weights_io(m, flat, false);
}

int hgx_mlp_set_tables(hgx_mlp *m, int64_t node_rows, const float *node_tab,
                       int64_t edge_rows, const float *edge_tab) {
  if (!m) return HGX_EINVAL;
  hgx_ctx *ctx = m->ctx;
  HGX_CHECK(ctx, node_rows > 0 && edge_rows > 0 && node_tab && edge_tab,
            HGX_EINVAL, "both embedding tables are required");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const size_t row = sizeof(float) * m->ldt;
  HGX_TRY(alloc_zero(ctx, m->tn, row * node_rows));
  HGX_TRY(alloc_zero(ctx, m->te, row * edge_rows));
  HGX_HIP(ctx, hipMemcpy2DAsync(m->tn.p, row, node_tab, sizeof(float) * m->twidth,
                                sizeof(float) * m->twidth, node_rows,
                                hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpy2DAsync(m->te.p, row, edge_tab, sizeof(float) * m->twidth,
                                sizeof(float) * m->twidth, edge_rows,
                                hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  m->tn_rows = node_rows;
  m->te_rows = edge_rows;
  return HGX_OK;
}

static int check_rows(hgx_mlp *m, int64_t n, const int32_t *nr, const int32_t *er) {
  for (int64_t i = 0; i < n; i++) {
    if (nr && (nr[i] < 0 || nr[i] >= m->tn_rows))
      return hgx_fail(m->ctx, HGX_EINVAL, "node row %d out of range", nr[i]);
    if (er && (er[i] < 0 || er[i] >= m->te_rows))
      return hgx_fail(m->ctx, HGX_EINVAL, "edge row %d out of range", er[i]);
  }
  return HGX_OK;
}

int hgx_mlp_set_samples(hgx_mlp *m, int64_t n, const int32_t *node_row,
                        const int32_t *edge_row, const float *label) {
  if (!m) return HGX_EINVAL;
  hgx_ctx *ctx = m->ctx;
  HGX_CHECK(ctx, m->tn_rows > 0, HGX_ESTATE, "hgx_mlp_set_tables first");
  HGX_CHECK(ctx, n > 0 && n < (int64_t)INT32_MAX && node_row && edge_row && label,
            HGX_EINVAL, "samples: 0 < n < 2^31 with node, edge and label arrays");
  HGX_TRY(check_rows(m, n, node_row, edge_row));
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, m->s_node, sizeof(int) * n));
  HGX_TRY(hgx_ensure(ctx, m->s_edge, sizeof(int) * n));
  HGX_TRY(hgx_ensure(ctx, m->s_label, sizeof(float) * n));
  HGX_HIP(ctx, hipMemcpyAsync(m->s_node.p, node_row, sizeof(int) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(m->s_edge.p, edge_row, sizeof(int) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(m->s_label.p, label, sizeof(float) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  m->ns = n;
  return HGX_OK;
}

int hgx_mlp_fit(hgx_mlp *m, int batch, int max_epochs, float lr, float eps,
                float min_delta, uint64_t seed, const int64_t *perms,
                float *epoch_loss, int *epochs_run) {
  if (!m) return HGX_EINVAL;
  hgx_ctx *ctx = m->ctx;
  HGX_CHECK(ctx, m->ns > 0, HGX_ESTATE, "hgx_mlp_set_samples first");
  HGX_CHECK(ctx, batch >= 1 && batch <= 256, HGX_EUNSUP,
            "batch sizes 1..256 are supported (the reference uses 256)");
  HGX_CHECK(ctx, max_epochs >= 0, HGX_EINVAL, "epochs >= 0");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int64_t n = m->ns;
  const int64_t nb = (n + batch - 1) / batch;
  const int nslot = loss_slots(m);
  constexpr int kLossChunk = 1024;  // batches per loss-partial buffer
  HGX_TRY(hgx_ensure(ctx, m->perm, sizeof(int) * n));
  HGX_TRY(hgx_ensure(ctx, m->p_node, sizeof(int) * n));
  HGX_TRY(hgx_ensure(ctx, m->p_edge, sizeof(int) * n));
  HGX_TRY(hgx_ensure(ctx, m->p_label, sizeof(float) * n));
  HGX_TRY(hgx_ensure(ctx, m->part, sizeof(float) * (size_t)kLossChunk * nslot));
  HGX_TRY(hgx_ensure(ctx, m->bloss, sizeof(double) * nb));
  // combiners: batch bi + 1's input rows are gathered during batch bi
  const bool prefetch = m->kind != HGX_MLP_LP_CLASSIFIER && ctx->tune.mlp_prefetch;
  if (prefetch)
    for (DevBuf &x : m->xpf)
      HGX_TRY(hgx_ensure(ctx, x, sizeof(float) * 2 * kPfRows * (size_t)m->ldt));
  int *perm = m->perm.as<int>();
  unsigned long long *kin = nullptr, *kout = nullptr;
  int *vin = nullptr;
  size_t tmp_bytes = 0;
  if (!perms) {
    HGX_TRY(hgx_ensure(ctx, m->keys, sizeof(unsigned long long) * 2 * n + sizeof(int) * n));
    kin = m->keys.as<unsigned long long>();
    kout = kin + n;
    vin = reinterpret_cast<int *>(kout + n);
    HGX_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin,
                                                    perm, (int)n));
    HGX_TRY(hgx_ensure(ctx, m->sort_tmp, tmp_bytes + 16));
  }
  std::vector<double> bl(nb);
  std::vector<int> hperm;
  // debug: from batch HGX_MLP_GRAD_AT on, weights receive the raw gradient
  const char *ga = hgx_debug_env_str("HGX_MLP_GRAD_AT");
  const int64_t grad_at = ga ? atoll(ga) : -1;
  double best = INFINITY;
  int ran = 0;
  m->ms = 0;
  m->flops = 0;
  m->samples = 0;
  m->batches = 0;
  for (int ep = 0; ep < max_epochs; ep++) {
    if (perms) {
      hperm.resize(n);
      for (int64_t i = 0; i < n; i++) {
        const int64_t v = perms[(int64_t)ep * n + i];
        HGX_CHECK(ctx, v >= 0 && v < n, HGX_EINVAL, "permutation entry out of range");
        hperm[i] = (int)v;
      }
      HGX_HIP(ctx, hipMemcpyAsync(perm, hperm.data(), sizeof(int) * n,
                                  hipMemcpyHostToDevice, ctx->stream));
    } else {
      hipLaunchKernelGGL(mlp_shuffle_keys, dim3(grid_for(n, 256)), dim3(256), 0,
                         ctx->stream, seed, ep, n, kin, vin);
      HGX_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(m->sort_tmp.p, tmp_bytes, kin,
                                                      kout, vin, perm, (int)n, 0, 64,
                                                      ctx->stream));
    }
    hipLaunchKernelGGL(mlp_permute, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream,
                       perm, n, m->s_node.as<int>(), m->s_edge.as<int>(),
                       m->s_label.as<float>(), m->p_node.as<int>(), m->p_edge.as<int>(),
                       m->p_label.as<float>());
    HGX_LAUNCH_CHECK(ctx);
    HGX_HIP(ctx, hipEventRecord(m->e0, ctx->stream));
    const uint32_t dstream = 0x44000000u + 4u * (uint32_t)ep;
    for (int64_t c0 = 0; c0 < nb; c0 += kLossChunk) {
      const int64_t c1 = std::min<int64_t>(nb, c0 + kLossChunk);
      HGX_HIP(ctx, hipMemsetAsync(m->part.p, 0, sizeof(float) * (size_t)kLossChunk * nslot,
                                  ctx->stream));
      for (int64_t bi = c0; bi < c1; bi++) {
        Ctx c;
        c.pbase = bi * batch;
        c.M = (int)std::min<int64_t>(batch, n - c.pbase);
        c.dseed = seed;
        c.lr = lr;
        c.eps = eps;
        c.grad_only = grad_at >= 0 && ep * nb + bi >= grad_at;
        const int64_t nx = (bi + 1) * batch;
        float *xin = prefetch && bi > 0 ? m->xpf[bi & 1].as<float>() : nullptr;
        float *xout = prefetch && bi + 1 < nb ? m->xpf[(bi + 1) & 1].as<float>() : nullptr;
        HGX_TRY(run_batch(m, c, m->p_node.as<int>(), m->p_edge.as<int>(),
                          m->p_label.as<float>(), dstream, true, 0,
                          m->part.as<float>() + (bi - c0) * nslot, nullptr, xin, xout, nx,
                          (int)std::min<int64_t>(batch, n - nx)));
        m->flops += batch_flops(m, c.M);
      }
      hipLaunchKernelGGL(mlp_loss_reduce, dim3((unsigned)((c1 - c0 + 255) / 256)),
                         dim3(256), 0, ctx->stream, m->part.as<float>(), nslot,
                         (int)(c1 - c0), m->bloss.as<double>() + c0);
      HGX_LAUNCH_CHECK(ctx);
    }
    HGX_HIP(ctx, hipEventRecord(m->e1, ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(bl.data(), m->bloss.p, sizeof(double) * nb,
                                hipMemcpyDeviceToHost, ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    float ems = 0;
    HGX_HIP(ctx, hipEventElapsedTime(&ems, m->e0, m->e1));
    m->ms += ems;
    m->samples += n;
    m->batches += nb;
    // Keras' epoch loss: batch losses weighted by batch size
    double tot = 0;
    for (int64_t bi = 0; bi < nb; bi++)
      tot += bl[bi] * (double)std::min<int64_t>(batch, n - bi * batch);
    const double eloss = tot / (double)n;
    if (epoch_loss) epoch_loss[ep] = (float)eloss;
    ran = ep + 1;
    // EarlyStopping(monitor='loss', min_delta, patience=0) (Keras 2.x)
    if (eloss + (double)min_delta < best) {
      best = eloss;
    } else {
      break;
    }
  }
  if (epochs_run) *epochs_run = ran;
#if HGX_MLP_DIAG_TIME
  {
    unsigned long long t[8][12], nn[8];
    hipMemcpyFromSymbol(t, HIP_SYMBOL(g_mlp_t), sizeof(t));
    hipMemcpyFromSymbol(nn, HIP_SYMBOL(g_mlp_n), sizeof(nn));
    const char *nm[8] = {"fwd8 gather", "fwd6", "fwd8 dense", "bwd FH", "bwd", "wgrad", "fwd other", "-"};
    for (int k = 0; k < 7; k++)
      if (nn[k]) {
        fprintf(stderr, "[mlp diag] %-12s wg %10llu  us to:", nm[k], nn[k]);
        for (int q = 1; q < 11; q++)
          if (q < 6 || t[k][q]) fprintf(stderr, " %6.2f", t[k][q] * 0.01 / nn[k]);
        fprintf(stderr, "\n");
      }
  }
#endif
  return HGX_OK;
}

int hgx_mlp_predict(hgx_mlp *m, int output, int64_t n, const int32_t *node_row,
                    const int32_t *edge_row, float *out) {
  if (!m || !out) return HGX_EINVAL;
  hgx_ctx *ctx = m->ctx;
  HGX_CHECK(ctx, m->tn_rows > 0, HGX_ESTATE, "hgx_mlp_set_tables first");
  HGX_CHECK(ctx, output >= 0 && output <= 2, HGX_EINVAL, "output 0 (label), 1, 2");
  HGX_CHECK(ctx, output == 0 || m->kind != HGX_MLP_LP_CLASSIFIER, HGX_EINVAL,
            "the classifier has no joint embedding output");
  HGX_CHECK(ctx, n >= 0, HGX_EINVAL, "n >= 0");
  if (n == 0) return HGX_OK;
  const bool need_n = output != 2, need_e = output != 1;
  HGX_CHECK(ctx, (!need_n || node_row) && (!need_e || edge_row), HGX_EINVAL,
            "row arrays required for this output");
  HGX_TRY(check_rows(m, n, need_n ? node_row : nullptr, need_e ? edge_row : nullptr));
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, m->idx_a, sizeof(int) * n));
  HGX_TRY(hgx_ensure(ctx, m->idx_b, sizeof(int) * n));
  if (need_n)
    HGX_HIP(ctx, hipMemcpyAsync(m->idx_a.p, node_row, sizeof(int) * n,
                                hipMemcpyHostToDevice, ctx->stream));
  else
    HGX_HIP(ctx, hipMemsetAsync(m->idx_a.p, 0, sizeof(int) * n, ctx->stream));
  if (need_e)
    HGX_HIP(ctx, hipMemcpyAsync(m->idx_b.p, edge_row, sizeof(int) * n,
                                hipMemcpyHostToDevice, ctx->stream));
  else
    HGX_HIP(ctx, hipMemsetAsync(m->idx_b.p, 0, sizeof(int) * n, ctx->stream));
  const int d = m->out;
  const int NpJ = m->kind == HGX_MLP_LP_CLASSIFIER ? 0 : m->L[m->joint_n].Np;
  for (int64_t p0 = 0; p0 < n; p0 += kMcap) {
    Ctx c;
    c.pbase = p0;
    c.M = (int)std::min<int64_t>(kMcap, n - p0);
    c.dseed = 0;
    c.lr = 0;
    c.eps = 0;
    c.grad_only = 0;
    HGX_TRY(run_batch(m, c, m->idx_a.as<int>(), m->idx_b.as<int>(), nullptr, 0, false,
                      output, nullptr, output == 0 ? m->A_y.as<float>() : nullptr));
    HGX_LAUNCH_CHECK(ctx);
    if (output == 0) {
      HGX_HIP(ctx, hipMemcpyAsync(out + p0, m->A_y.p, sizeof(float) * c.M,
                                  hipMemcpyDeviceToHost, ctx->stream));
    } else {
      const float *src = m->A_j.as<float>() + (output == 2 ? NpJ : 0);
      HGX_HIP(ctx, hipMemcpy2DAsync(out + p0 * d, sizeof(float) * d, src,
                                    sizeof(float) * m->ldJ, sizeof(float) * d, c.M,
                                    hipMemcpyDeviceToHost, ctx->stream));
    }
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

int hgx_mlp_last_stats(const hgx_mlp *m, double *ms, int64_t *samples,
                       int64_t *batches, double *flops) {
  if (!m) return HGX_EINVAL;
  if (ms) *ms = m->ms;
  if (samples) *samples = m->samples;
  if (batches) *batches = m->batches;
  if (flops) *flops = m->flops;
  return HGX_OK;
}

}  // extern "C"
