// FOBE/HOBE trainer on MI355X: Keras-semantics Adagrad over the record
// stream, one synchronous batch at a time.
//
// Reference: hg2v_model.py:51-125 (BooleanModel: sigmoid heads, KLD),
// 129-203 (UnweightedFloatModel: relu heads, MSE); embedding.py:269-305
// (fit: batch 256, shuffle per epoch, EarlyStopping(loss, min_delta 1e-3,
// patience 0)); KerasModelToEmbedding hg2v_model.py:31-48 (row idx+1).
//   nn = act(N[ln].N[rn]), ee = act(E[le].E[re]),
//   ne = mean_k act(N[nn_k].N[ln]) * mean_k act(E[ne_k].E[re]);
//   loss = sum over heads of the batch mean; Adagrad a += g^2,
//   p -= lr*g/(sqrt(a)+eps) with the gradients of duplicate rows summed
//   (TF densifies the IndexedSlices before the update).
//
// Per batch (strictly sequential, like Keras):
//   K1 train_fwd_bwd  -- one L-lane group per record (L*VPL*4 = padded d):
//      gather the 4+2K rows, 2+2K dots (xor-shuffle reductions), heads,
//      loss, and the per-slot gradient rows -> gslot[B*R][dp]. Gradients of
//      the padding row 0 (touched by almost every record) are pre-summed
//      per workgroup -> gzero[blk][2][dp], so no row sees >~B/RPB addends.
//   K2 train_update   -- one group per unique touched row of the batch:
//      sum its slot rows in sorted slot order (deterministic) and apply
//      Adagrad in place.
// The unique-row lists come from train_prep, run for a whole chunk of
// batches in parallel (one workgroup per batch: block radix sort of the
// batch's (row, slot) keys; an LDS bitonic network for other batch shapes). K1/K2 for a run of batches are captured once
// as direct launches (or hipGraphs of 64 batches, HGX_GRAPH=1), the
// chunk-local batch index passed as a kernel argument (no device counters,
// no dependent index load).
// Preparation runs once per chunk of up to 1024 batches, by default on the
// same stream before the chunk's batches; tuning train_prep_overlap runs
// chunk c + 1's on a second stream while chunk c trains (train_prep_cus:
// disjoint CU masks for the two streams).
#include <hipcub/hipcub.hpp>
#include <rocprim/block/block_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hgx_internal.h"

namespace {

constexpr int kTB = 256;
constexpr int kGraphBatches = 64;  // batches per chunk buffer and per graph

// diagnostic ablation bits (HGX_TRAIN_ABLATE, timing experiments only;
// results are wrong when set): 1 empty K1, 2 empty K2, 4 K1 gathers hit
// row 0, 8 K1 skips gradient stores, 16 K2 skips slot sums, 32 K2 skips
// the table read-modify-write; train_step: 1024 shared-row gradients by
// plain stores, 2048 no row-0 partial loads, 4096 no forward reductions,
// 8192 no Adagrad arithmetic, 16384 no end-of-batch barrier / partial
// stores, 32768 no neighbour-list gathers (timing ablations: wrong sums).
#ifdef HGX_DEBUG_KNOBS
__constant__ int g_tab = 0;  // ablation bits (diagnostic builds only)
#else
static constexpr int g_tab = 0;
#endif

// diagnostic phase trace (HGX_TRAIN_TRACE=<file>, timing experiments only):
// wave 0 of every workgroup stamps s_memrealtime (100 MHz) at phase ends
// for the first g_trace_nb batches; slots [batch][kernel][block < 1024][8].
// Diagnostic builds only: in a release build the trace pointer is a
// compile-time null, so the step's prologue has no dependent scalar load of a
// device global (GOT entry, then the value) ahead of its kernel-argument
// loads.
#ifdef HGX_DEBUG_KNOBS
__constant__ unsigned long long *g_trace = nullptr;
__constant__ int g_trace_nb = 0;
#else
static constexpr unsigned long long *g_trace = nullptr;
static constexpr int g_trace_nb = 0;
#endif
#define HGX_STAMP(var)                                              \
  do {                                                              \
    if (g_trace) {                                                  \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   \
      var = __builtin_amdgcn_s_memrealtime();                       \
    }                                                               \
  } while (0)
__device__ __forceinline__ void trace_put(int gb, int kern, int nst,
                                          const unsigned long long *t) {
  if (g_trace && threadIdx.x == 0 && gb < g_trace_nb && blockIdx.x < 1024) {
    unsigned long long *q = g_trace + (((size_t)gb * 2 + kern) * 1024 + blockIdx.x) * 8;
    for (int i = 0; i < nst; i++) q[i] = t[i];
  }
}

struct TrainArgs {
  const int *idx;
  const float *tgt;
  const int *perm;
  int64_t n;
  int B, R, K, dp;
  float *ntab, *etab, *nacc, *eacc;
  float *gslot, *gzero, *lossbuf;
  // chunk buffers written by train_prep: batch-ordered records, each
  // slot's position in its batch's sorted (row, slot) order, unique keys
  int *bidx;
  float *btgt;
  int *inv, *ukey, *uoff, *ucount;
  int2 *bmeta;  // per chunk-local batch: {records (0 = no batch), global batch}
  int SB, nblk1;
  int lstride;  // per-batch stride of lossbuf (>= the blocks of either path)
  float lr, eps;
  int loss, act;
  // deferred-row step (train_step, train_place): per chunk-local batch
  // ceil(B / prpb) workgroups x prpb groups of RW words (R slot ids / codes
  // + kFX flush slots) and 3 targets; per-slot codes and the deferred rows'
  // keys from train_prep; deferred entries per batch (pM), flush overflow
  // list (pfo). gacc [3][MX][dp] fixed-point sums and shadow [3][MX][2][dp]
  // base rows of deferred entries by batch parity (entries 0 / 1: row 0 of
  // the node / edge table, shadow only); r0acc the padding row's gradient
  // sums, kR0Slots fixed-point accumulators per batch parity; ovf the
  // fixed-point range flag.
  int fused, prpb, RW, MX, Mmax;
  int *pidx, *pbrk;
  unsigned *pcode, *scode;
  float *ptgt;
  int2 *pfo;
  long long *gacc;
  float *shadow;
  long long *r0acc;  // [3][kR0Slots][2][dp] fixed point, see Row0Loads
  int *ovf;
};

// slot codes of the deferred-row step (train_prep / train_place -> train_step)
constexpr unsigned kSShared = 0x80000000u;  // row in several records: deferred entry m
constexpr unsigned kSOwn = 0x40000000u;     // this slot writes the row (or its shadow)
constexpr unsigned kSPend = 0x20000000u;    // row deferred by the previous batch: entry m'
constexpr unsigned kSLocal = 0x10000000u;   // row in several slots of ONE record
constexpr unsigned kSFirst = 0x08000000u;   // local: first slot in emit order (no read)
                                            // local: bits 0..3 the owner slot
constexpr unsigned kFEdge = 0x10000000u;    // flush slot words: edge table
constexpr int kDefBits = 14;                // m / slot mask in bits 0..13, m' in 14..25
constexpr unsigned kDefMask = 0xfffu;
constexpr unsigned kSlotMask = 0x3fffu;
constexpr int kFX = 4;                      // flush slots per record group
constexpr int kWX = kFX + 2;                // + batch words: overflow flushes,
                                            //   gacc entries to zero
constexpr int kPackB = 512;                 // max records per step batch
constexpr int kPrepB = 1366;  // max records per prepared batch: 8192 slots / R >= 6
constexpr int kSortP = 4096;  // prepared-batch slot count sorted by block radix sort

__device__ __forceinline__ bool slot_is_edge(int s, int K) {
  return s == 1 || s == 3 || s >= 4 + K;
}

__device__ __forceinline__ float act_f(int act, float z) {
  return act == 0 ? 1.0f / (1.0f + expf(-z)) : (z > 0.f ? z : 0.f);
}
__device__ __forceinline__ float act_d(int act, float z, float y) {
  return act == 0 ? y * (1.0f - y) : (z > 0.f ? 1.f : 0.f);
}
// per-sample loss value and dL/dyhat (before the 1/batch factor)
__device__ __forceinline__ void head_loss(int loss, float y, float yt,
                                          float &lv, float &g) {
  const float eps = 1e-7f;
  if (loss == 0) {  // KLD with Keras clipping
    const float ytc = fminf(fmaxf(yt, eps), 1.f);
    const float ypc = fminf(fmaxf(y, eps), 1.f);
    lv = ytc * logf(ytc / ypc);
    g = (y >= eps && y <= 1.f) ? -ytc / ypc : 0.f;
  } else {  // MSE
    const float df = y - yt;
    lv = df * df;
    g = 2.f * df;
  }
}

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 operator+(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 fma4(float s, float4 v, float4 a) {
  return make_float4(fmaf(s, v.x, a.x), fmaf(s, v.y, a.y), fmaf(s, v.z, a.z),
                     fmaf(s, v.w, a.w));
}
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}

template <int L>
__device__ __forceinline__ float group_sum(float v) {
  return hgx::group_allreduce_sum<L>(v);
}

template <int L, int VPL>
__device__ __forceinline__ void load_row(const float *tab, int row, int dp,
                                         int lane, float4 (&out)[VPL]) {
  const float4 *p = reinterpret_cast<const float4 *>(tab + (size_t)row * dp);
#pragma unroll
  for (int v = 0; v < VPL; v++) out[v] = p[v * L + lane];
}

// MODE: 0 = activation and loss read from the arguments; 1 = FOBE (sigmoid,
// KLD); 2 = HOBE (relu, MSE). KEXACT: K == KMAX at compile time. The
// specialised forms drop the per-record branches, exp and log of the other
// head types: each wave runs its record chain alone on its SIMD, so its
// instruction count is its latency.
template <int L, int VPL, int KMAX, bool KEXACT, int MODE, int TB>
__global__ __launch_bounds__(TB) void train_fwd_bwd(TrainArgs a, int cb) {
  constexpr int RPB = TB / L;
  __shared__ float4 s_z[2][RPB][L * VPL];
  __shared__ float s_loss[RPB];
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g_trace) ts[0] = __builtin_amdgcn_s_memrealtime();
  const int grp = threadIdx.x / L, lane = threadIdx.x % L;
  const int rib = blockIdx.x * RPB + grp;
  const int K = KEXACT ? KMAX : a.K, R = KEXACT ? 4 + 2 * KMAX : a.R;
  const int dp = a.dp;
  // everything below depends only on (cb, rib): the batch metadata and the
  // record's ids / slot positions load together (buffers are padded)
  const int2 bm = a.bmeta[cb];
  const int *ri = a.bidx + ((size_t)cb * a.B + rib) * R;
  const float *yt = a.btgt + ((size_t)cb * a.B + rib) * 3;
  const int *pos = a.inv + (size_t)cb * a.SB + (size_t)rib * R;
  int ln = ri[0], le = ri[1], rn = ri[2], re = ri[3];
  int nnk[KMAX], nek[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; k++) {
    nnk[k] = k < K ? ri[4 + k] : 0;
    nek[k] = k < K ? ri[4 + K + k] : 0;
  }
  const int nb = bm.x;
  HGX_STAMP(ts[1]);
  if (nb == 0 || (g_tab & 1)) return;
  const float inv_b = 1.0f / (float)nb;
  float4 zN[VPL], zE[VPL];
#pragma unroll
  for (int v = 0; v < VPL; v++) zN[v] = zE[v] = f4(0.f);
  float lrec = 0.f;
  if (rib < nb) {
    if (g_tab & 4) {
      ln = le = rn = re = 0;
#pragma unroll
      for (int k = 0; k < KMAX; k++) nnk[k] = nek[k] = 0;
    }
    float4 Nl[VPL], Nr[VPL], El[VPL], Er[VPL], Nk[KMAX][VPL], Ek[KMAX][VPL];
    load_row<L, VPL>(a.ntab, ln, dp, lane, Nl);
    load_row<L, VPL>(a.ntab, rn, dp, lane, Nr);
    load_row<L, VPL>(a.etab, le, dp, lane, El);
    load_row<L, VPL>(a.etab, re, dp, lane, Er);
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      if (k < K) {
        load_row<L, VPL>(a.ntab, nnk[k], dp, lane, Nk[k]);
        load_row<L, VPL>(a.etab, nek[k], dp, lane, Ek[k]);
      }
    }
    HGX_STAMP(ts[2]);
    float z1 = 0.f, z2 = 0.f, za[KMAX], zb[KMAX];
#pragma unroll
    for (int v = 0; v < VPL; v++) {
      z1 += dot4(Nl[v], Nr[v]);
      z2 += dot4(El[v], Er[v]);
    }
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      za[k] = zb[k] = 0.f;
      if (k < K) {
#pragma unroll
        for (int v = 0; v < VPL; v++) {
          za[k] += dot4(Nk[k][v], Nl[v]);
          zb[k] += dot4(Ek[k][v], Er[v]);
        }
      }
    }
    z1 = group_sum<L>(z1);
    z2 = group_sum<L>(z2);
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      if (k < K) {
        za[k] = group_sum<L>(za[k]);
        zb[k] = group_sum<L>(zb[k]);
      }
    }
    const int act = MODE == 1 ? 0 : MODE == 2 ? 1 : a.act;
    const int lossk = MODE == 1 ? 0 : MODE == 2 ? 1 : a.loss;
    const float y1 = act_f(act, z1), y2 = act_f(act, z2);
    float sa[KMAX], sb[KMAX], P = 0.f, Q = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      if (k < K) {
        sa[k] = act_f(act, za[k]);
        sb[k] = act_f(act, zb[k]);
        P += sa[k];
        Q += sb[k];
      }
    }
    P = P / (float)K;
    Q = Q / (float)K;
    const float y3 = P * Q;
    float l1, l2, l3, g1, g2, g3;
    head_loss(lossk, y1, yt[0], l1, g1);
    head_loss(lossk, y2, yt[1], l2, g2);
    head_loss(lossk, y3, yt[2], l3, g3);
    lrec = l1 + l2 + l3;
    HGX_STAMP(ts[3]);
    g1 *= inv_b;
    g2 *= inv_b;
    g3 *= inv_b;
    const float dz1 = g1 * act_d(act, z1, y1);
    const float dz2 = g2 * act_d(act, z2, y2);
    const float dP = g3 * Q / (float)K, dQ = g3 * P / (float)K;
    auto emit = [&](int s, int row, bool edge, const float4(&g)[VPL]) {
      if (row == 0) {
#pragma unroll
        for (int v = 0; v < VPL; v++) {
          if (edge) zE[v] = zE[v] + g[v];
          else zN[v] = zN[v] + g[v];
        }
      } else if (!(g_tab & 8)) {
        float4 *p = reinterpret_cast<float4 *>(a.gslot + (size_t)pos[s] * dp);
#pragma unroll
        for (int v = 0; v < VPL; v++) p[v * L + lane] = g[v];
      }
    };
    float4 gln[VPL], gre[VPL], tmp[VPL];
#pragma unroll
    for (int v = 0; v < VPL; v++) {
      gln[v] = fma4(dz1, Nr[v], f4(0.f));
      gre[v] = fma4(dz2, El[v], f4(0.f));
    }
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      if (k < K) {
        const float da = dP * act_d(act, za[k], sa[k]);
        const float db = dQ * act_d(act, zb[k], sb[k]);
#pragma unroll
        for (int v = 0; v < VPL; v++) {
          gln[v] = fma4(da, Nk[k][v], gln[v]);
          gre[v] = fma4(db, Ek[k][v], gre[v]);
          tmp[v] = fma4(da, Nl[v], f4(0.f));
        }
        emit(4 + k, nnk[k], false, tmp);
#pragma unroll
        for (int v = 0; v < VPL; v++) tmp[v] = fma4(db, Er[v], f4(0.f));
        emit(4 + K + k, nek[k], true, tmp);
      }
    }
    emit(0, ln, false, gln);
    emit(3, re, true, gre);
#pragma unroll
    for (int v = 0; v < VPL; v++) tmp[v] = fma4(dz1, Nl[v], f4(0.f));
    emit(2, rn, false, tmp);
#pragma unroll
    for (int v = 0; v < VPL; v++) tmp[v] = fma4(dz2, Er[v], f4(0.f));
    emit(1, le, true, tmp);
    HGX_STAMP(ts[4]);
  }
  // padding-row partials and loss: reduce over the record groups
#pragma unroll
  for (int v = 0; v < VPL; v++) {
    s_z[0][grp][v * L + lane] = zN[v];
    s_z[1][grp][v * L + lane] = zE[v];
  }
  if (lane == 0) s_loss[grp] = lrec;
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * L * VPL; t += TB) {
    const int tab = t / (L * VPL), j = t % (L * VPL);
    float4 s = f4(0.f);
    for (int g = 0; g < RPB; g++) s = s + s_z[tab][g][j];
    reinterpret_cast<float4 *>(a.gzero + ((size_t)blockIdx.x * 2 + tab) * dp)[j] = s;
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int g = 0; g < RPB; g++) s += s_loss[g];
    a.lossbuf[(size_t)bm.y * a.lstride + blockIdx.x] = s;
  }
  HGX_STAMP(ts[5]);
  trace_put(bm.y, 0, 6, ts);
}

// Adagrad on one float4 of a row (Keras 2.x formulas, round-to-nearest ops
// so the device matches the oracle's rounding)
__device__ __forceinline__ void adagrad4(float4 &p, float4 &ac, float4 g,
                                         float lr, float eps) {
  float *pp = &p.x, *aa = &ac.x;
  const float *gv = &g.x;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const float na = __fadd_rn(aa[c], __fmul_rn(gv[c], gv[c]));
    aa[c] = na;
    pp[c] = __fsub_rn(pp[c], __fdiv_rn(__fmul_rn(lr, gv[c]),
                                       __fadd_rn(sqrtf(na), eps)));
  }
}

// The same update with the hardware square root and reciprocal (<= 1 ulp
// each; the fused step runs every row update of a record on one wave, where
// the correctly rounded sequences cost ~30 instructions per element).
__device__ __forceinline__ void adagrad4_hw(float4 &p, float4 &ac, float4 g,
                                            float lr, float eps) {
  float *pp = &p.x, *aa = &ac.x;
  const float *gv = &g.x;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const float na = __fadd_rn(aa[c], __fmul_rn(gv[c], gv[c]));
    aa[c] = na;
    const float den = __fadd_rn(__builtin_amdgcn_sqrtf(na), eps);
    pp[c] = __fsub_rn(pp[c], __fmul_rn(__fmul_rn(lr, gv[c]), __builtin_amdgcn_rcpf(den)));
  }
}

// K2. Workgroups [0, gridDim-2): one L-lane group per unique touched row.
// The last two workgroups: the padding row 0 of the node / edge table, its
// gradient = the sum of the nblk1 per-K1-workgroup partials, loaded by all
// 256 threads at once and tree-summed in LDS (fixed order: deterministic).
template <int L, int VPL, int TB>
__global__ __launch_bounds__(TB) void train_update(TrainArgs a, int cb) {
  constexpr int GPB = TB / L;
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g_trace) ts[0] = __builtin_amdgcn_s_memrealtime();
  const int dp = a.dp, SB = a.SB;
  const int2 bm = a.bmeta[cb];
  if (blockIdx.x >= gridDim.x - 2) {
    __shared__ float4 s_part[TB];
    const int table = blockIdx.x - (gridDim.x - 2);
    const int NC = dp / 4;                  // float4 columns, <= 256
    const int TPC = TB / NC;               // threads per column (>= 1)
    const int col = threadIdx.x % NC, sub = threadIdx.x / NC;
    float4 *P = reinterpret_cast<float4 *>(table ? a.etab : a.ntab);
    float4 *A = reinterpret_cast<float4 *>(table ? a.eacc : a.nacc);
    const bool own = sub == 0;
    float4 pv = f4(0.f), av = f4(0.f);
    if (own && threadIdx.x < NC * TPC) {
      pv = P[col];
      av = A[col];
    }
    HGX_STAMP(ts[1]);
    if (bm.x == 0 || (g_tab & 2)) return;
    float4 g = f4(0.f);
    if (sub < TPC && !(g_tab & 16)) {
      const float4 *base = reinterpret_cast<const float4 *>(a.gzero) +
                           (size_t)table * NC + col;
      const size_t bstride = (size_t)2 * NC;
      for (int b = sub; b < a.nblk1; b += TPC) g = g + base[b * bstride];
    }
    s_part[threadIdx.x] = g;
    __syncthreads();
    for (int w = TPC / 2; w > 0; w >>= 1) {  // TPC is a power of two
      if (sub < w) s_part[threadIdx.x] = s_part[threadIdx.x] + s_part[threadIdx.x + w * NC];
      __syncthreads();
    }
    HGX_STAMP(ts[2]);
    if (own && !(g_tab & 32)) {
      adagrad4(pv, av, s_part[col], a.lr, a.eps);
      P[col] = pv;
      A[col] = av;
    }
    HGX_STAMP(ts[3]);
    trace_put(bm.y, 1, 4, ts);
    return;
  }
  const int grp = threadIdx.x / L, lane = threadIdx.x % L;
  const int it = blockIdx.x * GPB + grp;
  // the task's key and slot range load beside the batch metadata
  const int *ukey = a.ukey + (size_t)cb * SB;
  const int *uoff = a.uoff + (size_t)cb * (SB + 1);
  const int itc = min(it, SB - 1);
  const int key = ukey[itc], j0 = uoff[itc], j1 = uoff[min(it + 1, SB)];
  const int U = a.ucount[cb];
  HGX_STAMP(ts[1]);
  if (bm.x == 0 || (g_tab & 2) || it >= U) {
    ts[2] = ts[3] = ts[1];
    trace_put(bm.y, 1, 4, ts);
    return;
  }
  const int table = key >> 30, row = key & 0x3fffffff;
  float4 *P = reinterpret_cast<float4 *>((table ? a.etab : a.ntab) + (size_t)row * dp);
  float4 *A = reinterpret_cast<float4 *>((table ? a.eacc : a.nacc) + (size_t)row * dp);
  // table row and accumulator first: their latency hides under the sums
  float4 pv[VPL], av[VPL];
  if (!(g_tab & 32)) {
#pragma unroll
    for (int v = 0; v < VPL; v++) {
      pv[v] = P[v * L + lane];
      av[v] = A[v * L + lane];
    }
  }
  float4 g[VPL];
#pragma unroll
  for (int v = 0; v < VPL; v++) g[v] = f4(0.f);
  if (!(g_tab & 16)) {
    // this row's slot gradients are contiguous (prep sorted them)
    for (int j = j0; j < j1; j++) {
      const float4 *p = reinterpret_cast<const float4 *>(a.gslot + (size_t)j * dp);
#pragma unroll
      for (int v = 0; v < VPL; v++) g[v] = g[v] + p[v * L + lane];
    }
  }
  HGX_STAMP(ts[2]);
  if (g_tab & 32) return;
#pragma unroll
  for (int v = 0; v < VPL; v++) {
    adagrad4(pv[v], av[v], g[v], a.lr, a.eps);
    P[v * L + lane] = pv[v];
    A[v * L + lane] = av[v];
  }
  HGX_STAMP(ts[3]);
  trace_put(bm.y, 1, 4, ts);
}

// Padding-row (row 0) state for the fused path, computed by every workgroup
// of a batch (identical inputs and order, so identical values): mode 0 ->
// the tables hold it; mode 1 -> it is pending from the previous fused batch:
// (p, acc) = Adagrad(r0src, sum of that batch's np per-workgroup partials).
// row0_issue starts every load unconditionally (a load under a branch is
// waited for at the join), first thing in the kernel; row0_finish sums in a
// fixed order (thread `sub` of a column: partials sub, sub+TPC, ...; then
// the TPC sums in order) and returns the column's (p, acc) on sub == 0.
// col < 2L covers both tables (table = col / L, float4 column col % L).
// Block-wide exclusive scan of one int per thread.
__device__ int block_exclusive_scan(int v, int *total, int *s_ws) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(inc, off);
    if (lane >= off) inc += o;
  }
  if (lane == 63) s_ws[wave] = inc;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < kTB / 64; w++) {
    if (w < wave) base += s_ws[w];
    tot += s_ws[w];
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// ---------------------------------------------------------------------------
// Deferred-row batch step (train_step): one launch per batch, no packing
// constraint on which workgroup holds which record.
//
// Keras applies one Adagrad update per batch with the gradients of a row's
// slots summed (hg2v_model.py:51-203 through TF's dense IndexedSlices sum).
//  - A row with ONE slot in batch b (most rows) is updated in place by the
//    lane group of its record, right after the backward pass.
//  - A row with several slots in b ("deferred" row, entry m of b) cannot be
//    summed in one place without a grid-wide barrier. Each slot adds its
//    gradient to gacc[b % 3][m] as 2^44 fixed point with integer atomics:
//    the sum is exact and independent of arrival order, so the step stays
//    bitwise reproducible. The row's owner slot writes the row's state as b
//    read it, (p, a), to shadow[b % 3][m]. The update itself is applied by
//    launch b + 1: every slot of b + 1 that touches the row ("pending" slot,
//    code kSPend, entry m') reads shadow + gacc and folds the Adagrad step
//    of b in registers (all readers compute the same bits); a deferred row of
//    b that b + 1 does not touch is written back by a "flush slot" of b + 1.
//  - The padding row 0 of both tables (nearly every record) goes the same
//    way without atomics: each workgroup stores its fixed-order LDS partial
//    (plain stores: an atomic add's completion at the kernel tail measured
//    0.7 us), every workgroup of b + 1 sums the partials in a fixed order and
//    folds the step; workgroup 0 keeps the base in shadow entry 0 / 1.
// Nothing of batch b + 1 reads a location batch b + 1 writes: the table rows
// it writes are single-slot rows of b + 1 (read only by their own group) or
// flushed rows (not read by b + 1); shadow and gacc are triple-buffered by
// batch parity, gp double-buffered. train_flush applies the last batch's
// deferred rows at the end of every epoch. A parity's gacc entries are zeroed
// two launches after their use (the count rides in the record words).
// ---------------------------------------------------------------------------

// fixed point of the deferred-row gradient sums: 2^44 units, |one added
// value| < kFixLimit; at most 2^13 adds per entry and batch keep the sum
// below 2^63. A value outside the range (a diverged run, or NaN) raises the
// step's overflow flag and hgx_train fails with HGX_ENUMERIC.
constexpr double kFixScale = 17592186044416.0;  // 2^44
constexpr double kFixInv = 1.0 / 17592186044416.0;
constexpr float kFixLimit = 32.f;

// rounded to the nearest 2^-44 unit (not truncated toward zero)
__device__ __forceinline__ unsigned long long to_fix(float v) {
  return (unsigned long long)__double2ll_rn((double)v * kFixScale);
}
__device__ __forceinline__ float from_fix(long long v) {
  return (float)((double)v * kFixInv);
}
// The step's per-lane vector: VW floats of a row (float4: dp = 4L, float2:
// dp = 2L), the fixed-point view of this lane's part of a gacc entry, and the
// ops on them
template <int VW>
struct SV;
template <>
struct SV<4> {
  using T = float4;
  struct Fx {
    longlong2 a, b;
  };
  static __device__ __forceinline__ T zero() { return f4(0.f); }
  static __device__ __forceinline__ T add(T x, T y) { return x + y; }
  static __device__ __forceinline__ T mul(T x, float m) {
    return make_float4(x.x * m, x.y * m, x.z * m, x.w * m);
  }
  static __device__ __forceinline__ T fma(float s, T v, T c) { return fma4(s, v, c); }
  static __device__ __forceinline__ float dot(T x, T y) { return dot4(x, y); }
  static __device__ __forceinline__ void adagrad(T &p, T &ac, T g, float lr, float eps) {
    adagrad4_hw(p, ac, g, lr, eps);
  }
  static __device__ __forceinline__ void pin(T &v) {
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
  }
  static __device__ __forceinline__ Fx ldfix(const long long *e, int lane) {
    const longlong2 *g = reinterpret_cast<const longlong2 *>(e) + 2 * lane;
    return {g[0], g[1]};
  }
  static __device__ __forceinline__ T unfix(const Fx &g) {
    return make_float4(from_fix(g.a.x), from_fix(g.a.y), from_fix(g.b.x), from_fix(g.b.y));
  }
  static __device__ __forceinline__ void addfix(long long *e, int lane, T v, int &bad) {
    bad |= !(fabsf(v.x) < kFixLimit) | !(fabsf(v.y) < kFixLimit) |
           !(fabsf(v.z) < kFixLimit) | !(fabsf(v.w) < kFixLimit);
    unsigned long long *d = reinterpret_cast<unsigned long long *>(e) + 4 * lane;
    atomicAdd(d + 0, to_fix(v.x));
    atomicAdd(d + 1, to_fix(v.y));
    atomicAdd(d + 2, to_fix(v.z));
    atomicAdd(d + 3, to_fix(v.w));
  }
  static __device__ __forceinline__ void zerofix(long long *e, int lane) {
    longlong2 *g = reinterpret_cast<longlong2 *>(e) + 2 * lane;
    g[0] = g[1] = make_longlong2(0, 0);
  }
  static __device__ __forceinline__ Fx fxadd(const Fx &x, const Fx &y) {
    return {make_longlong2(x.a.x + y.a.x, x.a.y + y.a.y),
            make_longlong2(x.b.x + y.b.x, x.b.y + y.b.y)};
  }
  static __device__ __forceinline__ Fx fxzero() {
    return {make_longlong2(0, 0), make_longlong2(0, 0)};
  }
};
template <>
struct SV<2> {
  using T = float2;
  struct Fx {
    longlong2 a;
  };
  static __device__ __forceinline__ T zero() { return make_float2(0.f, 0.f); }
  static __device__ __forceinline__ T add(T x, T y) { return make_float2(x.x + y.x, x.y + y.y); }
  static __device__ __forceinline__ T mul(T x, float m) { return make_float2(x.x * m, x.y * m); }
  static __device__ __forceinline__ T fma(float s, T v, T c) {
    return make_float2(fmaf(s, v.x, c.x), fmaf(s, v.y, c.y));
  }
  static __device__ __forceinline__ float dot(T x, T y) { return x.x * y.x + x.y * y.y; }
  static __device__ __forceinline__ void adagrad(T &p, T &ac, T g, float lr, float eps) {
    const float *gv = &g.x;
    float *pp = &p.x, *aa = &ac.x;
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const float na = __fadd_rn(aa[c], __fmul_rn(gv[c], gv[c]));
      aa[c] = na;
      const float den = __fadd_rn(__builtin_amdgcn_sqrtf(na), eps);
      pp[c] = __fsub_rn(pp[c], __fmul_rn(__fmul_rn(lr, gv[c]), __builtin_amdgcn_rcpf(den)));
    }
  }
  static __device__ __forceinline__ void pin(T &v) { asm volatile("" : "+v"(v.x), "+v"(v.y)); }
  static __device__ __forceinline__ Fx ldfix(const long long *e, int lane) {
    return {reinterpret_cast<const longlong2 *>(e)[lane]};
  }
  static __device__ __forceinline__ T unfix(const Fx &g) {
    return make_float2(from_fix(g.a.x), from_fix(g.a.y));
  }
  static __device__ __forceinline__ void addfix(long long *e, int lane, T v, int &bad) {
    bad |= !(fabsf(v.x) < kFixLimit) | !(fabsf(v.y) < kFixLimit);
    unsigned long long *d = reinterpret_cast<unsigned long long *>(e) + 2 * lane;
    atomicAdd(d + 0, to_fix(v.x));
    atomicAdd(d + 1, to_fix(v.y));
  }
  static __device__ __forceinline__ void zerofix(long long *e, int lane) {
    reinterpret_cast<longlong2 *>(e)[lane] = make_longlong2(0, 0);
  }
  static __device__ __forceinline__ Fx fxadd(const Fx &x, const Fx &y) {
    return {make_longlong2(x.a.x + y.a.x, x.a.y + y.a.y)};
  }
  static __device__ __forceinline__ Fx fxzero() { return {make_longlong2(0, 0)}; }
};
// the deferred Adagrad step of the previous batch: (p, a) += sum
template <int VW>
__device__ __forceinline__ void fold(typename SV<VW>::T &p, typename SV<VW>::T &ac,
                                     const typename SV<VW>::Fx &g, float lr, float eps) {
  SV<VW>::adagrad(p, ac, SV<VW>::unfix(g), lr, eps);
}

// views of the deferred-row buffers (L lanes x VW floats per row: dp = VW L)
template <int L, int VW>
__device__ __forceinline__ typename SV<VW>::T *sh_row(const TrainArgs &a, int par, int m,
                                                      int which) {
  return reinterpret_cast<typename SV<VW>::T *>(a.shadow) +
         (((size_t)par * a.MX + m) * 2 + which) * L;
}
// the dp int64 of gacc entry m
template <int L, int VW>
__device__ __forceinline__ long long *gacc_row(const TrainArgs &a, int par, int m) {
  return a.gacc + ((size_t)par * a.MX + m) * (VW * L);
}
template <int L, int VW>
__device__ __forceinline__ typename SV<VW>::T *tab_row(const TrainArgs &a, bool edge, int acc,
                                                       int row) {
  float *t = acc ? (edge ? a.eacc : a.nacc) : (edge ? a.etab : a.ntab);
  return reinterpret_cast<typename SV<VW>::T *>(t) + (size_t)row * L;
}

// The step's row stores are write-through (`global_store … sc1`), so the
// ~57 KB a workgroup writes per batch leaves no dirty lines in its XCD's L2
// for the kernel-end release to write back. Interleaved A/B against plain
// stores (profiles/r03/trainer/ab_wt_*.log): d = 128 (float2 rows) 6.88 ->
// 6.68 us per batch, d = 256 (float4 rows) 8.70 -> 8.49.
// float2: an agent-scope relaxed atomic store, which is exactly that store.
__device__ __forceinline__ void st_row(float2 *p, float2 v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p),
                     __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// float4: there is no 16-byte atomic store, so the instruction is written
// out. s_nop 1: the wait states a >8-byte store's data registers need
// before a VALU may overwrite them (the compiler's hazard check does not see
// into asm; without it d = 256 training diverged). The "memory" clobber keeps
// the compiler's memory operations in program order around it; its vmcnt
// waits only get stricter for an extra store in flight (loads still return
// in order). HGX_TRAIN_WT4=0 (A/B builds): a plain store.
// r04: the compiler-visible form -- a raw buffer store with the sc1 policy
// bit, its base the first lane's row address (two readfirstlanes) -- is
// correct but measured 8.62 -> 8.93 us per batch at d = 256 (interleaved
// A/B, C3 HOBE records, profiles/r04/trainer/ab_wt4_builtin.log), so the
// asm stays. Every d = 256 trainer test checks the stored rows against the
// oracle (test_gpu_train.py, the C4 window in test_gpu_c4.py): a toolchain
// that broke the hazard would fail them.
#ifndef HGX_TRAIN_WT4
#define HGX_TRAIN_WT4 1
#endif
__device__ __forceinline__ void st_row(float4 *p, float4 v) {
  if (HGX_TRAIN_WT4) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(x) : "memory");
  } else {
    *p = v;
  }
}

// one flush entry: the deferred row (table bit 30 | row) of entry m of the
// previous batch folded and written back
template <int L, int VW>
__device__ __forceinline__ void flush_row(const TrainArgs &a, int par, int key, int m,
                                          int lane) {
  const bool edge = key >> 30;
  const int row = key & 0x3fffffff;
  typename SV<VW>::T p = sh_row<L, VW>(a, par, m, 0)[lane], ac = sh_row<L, VW>(a, par, m, 1)[lane];
  fold<VW>(p, ac, SV<VW>::ldfix(gacc_row<L, VW>(a, par, m), lane), a.lr, a.eps);
  st_row(&tab_row<L, VW>(a, edge, 0, row)[lane], p);
  st_row(&tab_row<L, VW>(a, edge, 1, row)[lane], ac);
}

// The padding row (row 0 of both tables) of the previous batch. Its
// gradient sum arrives in kR0Slots fixed-point accumulators r0acc[q % 3]:
// every workgroup of batch q adds its records' row-0 gradients (a
// fixed-order float sum over its records, then one 2^44 fixed-point
// integer atomic per element) to slot blockIdx % kR0Slots, so the sum is
// exact and independent of arrival order. Batch q + 1 reads the kR0Slots
// slots (the owner thread of each column: kR0Slots x VW int64), adds them
// as integers and applies the Adagrad step to the base (the previous
// batch's shadow, or the table for the first batch of an epoch); batch q
// zeroes set (q + 1) % 3 for the next batch. r02/r03a instead had every
// workgroup store a float partial and every workgroup of the next batch
// read all 64 of them: 64 KB per workgroup from the Infinity Cache, about
// 0.9 us per batch at its per-CU rate (tools/ablate_train.py); now 16 KB.
// Slots per row width (interleaved A/B, profiles/r03/trainer/ab_slots_*.txt):
// 128-float rows (each record adds its own sums, 256 adders per batch) 8
// slots: 6.68 us per batch vs 7.77 at 4 and 6.81 at 16; 256-float rows (one
// add per workgroup, 64 adders) 4 slots: 8.36 vs 8.50 at 8 and 9.12 at 16.
constexpr int kR0Slots = 8;  // the most any width uses (buffer sizing)
template <int DP>
struct R0S {
  static constexpr int n = DP >= 256 ? 4 : kR0Slots;
};
template <int L, int VW>
__device__ __forceinline__ long long *r0_row(const TrainArgs &a, int par, int slot,
                                             int tab) {
  return a.r0acc + (((size_t)par * R0S<VW * L>::n + slot) * 2 + tab) * (VW * L);
}
template <int L, int VW>
struct Row0Loads {
  static constexpr int NC = 2 * L;  // V columns (both tables)
  typename SV<VW>::Fx g[R0S<VW * L>::n];
  typename SV<VW>::T rp, ra;
};
// every load issued unconditionally, first thing in the kernel (a load
// under a branch is waited for at the join); threads >= NC load column
// col - NC's words too (unused), q == 0 loads set 2 (not read)
template <int L, int VW>
__device__ __forceinline__ void row0_issue(const TrainArgs &a, int q,
                                           Row0Loads<L, VW> &ld) {
  using RL = Row0Loads<L, VW>;
  const int col = threadIdx.x % RL::NC;
  const int tab = col / L, c = col % L, ppar = (q + 2) % 3;
  // the address is selected (q is uniform), not the loaded value
  ld.rp = (q ? sh_row<L, VW>(a, ppar, tab, 0) : tab_row<L, VW>(a, tab, 0, 0))[c];
  ld.ra = (q ? sh_row<L, VW>(a, ppar, tab, 1) : tab_row<L, VW>(a, tab, 1, 0))[c];
#pragma unroll
  for (int j = 0; j < R0S<VW * L>::n; j++)
    ld.g[j] = SV<VW>::ldfix(r0_row<L, VW>(a, ppar, j, tab), c);
}
// column owners (threads < NC): the slots' exact integer sum, the previous
// batch's row-0 step (zero gradient for the first batch of an epoch)
template <int L, int VW>
__device__ __forceinline__ void row0_finish(const TrainArgs &a, int q,
                                            const Row0Loads<L, VW> &ld,
                                            typename SV<VW>::T &p0, typename SV<VW>::T &a0) {
  using S = SV<VW>;
  typename S::Fx t = ld.g[0];
#pragma unroll
  for (int j = 1; j < R0S<VW * L>::n; j++) t = S::fxadd(t, ld.g[j]);
  if (g_tab & 2048) t = S::fxzero();  // (debug ablation)
  if (q) S::adagrad(p0, a0, S::unfix(t), a.lr, a.eps);
}

// One launch = one batch. q = the batch's index in the epoch (parities
// q % 3 and q & 1). One L-lane group per record (dp == 4L), RPB = TB / L
// records per workgroup, ceil(B / RPB) workgroups; records placed by
// train_place, those without neighbour lists first (whole waves skip the list
// gathers).
// Early row-0 sums (float2 rows, d = 128): every record group adds its own
// row-0 gradients (the same float adds in emit order) to the fixed-point
// slot right after its forward pass, before its row stores, and stores its
// own loss word: no end-of-batch workgroup barrier. Interleaved A/B on C3
// HOBE records: 6.69 -> 6.65 us per batch, epoch 36.85M -> 37.09M records/s
// (profiles/r03/trainer/prep2/ab_diet_128.txt). HGX_TRAIN_R0EARLY=0 (A/B
// builds): the workgroup's fixed-order float sum, one atomic per column.
#ifndef HGX_TRAIN_R0EARLY
#define HGX_TRAIN_R0EARLY 1
#endif
template <int L, int VW, int KMAX, int MODE, int TB, bool MULTI>
__global__ __launch_bounds__(TB) void train_step(TrainArgs a, int cb, int gb, int nb, int q) {
  constexpr int RPB = TB / L, R = 4 + 2 * KMAX, K = KMAX, NC = 2 * L;
  using S = SV<VW>;
  using V = typename S::T;
  static_assert(L == 32 || L == 64, "step geometry");
  static_assert(R + kWX <= 32, "slot and batch words fit the first 32 lanes");
  // early row-0 sums at float2 rows only (at float4 rows, d = 256, the 4x
  // integer atomics cost more than the barrier: 8.49 -> 10.42 us per batch)
  constexpr bool kR0E = HGX_TRAIN_R0EARLY && VW == 2;
  __shared__ V s_z[2][RPB][L];
  __shared__ V s_gl[RPB][R][L];  // gradients of local (one-record) rows
  __shared__ V s_r0[2][L];
  __shared__ float s_loss[RPB];
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g_trace) ts[0] = __builtin_amdgcn_s_memrealtime();
  const int grp = threadIdx.x / L, lane = threadIdx.x % L;
  const int NBF = gridDim.x, RW = a.RW;
  const int par = q % 3, ppar = (q + 2) % 3, zpar = (q + 1) % 3;
  // round trip 1 (kernel arguments only): record ids and slot codes (one
  // load per lane, readlane broadcast), flush slots, the batch words,
  // targets, the row-0 base and the previous batch's row-0 partials
  const size_t gi = ((size_t)cb * NBF + blockIdx.x) * RPB + grp;
  const int *ri = a.pidx + gi * RW;
  const unsigned *rc = a.pcode + gi * RW;
  const float *yt = a.ptgt + gi * 3;
  int row[R], frow[kFX];
  unsigned code[R], fcode[kFX];
  int nfo, zc;  // batch words: overflow flushes, gacc entries to zero
  // every round-trip-1 load is issued before the first use of any of them
  // (the readlane broadcasts below wait for the id words)
  const int sl = lane < RW ? lane : 0;
  const int rv = ri[sl];
  const int cv = (int)rc[sl];
  const int tv = __float_as_int(yt[L == 64 ? (lane < 3 ? lane : 0) : 0]);
  float yt1 = 0.f, yt2 = 0.f;
  if (L == 32) {
    yt1 = yt[1];
    yt2 = yt[2];
  }
  // the previous batch's row-0 gradient slots (none for the first batch of
  // an epoch: row 0 from the table)
  Row0Loads<L, VW> r0l;
  row0_issue<L, VW>(a, q, r0l);
  {
#pragma unroll
    for (int s = 0; s < R + kFX; s++) {
      int r, c;
      if (L == 64) {
        r = __builtin_amdgcn_readlane(rv, s);
        c = __builtin_amdgcn_readlane(cv, s);
      } else {
        const bool hi = threadIdx.x & 32;
        const int r0 = __builtin_amdgcn_readlane(rv, s), r1 = __builtin_amdgcn_readlane(rv, 32 + s);
        const int c0 = __builtin_amdgcn_readlane(cv, s), c1 = __builtin_amdgcn_readlane(cv, 32 + s);
        r = hi ? r1 : r0;
        c = hi ? c1 : c0;
      }
      if (s < R) {
        row[s] = r;
        code[s] = (unsigned)c;
      } else {
        frow[s - R] = r;
        fcode[s - R] = (unsigned)c;
      }
    }
    // the same in every group of the batch: lane R + kFX + i of the low half
    nfo = __builtin_amdgcn_readlane(rv, R + kFX);
    zc = __builtin_amdgcn_readlane(rv, R + kFX + 1);
  }
  float yt0 = __int_as_float(tv);
  if (L == 64) {
    // lane c < 3 loaded target c: readlanes broadcast them (scalar)
    yt0 = __int_as_float(__builtin_amdgcn_readlane(tv, 0));
    yt1 = __int_as_float(__builtin_amdgcn_readlane(tv, 1));
    yt2 = __int_as_float(__builtin_amdgcn_readlane(tv, 2));
  }
  HGX_STAMP(ts[1]);
  // records were dealt round robin over the workgroups (train_place)
  const int nval = min(max(nb - (int)blockIdx.x + NBF - 1, 0) / NBF, RPB);
  const bool has = grp < nval;
  const int col = threadIdx.x % NC, sub = threadIdx.x / NC, tab0 = col / L, c0 = col % L;
  int bad = 0;
  if (nval > 0) {
    V p0 = r0l.rp, a0 = r0l.ra;
    S::pin(p0);
    S::pin(a0);
    // round trip 2: every slot's table row and the accumulator row where
    // this slot owns the row's update (else the hot row 0; a pending slot's
    // rows are replaced by the previous batch's shadow below). List slots
    // are skipped by a WAVE-uniform branch when no record of the wave has a
    // list.
    V Pv[R], Av[R];
    bool lists = false;
#pragma unroll
    for (int s = 4; s < R; s++) lists |= row[s] != 0;
    const bool wave_lists = __any(lists);
    // (table rows only: a per-lane select between the table and the shadow
    // as the load base made the gathers 64-bit per-lane addresses and cost
    // 0.6 us per batch)
    auto gather = [&](int s) {
      const bool edge = slot_is_edge(s, K);
      const V *T = reinterpret_cast<const V *>(edge ? a.etab : a.ntab);
      const V *Ac = reinterpret_cast<const V *>(edge ? a.eacc : a.nacc);
      const int arow = (code[s] & kSOwn) ? row[s] : 0;
      Pv[s] = T[(size_t)row[s] * L + lane];
      Av[s] = Ac[(size_t)arow * L + lane];
    };
#pragma unroll
    for (int s = 0; s < 4; s++) {
      // at L = 64 (one record per wave, scalar ids) the two padding slots of
      // the first four are skipped: their value comes from s_r0 below
      if (L == 64 && row[s] == 0) {
        Pv[s] = Av[s] = S::zero();
        continue;
      }
      gather(s);
    }
    if (wave_lists && !(g_tab & 32768)) {  // (debug ablation: no list gathers)
#pragma unroll
      for (int s = 4; s < R; s++) gather(s);
    } else if (wave_lists) {
#pragma unroll
      for (int s = 4; s < R; s++) Pv[s] = Av[s] = S::zero();
    }
    // flush slot 0 (one deferred row per group in the common case) rides on
    // the same round trip
    // (no default values: a conditional assignment over a default makes the
    // compiler copy the loaded registers at the join, i.e. wait for them and
    // drain every gather before the barrier)
    V fp, fa;
    typename S::Fx fg;
    if (__any(frow[0] != 0)) {
      const int mf = (fcode[0] >> kDefBits) & kDefMask;
      fp = sh_row<L, VW>(a, ppar, mf, 0)[lane];
      fa = sh_row<L, VW>(a, ppar, mf, 1)[lane];
      fg = S::ldfix(gacc_row<L, VW>(a, ppar, mf), lane);
    }
    if (sub == 0) {
      row0_finish<L, VW>(a, q, r0l, p0, a0);
      s_r0[tab0][c0] = p0;
      if (blockIdx.x == 0) {
        st_row(&sh_row<L, VW>(a, par, tab0, 0)[c0], p0);
        st_row(&sh_row<L, VW>(a, par, tab0, 1)[c0], a0);
      }
    }
    __syncthreads();  // s_r0
    HGX_STAMP(ts[2]);
    // flush slot 0: folded and written back now (its registers are free
    // for the forward pass; nothing of this batch reads the row)
    if (has && frow[0] != 0) {
      fold<VW>(fp, fa, fg, a.lr, a.eps);
      const bool fe = fcode[0] & kFEdge;
      st_row(&tab_row<L, VW>(a, fe, 0, frow[0])[lane], fp);
      st_row(&tab_row<L, VW>(a, fe, 1, frow[0])[lane], fa);
    }
    // pending slots (rows deferred by the previous batch): base row from the
    // previous batch's shadow, folded with its gacc sum, written to every
    // slot of the record that names the same entry. A select pass handles
    // one entry per record (picked by v_cndmask: no dynamic register index,
    // no loop-carried copies of the rows). MULTI = 0: train_place found at
    // most one entry per record in this batch, one pass (normally not
    // taken); MULTI = 1: two passes, then slot by slot.
    unsigned pm = 0;
#pragma unroll
    for (int s = 0; s < R; s++)
      if (code[s] & kSPend) pm |= 1u << s;
    if (!has) pm = 0;
    auto fold_pass = [&]() {
      if (!__any(pm != 0)) return;
      const int ps = pm ? __builtin_ctz(pm) : 0;
      unsigned cd = 0;
#pragma unroll
      for (int s = 0; s < R; s++)
        if (s == ps) cd = code[s];
      const unsigned mp = (cd >> kDefBits) & kDefMask;
      const typename S::Fx gg = S::ldfix(gacc_row<L, VW>(a, ppar, mp), lane);
      V pp = sh_row<L, VW>(a, ppar, mp, 0)[lane], aa = sh_row<L, VW>(a, ppar, mp, 1)[lane];
      // the record's slots naming the same entry (a mask: the write-back
      // below is one bit test per slot)
      unsigned wm = 0;
#pragma unroll
      for (int s = 0; s < R; s++)
        if (((code[s] >> kDefBits) & kDefMask) == mp) wm |= 1u << s;
      wm &= pm;
      fold<VW>(pp, aa, gg, a.lr, a.eps);
#pragma unroll
      for (int s = 0; s < R; s++)
        if ((wm >> s) & 1u) {
          Pv[s] = pp;
          Av[s] = aa;
        }
      pm &= ~wm;
    };
    fold_pass();
    if (MULTI) {
      fold_pass();
      if (__any(pm != 0)) {
#pragma unroll
        for (int s = 0; s < R; s++) {
          if (!__any((pm >> s) & 1u)) continue;
          const int mp = (code[s] >> kDefBits) & kDefMask;
          const typename S::Fx gg = S::ldfix(gacc_row<L, VW>(a, ppar, mp), lane);
          V pp = sh_row<L, VW>(a, ppar, mp, 0)[lane], aa = sh_row<L, VW>(a, ppar, mp, 1)[lane];
          fold<VW>(pp, aa, gg, a.lr, a.eps);
          if ((pm >> s) & 1u) {
            Pv[s] = pp;
            Av[s] = aa;
          }
        }
      }
    }
    V zN = S::zero(), zE = S::zero();
    float lrec = 0.f;
    if (has) {
#pragma unroll
      for (int s = 0; s < R; s++)
        if (row[s] == 0) Pv[s] = s_r0[slot_is_edge(s, K) ? 1 : 0][lane];
      const float inv_b = 1.0f / (float)nb;
      const V &Nl = Pv[0], &El = Pv[1], &Nr = Pv[2], &Er = Pv[3];
      float z1, z2, za[K], zb[K];
      if (g_tab & 4096) {  // (debug ablation: no reductions)
        z1 = S::dot(Nl, Nr);
        z2 = S::dot(El, Er);
#pragma unroll
        for (int k = 0; k < K; k++) {
          za[k] = S::dot(Pv[4 + k], Nl);
          zb[k] = S::dot(Pv[4 + K + k], Er);
        }
      } else if constexpr (L == 64 && (2 + 2 * K) % 4 == 0) {
        // the 2 + 2K head dots reduced together (same sums, no serial chain)
        float zz[2 + 2 * K];
        zz[0] = S::dot(Nl, Nr);
        zz[1] = S::dot(El, Er);
#pragma unroll
        for (int k = 0; k < K; k++) {
          zz[2 + k] = S::dot(Pv[4 + k], Nl);
          zz[2 + K + k] = S::dot(Pv[4 + K + k], Er);
        }
        hgx::wave_allreduce_sum_n<2 + 2 * K>(zz);
        z1 = zz[0];
        z2 = zz[1];
#pragma unroll
        for (int k = 0; k < K; k++) {
          za[k] = zz[2 + k];
          zb[k] = zz[2 + K + k];
        }
      } else {
        z1 = group_sum<L>(S::dot(Nl, Nr));
        z2 = group_sum<L>(S::dot(El, Er));
#pragma unroll
        for (int k = 0; k < K; k++) {
          za[k] = group_sum<L>(S::dot(Pv[4 + k], Nl));
          zb[k] = group_sum<L>(S::dot(Pv[4 + K + k], Er));
        }
      }
      const int act = MODE == 1 ? 0 : 1;
      const int lossk = MODE == 1 ? 0 : 1;
      const float y1 = act_f(act, z1), y2 = act_f(act, z2);
      float sa[K], sb[K], P = 0.f, Q = 0.f;
#pragma unroll
      for (int k = 0; k < K; k++) {
        sa[k] = act_f(act, za[k]);
        sb[k] = act_f(act, zb[k]);
        P += sa[k];
        Q += sb[k];
      }
      P = P / (float)K;
      Q = Q / (float)K;
      const float y3 = P * Q;
      float l1, l2, l3, g1, g2, g3;
      head_loss(lossk, y1, yt0, l1, g1);
      head_loss(lossk, y2, yt1, l2, g2);
      head_loss(lossk, y3, yt2, l3, g3);
      lrec = l1 + l2 + l3;
      HGX_STAMP(ts[3]);
      g1 *= inv_b;
      g2 *= inv_b;
      g3 *= inv_b;
      const float dz1 = g1 * act_d(act, z1, y1);
      const float dz2 = g2 * act_d(act, z2, y2);
      const float dP = g3 * Q / (float)K, dQ = g3 * P / (float)K;
      auto emit = [&](int s, V g) {
        const unsigned cd = code[s];
        const bool edge = slot_is_edge(s, K);
        if (row[s] == 0) {
          if (!kR0E) {
            if (edge) zE = S::add(zE, g);
            else zN = S::add(zN, g);
          }
        } else if (cd & kSLocal) {
          // one record's slots of a row, summed in emit order in LDS (the
          // wave's own accesses, in order); the last one (owner) updates
          V *acc = &s_gl[grp][cd & 15u][lane];
          if (cd & kSOwn) {
            V pv = Pv[s], av = Av[s];
            S::adagrad(pv, av, S::add(*acc, g), a.lr, a.eps);
            st_row(&tab_row<L, VW>(a, edge, 0, row[s])[lane], pv);
            st_row(&tab_row<L, VW>(a, edge, 1, row[s])[lane], av);
          } else {
            *acc = (cd & kSFirst) ? g : S::add(*acc, g);
          }
        } else if (cd & kSShared) {
          const int m = cd & kDefMask;
          if (g_tab & 1024)  // (debug ablation: plain stores, wrong sums)
            reinterpret_cast<V *>(gacc_row<L, VW>(a, par, m))[lane] = g;
          else
            S::addfix(gacc_row<L, VW>(a, par, m), lane, g, bad);
          if (cd & kSOwn) {
            st_row(&sh_row<L, VW>(a, par, m, 0)[lane], Pv[s]);
            st_row(&sh_row<L, VW>(a, par, m, 1)[lane], Av[s]);
          }
        } else {
          V pv = Pv[s], av = Av[s];
          if (g_tab & 8192) {  // (debug ablation: no Adagrad arithmetic)
            pv = S::add(pv, g);
            av = S::add(av, g);
          } else {
            S::adagrad(pv, av, g, a.lr, a.eps);
          }
          st_row(&tab_row<L, VW>(a, edge, 0, row[s])[lane], pv);
          st_row(&tab_row<L, VW>(a, edge, 1, row[s])[lane], av);
        }
      };
      V gln = S::fma(dz1, Nr, S::zero()), gre = S::fma(dz2, El, S::zero());
      if (kR0E) {
        // the row-0 sums in emit order first (the same adds as below), added
        // to this record's slot before any row store
        float da[K], db[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
          da[k] = dP * act_d(act, za[k], sa[k]);
          db[k] = dQ * act_d(act, zb[k], sb[k]);
          gln = S::fma(da[k], Pv[4 + k], gln);
          gre = S::fma(db[k], Pv[4 + K + k], gre);
          if (row[4 + k] == 0) zN = S::add(zN, S::fma(da[k], Nl, S::zero()));
          if (row[4 + K + k] == 0) zE = S::add(zE, S::fma(db[k], Er, S::zero()));
        }
        if (row[0] == 0) zN = S::add(zN, gln);
        if (row[3] == 0) zE = S::add(zE, gre);
        if (row[2] == 0) zN = S::add(zN, S::fma(dz1, Nl, S::zero()));
        if (row[1] == 0) zE = S::add(zE, S::fma(dz2, Er, S::zero()));
        const int slot = (blockIdx.x * RPB + grp) % R0S<VW * L>::n;
        S::addfix(r0_row<L, VW>(a, par, slot, 0), lane, zN, bad);
        S::addfix(r0_row<L, VW>(a, par, slot, 1), lane, zE, bad);
        if (lane == 0) a.lossbuf[(size_t)gb * a.lstride + blockIdx.x * RPB + grp] = lrec;
#pragma unroll
        for (int k = 0; k < K; k++) {
          emit(4 + k, S::fma(da[k], Nl, S::zero()));
          emit(4 + K + k, S::fma(db[k], Er, S::zero()));
        }
      } else {
#pragma unroll
        for (int k = 0; k < K; k++) {
          const float da = dP * act_d(act, za[k], sa[k]);
          const float db = dQ * act_d(act, zb[k], sb[k]);
          gln = S::fma(da, Pv[4 + k], gln);
          gre = S::fma(db, Pv[4 + K + k], gre);
          emit(4 + k, S::fma(da, Nl, S::zero()));
          emit(4 + K + k, S::fma(db, Er, S::zero()));
        }
      }
      emit(0, gln);
      emit(3, gre);
      emit(2, S::fma(dz1, Nl, S::zero()));
      emit(1, S::fma(dz2, Er, S::zero()));
      HGX_STAMP(ts[4]);
    }
    if (!kR0E) {
      s_z[0][grp][lane] = zN;
      s_z[1][grp][lane] = zE;
      if (lane == 0) s_loss[grp] = lrec;
      if (!(g_tab & 16384)) __syncthreads();  // (debug ablation: no barrier)
      // this batch's row-0 gradients: the workgroup's fixed-order sum, added
      // to its slot of r0acc[q % 3] in fixed point
      if (threadIdx.x < NC && !(g_tab & 16384)) {
        V sz = S::zero();
        for (int g = 0; g < RPB; g++) sz = S::add(sz, s_z[tab0][g][c0]);
        S::addfix(r0_row<L, VW>(a, par, blockIdx.x % R0S<VW * L>::n, tab0), c0, sz, bad);
      }
      if (threadIdx.x == 0) {
        float sl = 0.f;
        for (int g = 0; g < RPB; g++) sl += s_loss[g];
        a.lossbuf[(size_t)gb * a.lstride + blockIdx.x] = sl;
      }
    }
    // flush slots 1.. (more deferred rows than records in the batch)
    bool more = false;
#pragma unroll
    for (int f = 1; f < kFX; f++) more |= frow[f] != 0;
    if (__any(more)) {
#pragma unroll
      for (int f = 1; f < kFX; f++)
        if (frow[f] != 0)
          flush_row<L, VW>(a, ppar, (fcode[f] & kFEdge ? 1 << 30 : 0) | frow[f],
                       (fcode[f] >> kDefBits) & kDefMask, lane);
    }
  }
  HGX_STAMP(ts[5]);
  // flush overflow list (rare: more deferred rows than kFX per record)
  for (int e = blockIdx.x * RPB + grp; e < nfo; e += NBF * RPB) {
    const int2 en = a.pfo[(size_t)cb * a.Mmax + e];
    flush_row<L, VW>(a, ppar, en.x, en.y, lane);
  }
  // zero the gacc parity the next batch adds into (its deferred entries
  // [2, 2 + zc) were used two batches ago) and the row-0 slots it adds into
  {
    longlong2 *z = reinterpret_cast<longlong2 *>(gacc_row<L, VW>(a, zpar, 2));
    const int tot = zc * (VW / 2) * L;
    for (int i = blockIdx.x * TB + threadIdx.x; i < tot; i += NBF * TB)
      z[i] = make_longlong2(0, 0);
    longlong2 *zr = reinterpret_cast<longlong2 *>(r0_row<L, VW>(a, zpar, 0, 0));
    for (int i = blockIdx.x * TB + threadIdx.x; i < R0S<VW * L>::n * VW * L; i += NBF * TB)
      zr[i] = make_longlong2(0, 0);
  }
  // (timing ablations compute wrong values: no overflow verdict for them)
  if (__any(bad) && !g_tab && (threadIdx.x & 63) == 0) atomicOr(a.ovf, 1);
  HGX_STAMP(ts[6]);
  trace_put(gb, 0, 7, ts);
}

// End of an epoch: the last batch's deferred rows folded into the tables
// (row 0 of both tables from its np partials, its shared rows from gacc;
// keys from train_prep), and every gacc entry still in use zeroed (the last
// batch's and the one before it, Ml and Mp entries). One L-lane group per
// entry.
template <int L>
__global__ __launch_bounds__(256) void train_flush(TrainArgs a, const int *keys,
                                                   const int *Ml, const int *Mp,
                                                   int q, int np) {
  constexpr int GPB = 256 / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x % L;
  const int par = q % 3, opar = (q + 2) % 3;
  const int M = 2 + *Ml, zc = Mp ? *Mp : 0;
  for (int e = blockIdx.x * GPB + grp; e < M; e += gridDim.x * GPB) {
    if (e < 2) {  // row 0: the last batch's slots, summed as train_step sums
      SV<4>::Fx t = SV<4>::ldfix(r0_row<L, 4>(a, par, 0, e), lane);
      for (int j = 1; j < R0S<4 * L>::n; j++)
        t = SV<4>::fxadd(t, SV<4>::ldfix(r0_row<L, 4>(a, par, j, e), lane));
      const float4 g = SV<4>::unfix(t);
      float4 p = sh_row<L, 4>(a, par, e, 0)[lane], ac = sh_row<L, 4>(a, par, e, 1)[lane];
      adagrad4_hw(p, ac, g, a.lr, a.eps);
      tab_row<L, 4>(a, e, 0, 0)[lane] = p;
      tab_row<L, 4>(a, e, 1, 0)[lane] = ac;
      continue;
    }
    flush_row<L, 4>(a, par, keys[e - 2], e, lane);
    SV<4>::zerofix(gacc_row<L, 4>(a, par, e), lane);
  }

  longlong2 *z = reinterpret_cast<longlong2 *>(gacc_row<L, 4>(a, opar, 2));
  for (int i = blockIdx.x * 256 + threadIdx.x; i < zc * 2 * L; i += gridDim.x * 256)
    z[i] = make_longlong2(0, 0);
}

// Slot codes of one batch (tail of train_prep, the batch's (row, slot) keys
// sorted in LDS). Per run of equal rows:
//  - one slot: kSOwn (in-place update by its group);
//  - several slots of ONE record: kSLocal; its group sums the slots'
//    gradients in LDS in emit order, the last slot in that order owns the
//    update (no deferral, no atomics);
//  - slots in several records: deferred entry m = 2 + its rank among the
//    batch's deferred rows (sorted key order), kSShared, the first slot owns
//    the shadow write.
// Writes per-slot codes (batch slot order), the deferred rows' keys
// (ascending) and their count. u0 = the unique-run index of this thread's
// first sorted position.
// position of slot s in train_step's emit order: 4 + k, 4 + K + k for
// k = 0..K-1, then 0, 3, 2, 1
__device__ __forceinline__ int emit_pos(int s, int K) {
  if (s >= 4 + K) return 2 * (s - 4 - K) + 1;
  if (s >= 4) return 2 * (s - 4);
  return 2 * K + (s == 0 ? 0 : s == 3 ? 1 : s == 2 ? 2 : 3);
}

__device__ void defer_codes(const TrainArgs &a, int cb, int V, int P, int u0,
                            const unsigned long long *s_key, int *s_ws, int *s_runm,
                            int *skey, int *sM) {
  const int per = P / kTB, t0 = threadIdx.x * per, t1 = min(t0 + per, V);
  const int R = a.R;
  constexpr int kDefer = 1 << 30;  // run class: deferred (m assigned below)
  auto k32 = [&](int t) { return (unsigned)(s_key[t] >> 32); };
  auto slot = [&](int t) { return (int)(unsigned)(s_key[t] & 0xffffffffu); };
  auto starts = [&](int t) { return t == 0 || k32(t - 1) != k32(t); };
  // classify the runs starting in this thread's chunk: 0 single, a slot mask
  // (local), or kDefer
  int ns = 0;
  int u = u0;
  for (int t = t0; t < t1; t++) {
    if (!starts(t)) continue;
    int e = t + 1;
    while (e < V && k32(e) == k32(t)) e++;
    int cls = 0;
    if (e - t > 1) {
      if (slot(t) / R == slot(e - 1) / R) {
        cls = 1;  // local
      } else {
        cls = kDefer;
        ns++;
      }
    }
    s_runm[u++] = cls;
  }
  int S = 0;
  int m = block_exclusive_scan(ns, &S, s_ws);
  int *keys = skey + (size_t)cb * a.Mmax;
  u = u0;
  for (int t = t0; t < t1; t++) {
    if (!starts(t)) continue;
    if (s_runm[u] == kDefer) {
      s_runm[u] = kDefer | (2 + m);
      keys[m++] = (int)k32(t);
    }
    u++;
  }
  __syncthreads();
  unsigned *sc = a.scode + (size_t)cb * a.SB;
  u = u0;
  for (int t = t0; t < t1; t++) {
    const bool st = starts(t);
    u += st;
    const int cls = s_runm[u - 1];
    unsigned code = kSOwn;
    if (cls & kDefer) {
      code = kSShared | (st ? kSOwn : 0u) | (unsigned)(cls & (kDefer - 1));
    } else if (cls) {
      // local: the run's slots in train_step's emit order; the last owns the
      // update, the first writes the LDS sum, bits 0..3 = the owner's slot
      int rs = t;  // the run start
      while (rs > 0 && k32(rs - 1) == k32(t)) rs--;
      int re = t + 1;
      while (re < V && k32(re) == k32(t)) re++;
      const int me = emit_pos(slot(t) % R, a.K);
      int first = 1, last = 1, own = slot(t) % R;
      for (int j = rs; j < re; j++) {
        const int e2 = emit_pos(slot(j) % R, a.K);
        first &= e2 >= me;
        last &= e2 <= me;
        if (e2 > emit_pos(own, a.K)) own = slot(j) % R;
      }
      code = kSLocal | (last ? kSOwn : 0u) | (first ? kSFirst : 0u) | (unsigned)own;
    }
    sc[slot(t)] = code;
  }
  if (threadIdx.x == 0) sM[cb] = S;
}

// The unique-key and slot-code phases of train_prep for the radix-sorted
// batch (P == kSortP), from the sort's registers: thread t holds sorted
// positions [t * PER, t * PER + PER) (keys kk, slots vv), the same chunk the
// generic path scans in LDS. Run starts, run ends (the last slot of the run
// by a backward pass over the chunk; a run leaving the chunk is followed in
// LDS) and the run classes stay in registers, every array indexed at compile
// time; local runs (rare) use the generic LDS scan. Same outputs as the
// generic unique phase + defer_codes, bit for bit.
template <int PER>
__device__ void prep_runs_regs(const TrainArgs &a, int cb, int P, const unsigned (&kk)[PER],
                               const int (&vv)[PER], const unsigned long long *s_key, int *s_ws,
                               unsigned short *s_runm, int *skey, int *sM) {
  const int R = a.R, t0 = threadIdx.x * PER;
  constexpr int kDefer = 1 << 30;
  const bool split = !a.fused;
  const unsigned kprev = t0 > 0 ? (unsigned)(s_key[t0 - 1] >> 32) : 0xffffffffu;
  const unsigned knext = t0 + PER < P ? (unsigned)(s_key[t0 + PER] >> 32) : 0xffffffffu;
  bool vld[PER], st[PER], eq[PER];
  int cnt = 0, valid = 0;
#pragma unroll
  for (int i = 0; i < PER; i++) {
    vld[i] = kk[i] != 0xffffffffu;
    st[i] = vld[i] && kk[i] != (i ? kk[i - 1] : kprev);
    eq[i] = vld[i] && kk[i] == (i + 1 < PER ? kk[i + 1] : knext);
    cnt += st[i];
    valid += vld[i];
  }
  int U = 0, V = 0;
  const int u0 = block_exclusive_scan(cnt, &U, s_ws);
  block_exclusive_scan(valid, &V, s_ws);
  {
    int *ukey = a.ukey + (size_t)cb * a.SB;
    int *uoff = a.uoff + (size_t)cb * (a.SB + 1);
    int *inv = a.inv + (size_t)cb * a.SB;
    int u = u0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
      if (!vld[i]) continue;
      if (split) inv[vv[i]] = t0 + i;
      if (st[i]) {
        ukey[u] = (int)kk[i];
        if (split) uoff[u] = t0 + i;
        u++;
      }
    }
    if (threadIdx.x == 0) {
      if (split) uoff[U] = V;
      a.ucount[cb] = U;
    }
  }
  if (!a.fused) return;
  // the last slot of the run through position i (a run leaving the chunk:
  // followed in LDS)
  int lastsl[PER];
  {
    int ls = vv[PER - 1];
    if (eq[PER - 1]) {
      int pos = t0 + PER;
      while (pos < V && (unsigned)(s_key[pos] >> 32) == kk[PER - 1]) pos++;
      ls = (int)(unsigned)s_key[pos - 1];
    }
    lastsl[PER - 1] = ls;
  }
#pragma unroll
  for (int i = PER - 2; i >= 0; i--) lastsl[i] = eq[i] ? lastsl[i + 1] : vv[i];
  // classes of the runs starting here: 0 single, 1 local, kDefer (+ 2 + m)
  int cls[PER];
  int ns = 0;
#pragma unroll
  for (int i = 0; i < PER; i++) {
    cls[i] = 0;
    if (st[i] && eq[i]) {
      cls[i] = (vv[i] / R == lastsl[i] / R) ? 1 : kDefer;
      ns += cls[i] == kDefer;
    }
  }
  int S = 0;
  int m = block_exclusive_scan(ns, &S, s_ws);
  int *keys = skey + (size_t)cb * a.Mmax;
  {
    int u = u0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
      if (!st[i]) continue;
      if (cls[i] == kDefer) {
        cls[i] = kDefer | (2 + m);
        keys[m++] = (int)kk[i];
      }
      // 16-bit in LDS: 0, 1 or 0x8000 | (2 + m) (2 + m <= SB / 2 + 2 < 2^15)
      s_runm[u++] = (unsigned short)(cls[i] & kDefer ? 0x8000 | (cls[i] & 0x7fff) : cls[i]);
    }
  }
  __syncthreads();
  auto k32 = [&](int t) { return (unsigned)(s_key[t] >> 32); };
  auto slot = [&](int t) { return (int)(unsigned)(s_key[t] & 0xffffffffu); };
  unsigned *sc = a.scode + (size_t)cb * a.SB;
  // the run through the chunk's first position began before it: its class
  int cur = 0;
  if (u0 > 0 && vld[0] && !st[0]) {
    const int v = s_runm[u0 - 1];
    cur = v & 0x8000 ? kDefer | (v & 0x7fff) : v;
  }
#pragma unroll
  for (int i = 0; i < PER; i++) {
    if (!vld[i]) continue;
    if (st[i]) cur = cls[i];
    const int t = t0 + i;
    unsigned code = kSOwn;
    if (cur & kDefer) {
      code = kSShared | (st[i] ? kSOwn : 0u) | (unsigned)(cur & (kDefer - 1));
    } else if (cur) {
      // local: as defer_codes
      int rs = t;
      while (rs > 0 && k32(rs - 1) == kk[i]) rs--;
      int re = t + 1;
      while (re < V && k32(re) == kk[i]) re++;
      const int me = emit_pos(vv[i] % R, a.K);
      int first = 1, last = 1, own = vv[i] % R;
      for (int j = rs; j < re; j++) {
        const int e2 = emit_pos(slot(j) % R, a.K);
        first &= e2 >= me;
        last &= e2 <= me;
        if (e2 > emit_pos(own, a.K)) own = slot(j) % R;
      }
      code = kSLocal | (last ? kSOwn : 0u) | (first ? kSFirst : 0u) | (unsigned)own;
    }
    sc[vv[i]] = code;
  }
  if (threadIdx.x == 0) sM[cb] = S;
}

__device__ __forceinline__ int bsearch_lds(const int *v, int n, int key) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && v[lo] == key ? lo : -1;
}

// Record placement of one batch for train_step (one workgroup per batch of
// the chunk, after train_prep): records without neighbour lists first
// (stable; position p to workgroup p % NBF), RW words per group (R slot ids / codes, kFX flush slots, the
// batch words: overflow flushes and the gacc entries train_step zeroes,
// i.e. the deferred rows of the batch two before this one). Slot
// codes get kSPend | m' << 12 where the row is deferred entry m' of the
// previous batch (that batch's keys: skey_cur[cb - 1], or the previous
// chunk's last batch). The previous batch's deferred rows this batch does not
// touch become flush slots (the group of record position f % nb, slot f / nb), past kFX * nb the
// overflow list.
__global__ __launch_bounds__(kTB) void train_place(TrainArgs a, int nbc, int CB,
                                                   const int *skey_cur, const int *sM_cur,
                                                   const int *skey_pc, const int *sM_pc,
                                                   int has_prev) {
  extern __shared__ int s_dyn[];
  __shared__ int s_pos[kPackB];
  __shared__ int s_ws[kTB / 64];
  const int cb = blockIdx.x;
  if (cb >= nbc) return;
  const int nb = a.bmeta[cb].x;
  const int R = a.R, K = a.K, RW = a.RW, RPB = a.prpb, SB = a.SB;
  const int G = (a.B + RPB - 1) / RPB * RPB;
  const int *prev = nullptr;
  int Mp = 0, Mpp = 0;  // deferred rows of the batches one and two before
  if (cb > 0) {
    prev = skey_cur + (size_t)(cb - 1) * a.Mmax;
    Mp = sM_cur[cb - 1];
  } else if (has_prev) {
    prev = skey_pc + (size_t)(CB - 1) * a.Mmax;
    Mp = sM_pc[CB - 1];
  }
  if (cb > 1) Mpp = sM_cur[cb - 2];
  else if (has_prev) Mpp = sM_pc[CB - 2 + cb];
  const int U = a.ucount[cb];
  int *s_prev = s_dyn, *s_u = s_dyn + a.Mmax;
  __shared__ int s_brk;
  if (threadIdx.x == 0) s_brk = 0;
  for (int j = threadIdx.x; j < Mp; j += kTB) s_prev[j] = prev[j];
  for (int j = threadIdx.x; j < U; j += kTB) s_u[j] = a.ukey[(size_t)cb * SB + j];
  const int *bidx = a.bidx + (size_t)cb * a.B * R;
  const float *btgt = a.btgt + (size_t)cb * a.B * 3;
  __syncthreads();
  // a record naming two of the previous batch's deferred rows: the batch
  // takes train_step's MULTI form (the light form folds one per record)
  for (int i = threadIdx.x; i < nb && Mp; i += kTB) {
    int e0 = -1;
    for (int s2 = 0; s2 < R; s2++) {
      const int row = bidx[i * R + s2];
      if (row == 0) continue;
      const int j = bsearch_lds(s_prev, Mp, ((int)slot_is_edge(s2, K) << 30) | row);
      if (j < 0) continue;
      if (e0 >= 0 && j != e0) s_brk = 1;
      e0 = j;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) a.pbrk[cb] = s_brk;
  // stable partition: records without lists first
  {
    const int per = (nb + kTB - 1) / kTB, i0 = threadIdx.x * per, i1 = min(i0 + per, nb);
    int cs = 0;
    for (int i = i0; i < i1; i++) {
      int any = 0;
      for (int s = 4; s < R; s++) any |= bidx[i * R + s];
      s_pos[i] = any;  // temporarily: has a list
      cs += any == 0;
    }
    int NS = 0;
    int bs = block_exclusive_scan(cs, &NS, s_ws);
    // position p of the partitioned order -> workgroup p % NBF, group p / NBF:
    // every workgroup gets its share of the list records (the step's slowest
    // workgroup sets the batch time), its list-less records first
    const int NBF = G / RPB;
    for (int i = i0; i < i1; i++) {
      const bool sh = s_pos[i] == 0;
      const int p = sh ? bs : NS + (i - bs);
      s_pos[i] = (p % NBF) * RPB + p / NBF;
      bs += sh;
    }
  }
  int *pidx = a.pidx + (size_t)cb * G * RW;
  unsigned *pcode = a.pcode + (size_t)cb * G * RW;
  float *ptgt = a.ptgt + (size_t)cb * G * 3;
  for (int t = threadIdx.x; t < G * RW; t += kTB) {
    pidx[t] = 0;
    pcode[t] = 0u;
  }
  for (int t = threadIdx.x; t < G * 3; t += kTB) ptgt[t] = 0.f;
  __syncthreads();  // s_pos, s_prev, s_u; zero fill before the scattered writes
  const unsigned *sc = a.scode + (size_t)cb * SB;
  for (int t = threadIdx.x; t < nb * R; t += kTB) {
    const int i = t / R, s = t - i * R;
    const int row = bidx[t];
    unsigned code = 0;
    if (row != 0) {
      code = sc[t];
      if (Mp) {
        const int j = bsearch_lds(s_prev, Mp, ((int)slot_is_edge(s, K) << 30) | row);
        if (j >= 0) code |= kSPend | ((unsigned)(2 + j) << kDefBits);
      }
    }
    pidx[s_pos[i] * RW + s] = row;
    pcode[s_pos[i] * RW + s] = code;
  }
  for (int t = threadIdx.x; t < nb * 3; t += kTB) {
    const int i = t / 3;
    ptgt[s_pos[i] * 3 + (t - 3 * i)] = btgt[t];
  }
  // flush entries, in the previous batch's entry order
  const int per = (Mp + kTB - 1) / kTB, j0 = threadIdx.x * per, j1 = min(j0 + per, Mp);
  int cf = 0;
  for (int j = j0; j < j1; j++) cf += bsearch_lds(s_u, U, s_prev[j]) < 0;
  int F = 0;
  int f = block_exclusive_scan(cf, &F, s_ws);
  const int cap = kFX * nb;
  for (int j = j0; j < j1; j++) {
    const int key = s_prev[j];
    if (bsearch_lds(s_u, U, key) >= 0) continue;
    if (f < cap) {
      const int p = f % nb, k = f / nb, g = (p % (G / RPB)) * RPB + p / (G / RPB);
      pidx[g * RW + R + k] = key & 0x3fffffff;
      pcode[g * RW + R + k] = ((key >> 30) ? kFEdge : 0u) | ((unsigned)(2 + j) << kDefBits);
    } else {
      a.pfo[(size_t)cb * a.Mmax + (f - cap)] = make_int2(key, 2 + j);
    }
    f++;
  }
  const int nfo = max(F - cap, 0);
  for (int g = threadIdx.x; g < G; g += kTB) {
    pidx[g * RW + R + kFX] = nfo;
    pidx[g * RW + R + kFX + 1] = Mpp;
  }
}

// One workgroup per batch of the chunk: sorted unique (table,row) keys of
// the non-padding slots and, per key, its slot ids in ascending order.
__global__ __launch_bounds__(kTB) void train_prep(TrainArgs a, int64_t base,
                                                  int nbc, int P, int *skey, int *sM) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_key[];
  __shared__ int s_ws[kTB / 64];
  const int cb = blockIdx.x;
  if (cb >= nbc) {  // graph nodes past the last batch find no work
    if (threadIdx.x == 0) a.bmeta[cb] = make_int2(0, 0);
    return;
  }
  // (diagnostic phase trace: the first chunk's workgroups in trace slot
  // [batch 0][kernel 1][cb], stamps: start, ids, slot gathers, sort, unique
  // runs, codes)
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g_trace) ts[0] = __builtin_amdgcn_s_memrealtime();
  const int64_t r0 = (base + cb) * a.B;
  const int nb = (int)min((int64_t)a.B, a.n - r0);
  if (threadIdx.x == 0) a.bmeta[cb] = make_int2(nb, (int)(base + cb));
  const int R = a.R, K = a.K;
  const int S = nb * R;
  int *bidx = a.bidx + (size_t)cb * a.B * R;
  float *btgt = a.btgt + (size_t)cb * a.B * 3;
  // the batch's record ids once into LDS, then every gather below has one
  // round trip; slot rows 8 per thread in flight before the stores
  // the batch's record ids, in the dynamic region behind the keys: where the
  // run classes go later (radix path: 16-bit classes, so 4 workgroups fit a
  // CU's LDS) or behind them (bitonic path)
  int *s_perm = reinterpret_cast<int *>(s_key + P) + (P == kSortP ? 0 : P);
  for (int i = threadIdx.x; i < nb; i += kTB) s_perm[i] = a.perm[r0 + i];
  __syncthreads();
  HGX_STAMP(ts[1]);
  for (int t = threadIdx.x; t < nb * 3; t += kTB) {
    const int i = t / 3;
    btgt[t] = a.tgt[(int64_t)s_perm[i] * 3 + (t - 3 * i)];
  }
  for (int t0 = threadIdx.x; t0 < P; t0 += 8 * kTB) {
    int rv[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int t = t0 + u * kTB, i = t / R;
      rv[u] = t < S ? a.idx[(int64_t)s_perm[i] * R + (t - i * R)] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int t = t0 + u * kTB;
      if (t >= P) break;
      unsigned long long key = ~0ull;
      if (t < S) {
        const int s = t % R, row = rv[u];
        bidx[t] = row;
        if (row != 0) {
          const unsigned k32 = ((unsigned)slot_is_edge(s, K) << 30) | (unsigned)row;
          key = ((unsigned long long)k32 << 32) | (unsigned)t;
        }
      }
      s_key[t] = key;
    }
  }
  __syncthreads();
  HGX_STAMP(ts[2]);
  constexpr int IPT = kSortP / kTB;
  unsigned kk[IPT];
  int vv[IPT];
  if (P == kSortP) {
    // the common batch (256 records x 14 slots): a block radix sort of the
    // 32-bit (table, row) keys with the slot as value, 8-bit digits, 4
    // passes, stable (equal keys keep slot order: the same order as the
    // 64-bit (key, slot) keys below); its storage aliases s_key. 4.5x faster
    // than the bitonic network (73 -> 16 us per batch).
    using BRS = rocprim::block_radix_sort<unsigned, kTB, kSortP / kTB, int>;
    static_assert(sizeof(typename BRS::storage_type) <= kSortP * 8 + kPrepB * 4,
                  "sort storage fits the radix path's dynamic LDS");
#pragma unroll
    for (int i = 0; i < IPT; i++) {
      const unsigned long long x = s_key[threadIdx.x * IPT + i];
      kk[i] = (unsigned)(x >> 32);  // padding: 0xffffffff, after every key
      vv[i] = (int)(unsigned)x;
    }
    __syncthreads();
    BRS().sort(kk, vv, *reinterpret_cast<typename BRS::storage_type *>(s_key));
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IPT; i++)
      s_key[threadIdx.x * IPT + i] =
          kk[i] == 0xffffffffu ? ~0ull : ((unsigned long long)kk[i] << 32) | (unsigned)vv[i];
    __syncthreads();
  } else {
    for (int size = 2; size <= P; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = threadIdx.x; t < P / 2; t += kTB) {
          const int lo = 2 * t - (t & (stride - 1));
          const int hi = lo + stride;
          const bool up = ((lo & size) == 0);
          const unsigned long long x = s_key[lo], y = s_key[hi];
          if ((x > y) == up) {
            s_key[lo] = y;
            s_key[hi] = x;
          }
        }
        __syncthreads();
      }
    }
  }
  HGX_STAMP(ts[3]);
  if (P == kSortP) {
    prep_runs_regs<IPT>(a, cb, P, kk, vv, s_key, s_ws,
                        reinterpret_cast<unsigned short *>(s_key + P), skey, sM);
    HGX_STAMP(ts[5]);
    ts[4] = ts[5];
    if (g_trace && base == 0) trace_put(0, 1, 6, ts);
    return;
  }
  // unique starts over a contiguous chunk per thread, then one block scan
  const int per = P / kTB;
  const int t0 = threadIdx.x * per;
  int cnt = 0, valid = 0;
  for (int t = t0; t < t0 + per; t++) {
    const unsigned long long x = s_key[t];
    if (x == ~0ull) break;
    valid++;
    if (t == 0 || (unsigned)(s_key[t - 1] >> 32) != (unsigned)(x >> 32)) cnt++;
  }
  int U = 0, V = 0;
  int u = block_exclusive_scan(cnt, &U, s_ws);
  const int u0 = u;
  block_exclusive_scan(valid, &V, s_ws);
  int *ukey = a.ukey + (size_t)cb * a.SB;
  int *uoff = a.uoff + (size_t)cb * (a.SB + 1);
  int *inv = a.inv + (size_t)cb * a.SB;
  // (slot positions and run offsets feed the two-kernel step only)
  const bool split = !a.fused;
  for (int t = t0; t < t0 + per; t++) {
    const unsigned long long x = s_key[t];
    if (x == ~0ull) break;
    if (split) inv[x & 0xffffffffu] = t;
    if (t == 0 || (unsigned)(s_key[t - 1] >> 32) != (unsigned)(x >> 32)) {
      ukey[u] = (int)(x >> 32);
      if (split) uoff[u] = t;
      u++;
    }
  }
  if (threadIdx.x == 0) {
    if (split) uoff[U] = V;
    a.ucount[cb] = U;
  }
  HGX_STAMP(ts[4]);
  if (a.fused)
    defer_codes(a, cb, V, P, u0, s_key, s_ws, reinterpret_cast<int *>(s_key + P), skey, sM);
  HGX_STAMP(ts[5]);
  if (g_trace && base == 0) trace_put(0, 1, 6, ts);
}

// deterministic two-level sum of the chunk's per-block losses:
// loss_partial (kLossBlocks blocks) then loss_final (one block)
constexpr int kLossBlocks = 256;
__global__ void loss_partial(const float *lossbuf, int64_t m, double *part) {
  __shared__ double s[kTB];
  double v = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)kTB + threadIdx.x; i < m;
       i += (int64_t)kLossBlocks * kTB)
    v += (double)lossbuf[i];
  s[threadIdx.x] = v;
  __syncthreads();
  for (int o = kTB / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}
__global__ void loss_final(const double *part, double *acc) {
  __shared__ double s[kLossBlocks];
  s[threadIdx.x] = part[threadIdx.x];
  __syncthreads();
  for (int o = kLossBlocks / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *acc += s[0];
}

// the identity order (records already in epoch order, ctx->rec_in_order)
__global__ void iota_perm(int64_t n, int *perm) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    perm[i] = (int)i;
}

__global__ void shuffle_keys(uint64_t seed, int epoch, int64_t n,
                             unsigned long long *keys, int *vals) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = hgx::rand64(seed, 0x5348554646ull + epoch, (uint64_t)i);
    vals[i] = (int)i;
  }
}

__global__ void max_index(const int *idx, int64_t n, int R, int K, int *out) {
  int mn = 0, me = 0, neg = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    const int *p = idx + r * R;
    for (int s = 0; s < R; s++) {
      const int v = p[s];
      neg |= v < 0;
      if (slot_is_edge(s, K)) me = max(me, v);
      else mn = max(mn, v);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mn = max(mn, __shfl_xor(mn, off));
    me = max(me, __shfl_xor(me, off));
    neg |= __shfl_xor(neg, off);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&out[0], mn);
    atomicMax(&out[1], me);
    atomicOr(&out[2], neg);
  }
}

__global__ void init_uniform(float *tab, int64_t rows, int d, int dp,
                             uint64_t seed, uint64_t stream) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < rows * dp; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % dp);
    float v = 0.f;
    if (c < d) {
      const uint64_t r = hgx::rand64(seed, stream, (uint64_t)i);
      v = -0.05f + 0.1f * (float)(r >> 40) * (1.0f / 16777216.0f);
    }
    tab[i] = v;
  }
}

__global__ void pad_rows(const float *src, float *dst, int64_t rows, int d,
                         int dp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < rows * dp; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / dp;
    const int c = (int)(i % dp);
    dst[i] = c < d ? src[r * d + c] : 0.f;
  }
}

__global__ void unpad_rows(const float *src, float *dst, int64_t rows, int d,
                           int dp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
       i < rows * d; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / d;
    const int c = (int)(i % d);
    dst[i] = src[r * dp + c];
  }
}

int grid_for(int64_t work, int per_block) {
  int64_t g = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 4096));
}

// lanes per record L (power of two <= 64) and float4 per lane VPL
void geometry(int d, int &L, int &VPL) {
  const int nv = (d + 3) / 4;
  L = 1;
  while (L < nv && L < 64) L *= 2;
  VPL = (nv + L - 1) / L;
  if (VPL == 3) VPL = 4;
}

using KFn = void (*)(TrainArgs, int);

int env_int(const char *name, int dflt) { return hgx_debug_env(name, dflt); }

template <int L, int VPL, int TB>
KFn fwd_spec(int K, int loss, int act) {
  if (K == 5 && loss == 0 && act == 0) return train_fwd_bwd<L, VPL, 5, true, 1, TB>;
  if (K == 5 && loss == 1 && act == 1) return train_fwd_bwd<L, VPL, 5, true, 2, TB>;
  return nullptr;
}

template <int L, int VPL>
KFn fwd_for(int K, int loss, int act, int tb1) {
  KFn f = tb1 == 512 ? fwd_spec<L, VPL, 512>(K, loss, act)
                     : fwd_spec<L, VPL, kTB>(K, loss, act);
  if (f) return f;
  if (K <= 2) return train_fwd_bwd<L, VPL, 2, false, 0, kTB>;
  if (K <= 5) return train_fwd_bwd<L, VPL, 5, false, 0, kTB>;
  if (K <= 8) return train_fwd_bwd<L, VPL, 8, false, 0, kTB>;
  return train_fwd_bwd<L, VPL, 16, false, 0, kTB>;
}

using KStepFn = void (*)(TrainArgs, int, int, int, int);
using KFlushFn = void (*)(TrainArgs, const int *, const int *, const int *, int, int);

// deferred-row step: d in (64, 256], K = 5 with the FOBE (sigmoid/KLD) or
// HOBE (relu/MSE) heads. One SL-lane group per record with VW floats per lane
// (dp = SL VW): float4 x 32 lanes or float2 x 64 lanes for dp = 128, float4 x
// 64 lanes for dp = 256. tb = the workgroup size (records per workgroup =
// tb / SL, ceil(batch / (tb / SL)) workgroups). The flush kernel views rows
// as float4.
template <int SL, int VW, int TB>
void step_fns(int loss, KStepFn *kf, KFlushFn &kfl) {
  kf[0] = loss == 0 ? train_step<SL, VW, 5, 1, TB, false>
                    : train_step<SL, VW, 5, 2, TB, false>;
  kf[1] = loss == 0 ? train_step<SL, VW, 5, 1, TB, true>
                    : train_step<SL, VW, 5, 2, TB, true>;
  kfl = train_flush<SL * VW / 4>;
}
// lanes = the tuning (0 auto, 32 or 64 lanes per record where dp = 128);
// sets sl (the step's lanes per record), tb and the kernels
bool pick_step(int L, int VPL, int K, int loss, int act, int lanes, int &sl,
               int &tb, KStepFn *kf, KFlushFn &kfl) {
  if (VPL != 1 || K != 5 || loss != act) return false;
  if (L != 32 && L != 64) return false;
  // dp = 128, measured r02 (tools/ab_train.py, interleaved, us per batch on
  // random / C3 HOBE records): float2 x 64 lanes at 256 threads 7.63 / 7.79;
  // float4 x 32 lanes at 128 threads 8.07 / 8.42 (8.33 / 8.75 at 256)
  const int vw = L == 32 && lanes != 32 ? 2 : 4;
  sl = L * 4 / vw;
  if (sl == 32) {
    tb = tb == 256 ? 256 : 128;
    if (tb == 128) step_fns<32, 4, 128>(loss, kf, kfl);
    else step_fns<32, 4, 256>(loss, kf, kfl);
  } else if (vw == 2) {
    tb = tb == 512 || tb == 128 ? tb : 256;
    if (tb == 512) step_fns<64, 2, 512>(loss, kf, kfl);
    else if (tb == 128) step_fns<64, 2, 128>(loss, kf, kfl);
    else step_fns<64, 2, 256>(loss, kf, kfl);
  } else {
    tb = 256;
    step_fns<64, 4, 256>(loss, kf, kfl);
  }
  return true;
}

bool pick_kernels(int L, int VPL, int K, int loss, int act, int &tb1, int tb2,
                  KFn &k1, KFn &k2) {
#define HGX_CASE(LL, VV)                                                     \
  if (L == LL && VPL == VV) {                                                \
    k1 = env_int("HGX_TRAIN_GENERIC", 0) == 1                                \
             ? train_fwd_bwd<LL, VV, 16, false, 0, kTB>                      \
             : fwd_for<LL, VV>(K, loss, act, tb1);                           \
    k2 = tb2 == 512 ? train_update<LL, VV, 512> : train_update<LL, VV, kTB>; \
    return true;                                                             \
  }
  HGX_CASE(1, 1) HGX_CASE(2, 1) HGX_CASE(4, 1) HGX_CASE(8, 1)
  HGX_CASE(16, 1) HGX_CASE(32, 1) HGX_CASE(64, 1) HGX_CASE(64, 2)
  HGX_CASE(64, 4)
#undef HGX_CASE
  return false;
}


}  // namespace

// ---------------------------------------------------------------------------
// records
// ---------------------------------------------------------------------------
extern "C" int hgx_records_set(hgx_ctx *ctx, int64_t n, int K,
                               const int32_t *idx, const float *tgt) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, n >= 0 && K >= 1 && K <= 16, HGX_EUNSUP,
            "num_neighbors K=%d outside [1,16]", K);
  HGX_CHECK(ctx, n == 0 || (idx && tgt), HGX_EINVAL, "null record buffer");
  const int R = 4 + 2 * K;
  for (int64_t i = 0; i < n * R; i++)
    HGX_CHECK(ctx, idx[i] >= 0, HGX_EINVAL, "negative record index");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, ctx->rec_idx, sizeof(int32_t) * (n * R + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->rec_tgt, sizeof(float) * (n * 3 + 1)));
  if (n) {
    HGX_HIP(ctx, hipMemcpyAsync(ctx->rec_idx.p, idx, sizeof(int32_t) * n * R,
                                hipMemcpyHostToDevice, ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->rec_tgt.p, tgt, sizeof(float) * n * 3,
                                hipMemcpyHostToDevice, ctx->stream));
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->n_rec = n;
  ctx->K = K;
  ctx->smp_family = -1;
  ctx->rec_in_order = false;
  ctx->store_carry = 0;  // no store batch tail survives a rewrite
  ctx->rec_bounds[0] = 0;
  ctx->rec_bounds[1] = n;
  ctx->n_rec_blocks = 1;
  return HGX_OK;
}

extern "C" int hgx_records_blocks(hgx_ctx *ctx, int *nblocks, int64_t *bounds) {
  if (!ctx) return HGX_EINVAL;
  if (nblocks) *nblocks = ctx->n_rec_blocks;
  if (bounds)
    for (int i = 0; i <= ctx->n_rec_blocks; i++) bounds[i] = ctx->rec_bounds[i];
  return HGX_OK;
}

extern "C" int hgx_records_export(hgx_ctx *ctx, void *d_idx, void *d_tgt) {
  if (!ctx) return HGX_EINVAL;
  const int64_t n = ctx->n_rec;
  const int R = 4 + 2 * ctx->K;
  if (n == 0) return HGX_OK;
  HGX_CHECK(ctx, d_idx || d_tgt, HGX_EINVAL, "null export buffer");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  if (d_idx)
    HGX_HIP(ctx, hipMemcpyAsync(d_idx, ctx->rec_idx.p, sizeof(int32_t) * n * R,
                                hipMemcpyDeviceToDevice, ctx->stream));
  if (d_tgt)
    HGX_HIP(ctx, hipMemcpyAsync(d_tgt, ctx->rec_tgt.p, sizeof(float) * n * 3,
                                hipMemcpyDeviceToDevice, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_records_import(hgx_ctx *ctx, int64_t n, int K,
                                  const void *d_idx, const void *d_tgt,
                                  int nblocks, const int64_t *bounds) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, n >= 0 && K >= 1 && K <= 16, HGX_EUNSUP,
            "num_neighbors K=%d outside [1,16]", K);
  HGX_CHECK(ctx, n == 0 || (d_idx && d_tgt), HGX_EINVAL, "null record buffer");
  HGX_CHECK(ctx, nblocks >= 0 && nblocks <= hgx_ctx::kMaxRecBlocks, HGX_EINVAL,
            "%d record blocks (at most %d)", nblocks, hgx_ctx::kMaxRecBlocks);
  if (nblocks > 0) {
    HGX_CHECK(ctx, bounds && bounds[0] == 0 && bounds[nblocks] == n, HGX_EINVAL,
              "block bounds must run from 0 to n");
    for (int i = 0; i < nblocks; i++)
      HGX_CHECK(ctx, bounds[i] <= bounds[i + 1], HGX_EINVAL,
                "block bounds not ascending");
  }
  const int R = 4 + 2 * K;
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_TRY(hgx_ensure(ctx, ctx->rec_idx, sizeof(int32_t) * (n * R + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->rec_tgt, sizeof(float) * (n * 3 + 1)));
  if (n) {
    HGX_HIP(ctx, hipMemcpyAsync(ctx->rec_idx.p, d_idx, sizeof(int32_t) * n * R,
                                hipMemcpyDeviceToDevice, ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->rec_tgt.p, d_tgt, sizeof(float) * n * 3,
                                hipMemcpyDeviceToDevice, ctx->stream));
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->n_rec = n;
  ctx->K = K;
  ctx->smp_family = -1;
  ctx->rec_in_order = false;
  ctx->store_carry = 0;  // no store batch tail survives a rewrite
  if (nblocks > 0) {
    for (int i = 0; i <= nblocks; i++) ctx->rec_bounds[i] = bounds[i];
    ctx->n_rec_blocks = nblocks;
  } else {
    ctx->rec_bounds[0] = 0;
    ctx->rec_bounds[1] = n;
    ctx->n_rec_blocks = 1;
  }
  return HGX_OK;
}

// The records of `src` (and their kind blocks) copied device to device into
// `dst` on the same device: the hand-over of a chunk sampled on one context
// (beside the training) to the training context.
extern "C" int hgx_records_copy(hgx_ctx *dst, hgx_ctx *src) {
  if (!dst || !src) return HGX_EINVAL;
  HGX_CHECK(dst, dst->device == src->device, HGX_EINVAL,
            "contexts on devices %d and %d", dst->device, src->device);
  HGX_HIP(dst, hipSetDevice(dst->device));
  HGX_HIP(dst, hipStreamSynchronize(src->stream));
  const int64_t n = src->n_rec;
  const int K = src->K, R = 4 + 2 * K;
  HGX_CHECK(dst, src->n_rec_blocks >= 0 && src->n_rec_blocks <= hgx_ctx::kMaxRecBlocks,
            HGX_EINVAL, "source has %d record blocks", src->n_rec_blocks);
  // the same one-element slack as every other record writer
  HGX_TRY(hgx_ensure(dst, dst->rec_idx, sizeof(int32_t) * (n * R + 1)));
  HGX_TRY(hgx_ensure(dst, dst->rec_tgt, sizeof(float) * (n * 3 + 1)));
  if (n > 0) {
    HGX_HIP(dst, hipMemcpyAsync(dst->rec_idx.p, src->rec_idx.p,
                                sizeof(int32_t) * n * R, hipMemcpyDeviceToDevice,
                                dst->stream));
    HGX_HIP(dst, hipMemcpyAsync(dst->rec_tgt.p, src->rec_tgt.p,
                                sizeof(float) * n * 3, hipMemcpyDeviceToDevice,
                                dst->stream));
  }
  HGX_HIP(dst, hipStreamSynchronize(dst->stream));
  dst->n_rec = n;
  dst->K = K;
  dst->smp_family = src->smp_family;
  dst->smp_seed = src->smp_seed;
  dst->rec_in_order = src->rec_in_order;
  dst->store_carry = 0;  // the tail (if any) stays with src's buffer
  dst->n_rec_blocks = src->n_rec_blocks;
  for (int i = 0; i <= src->n_rec_blocks; i++) dst->rec_bounds[i] = src->rec_bounds[i];
  return HGX_OK;
}

extern "C" int hgx_records_info(hgx_ctx *ctx, int64_t *n, int *K) {
  if (!ctx) return HGX_EINVAL;
  if (n) *n = ctx->n_rec;
  if (K) *K = ctx->K;
  return HGX_OK;
}

extern "C" int hgx_records_get(hgx_ctx *ctx, int32_t *idx, float *tgt) {
  if (!ctx) return HGX_EINVAL;
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int64_t n = ctx->n_rec;
  const int R = 4 + 2 * ctx->K;
  if (n == 0) return HGX_OK;
  if (idx)
    HGX_HIP(ctx, hipMemcpyAsync(idx, ctx->rec_idx.p, sizeof(int32_t) * n * R,
                                hipMemcpyDeviceToHost, ctx->stream));
  if (tgt)
    HGX_HIP(ctx, hipMemcpyAsync(tgt, ctx->rec_tgt.p, sizeof(float) * n * 3,
                                hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

// ---------------------------------------------------------------------------
// model
// ---------------------------------------------------------------------------
extern "C" int hgx_model_init(hgx_ctx *ctx, int d, int64_t node_rows,
                              int64_t edge_rows, uint64_t seed,
                              const float *node_tab, const float *edge_tab) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, d >= 1 && d <= 1024, HGX_EUNSUP, "dimension %d outside [1,1024]", d);
  HGX_CHECK(ctx, node_rows >= 1 && edge_rows >= 1 && node_rows < (1 << 30) &&
                     edge_rows < (1 << 30),
            HGX_EUNSUP, "table rows outside [1, 2^30)");
  HGX_CHECK(ctx, (node_tab == nullptr) == (edge_tab == nullptr), HGX_EINVAL,
            "give both initial tables or neither");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  int L, VPL;
  geometry(d, L, VPL);
  const int dp = 4 * L * VPL;
  ctx->d = d;
  ctx->dp = dp;
  ctx->node_rows = node_rows;
  ctx->edge_rows = edge_rows;
  const size_t nb = sizeof(float) * node_rows * dp, eb = sizeof(float) * edge_rows * dp;
  HGX_TRY(hgx_ensure(ctx, ctx->ntab, nb));
  HGX_TRY(hgx_ensure(ctx, ctx->etab, eb));
  HGX_TRY(hgx_ensure(ctx, ctx->nacc, nb));
  HGX_TRY(hgx_ensure(ctx, ctx->eacc, eb));
  HGX_HIP(ctx, hipMemsetAsync(ctx->nacc.p, 0, nb, ctx->stream));
  HGX_HIP(ctx, hipMemsetAsync(ctx->eacc.p, 0, eb, ctx->stream));
  if (node_tab) {
    const size_t hn = sizeof(float) * node_rows * d, he = sizeof(float) * edge_rows * d;
    HGX_TRY(hgx_ensure(ctx, ctx->s1, std::max(hn, he)));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->s1.p, node_tab, hn, hipMemcpyHostToDevice,
                                ctx->stream));
    hipLaunchKernelGGL(pad_rows, dim3(grid_for(node_rows * dp, 256)), dim3(256),
                       0, ctx->stream, ctx->s1.as<float>(), ctx->ntab.as<float>(),
                       node_rows, d, dp);
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->s1.p, edge_tab, he, hipMemcpyHostToDevice,
                                ctx->stream));
    hipLaunchKernelGGL(pad_rows, dim3(grid_for(edge_rows * dp, 256)), dim3(256),
                       0, ctx->stream, ctx->s1.as<float>(), ctx->etab.as<float>(),
                       edge_rows, d, dp);
  } else {
    hipLaunchKernelGGL(init_uniform, dim3(grid_for(node_rows * dp, 256)),
                       dim3(256), 0, ctx->stream, ctx->ntab.as<float>(),
                       node_rows, d, dp, seed, (uint64_t)1);
    hipLaunchKernelGGL(init_uniform, dim3(grid_for(edge_rows * dp, 256)),
                       dim3(256), 0, ctx->stream, ctx->etab.as<float>(),
                       edge_rows, d, dp, seed, (uint64_t)2);
  }
  HGX_LAUNCH_CHECK(ctx);
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_model_get(hgx_ctx *ctx, float *node_tab, float *edge_tab) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->d > 0, HGX_ESTATE, "no model on device");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int d = ctx->d, dp = ctx->dp;
  const size_t hn = sizeof(float) * ctx->node_rows * d;
  const size_t he = sizeof(float) * ctx->edge_rows * d;
  HGX_TRY(hgx_ensure(ctx, ctx->s1, std::max(hn, he)));
  if (node_tab) {
    hipLaunchKernelGGL(unpad_rows, dim3(grid_for(ctx->node_rows * d, 256)),
                       dim3(256), 0, ctx->stream, ctx->ntab.as<float>(),
                       ctx->s1.as<float>(), ctx->node_rows, d, dp);
    HGX_HIP(ctx, hipMemcpyAsync(node_tab, ctx->s1.p, hn, hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  if (edge_tab) {
    hipLaunchKernelGGL(unpad_rows, dim3(grid_for(ctx->edge_rows * d, 256)),
                       dim3(256), 0, ctx->stream, ctx->etab.as<float>(),
                       ctx->s1.as<float>(), ctx->edge_rows, d, dp);
    HGX_HIP(ctx, hipMemcpyAsync(edge_tab, ctx->s1.p, he, hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

__global__ void gather_rows(const float *__restrict__ src,
                            const int64_t *__restrict__ rows, float *dst,
                            int64_t n, int d, int dp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * d;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = i / d;
    dst[i] = src[rows[q] * dp + (int)(i % d)];
  }
}

extern "C" int hgx_model_get_rows(hgx_ctx *ctx, int table, int64_t n,
                                  const int64_t *rows, float *out) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->d > 0, HGX_ESTATE, "no model on device");
  HGX_CHECK(ctx, table == 0 || table == 1, HGX_EINVAL, "table must be 0 or 1");
  HGX_CHECK(ctx, n >= 0, HGX_EINVAL, "negative row count");
  if (n == 0) return HGX_OK;
  HGX_CHECK(ctx, rows && out, HGX_EINVAL, "null rows / out");
  const int64_t nr = table == 0 ? ctx->node_rows : ctx->edge_rows;
  for (int64_t q = 0; q < n; q++)
    HGX_CHECK(ctx, rows[q] >= 0 && rows[q] < nr, HGX_EINVAL,
              "row %lld outside the table (%lld rows)", (long long)rows[q],
              (long long)nr);
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int d = ctx->d;
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(int64_t) * n));
  HGX_TRY(hgx_ensure(ctx, ctx->s1, sizeof(float) * n * d));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->s2.p, rows, sizeof(int64_t) * n,
                              hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(gather_rows, dim3(grid_for(n * d, 256)), dim3(256), 0,
                     ctx->stream, (table == 0 ? ctx->ntab : ctx->etab).as<float>(),
                     ctx->s2.as<int64_t>(), ctx->s1.as<float>(), n, d, ctx->dp);
  HGX_LAUNCH_CHECK(ctx);
  HGX_HIP(ctx, hipMemcpyAsync(out, ctx->s1.p, sizeof(float) * n * d,
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

// ---------------------------------------------------------------------------
// fit
// ---------------------------------------------------------------------------
// The two streams of the overlapped chunk preparation (tuning
// train_prep_overlap): tstream[0] the batch steps, tstream[1] the
// preparation. With cus > 0 they get disjoint CU masks: the first `cus`
// CU-mask bits (rounded up to a multiple of 8) for the preparation, the rest
// for the steps (which use 64 workgroups per batch): a preparation workgroup
// never shares a CU with a batch step. Mask bit i is CU i / 8 of XCD i % 8
// (probed on MI355X, tools/cumask_probe.hip); a mask that leaves an XCD
// without CUs is ignored by the runtime (the whole device), so each side
// keeps CUs on every XCD.
static int train_streams(hgx_ctx *ctx, int cus) {
  if (ctx->tstream_cus == cus && ctx->tstream[0]) return HGX_OK;
  for (hipStream_t &s : ctx->tstream) {
    if (s) {
      HGX_HIP(ctx, hipStreamSynchronize(s));
      HGX_HIP(ctx, hipStreamDestroy(s));
      s = nullptr;
    }
  }
  ctx->tstream_cus = -1;
  if (cus <= 0) {
    for (hipStream_t &s : ctx->tstream)
      HGX_HIP(ctx, hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  } else {
    int ncu = 0;
    HGX_HIP(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount,
                                       ctx->device));
    HGX_CHECK(ctx, cus <= ncu / 2, HGX_EINVAL, "train_prep_cus %d above half of %d CUs",
              cus, ncu);
    const int W = (ncu + 31) / 32;
    std::vector<uint32_t> ms(W, 0u), mp(W, 0u);
    const int np = (cus + 7) / 8 * 8;
    for (int i = 0; i < ncu; i++) (i < np ? mp : ms)[i / 32] |= 1u << (i % 32);
    HGX_HIP(ctx, hipExtStreamCreateWithCUMask(&ctx->tstream[0], W, ms.data()));
    HGX_HIP(ctx, hipExtStreamCreateWithCUMask(&ctx->tstream[1], W, mp.data()));
  }
  ctx->tstream_cus = cus;
  return HGX_OK;
}

extern "C" int hgx_train(hgx_ctx *ctx, int batch, int max_epochs, float lr,
                         float eps, int loss, int act, float min_delta,
                         uint64_t shuffle_seed, const int64_t *perms,
                         float *epoch_loss, int *epochs_run) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->d > 0, HGX_ESTATE, "hgx_model_init not called");
  HGX_CHECK(ctx, ctx->n_rec > 0, HGX_ESTATE, "no records on device");
  HGX_CHECK(ctx, batch >= 1, HGX_EINVAL, "batch_size must be >= 1");
  HGX_CHECK(ctx, max_epochs >= 0, HGX_EINVAL, "epochs must be >= 0");
  HGX_CHECK(ctx, loss == 0 || loss == 1, HGX_EINVAL, "loss must be 0 or 1");
  HGX_CHECK(ctx, act == 0 || act == 1, HGX_EINVAL, "act must be 0 or 1");
  HGX_CHECK(ctx, ctx->n_rec < (int64_t)INT32_MAX, HGX_EUNSUP,
            "more than 2^31 records");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int64_t n = ctx->n_rec;
  const int K = ctx->K, R = 4 + 2 * K, dp = ctx->dp;
  const int SB = batch * R;
  int P = 1;
  while (P < SB) P <<= 1;
  P = std::max(P, kTB);
  HGX_CHECK(ctx, (size_t)P * 8 <= 64 * 1024, HGX_EUNSUP,
            "batch_size*(4+2K)=%d exceeds the 8192-slot batch limit", SB);

  // indices must fit the tables (kernels do not bounds-check)
  HGX_TRY(hgx_ensure(ctx, ctx->s0, 16));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s0.p, 0, 16, ctx->stream));
  hipLaunchKernelGGL(max_index, dim3(grid_for(n, 256)), dim3(256), 0,
                     ctx->stream, ctx->rec_idx.as<int>(), n, R, K,
                     ctx->s0.as<int>());
  HGX_LAUNCH_CHECK(ctx);
  int mx[4] = {0, 0, 0, 0};
  HGX_HIP(ctx, hipMemcpyAsync(mx, ctx->s0.p, 16, hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  HGX_CHECK(ctx, mx[2] == 0, HGX_EINVAL, "negative record index");
  HGX_CHECK(ctx, mx[0] < ctx->node_rows && mx[1] < ctx->edge_rows, HGX_EINVAL,
            "record index (node %d, edge %d) outside the tables (%lld, %lld)",
            mx[0], mx[1], (long long)ctx->node_rows, (long long)ctx->edge_rows);

  int L, VPL;
  geometry(ctx->d, L, VPL);
  // K1 workgroup size: 8 records per workgroup measured best (d=128: 256
  // threads, 10.5 us/batch vs 11.0 at 128 / 12.8 at 64 / 10.9 at 512;
  // d=256: 512 threads, 13.6 vs 14.7 at 256). Specialised FOBE/HOBE
  // kernels only; HGX_TRAIN_TB1=256|512 overrides.
  int tb1 = env_int("HGX_TRAIN_TB1", L >= 64 ? 512 : kTB);
  if (tb1 != 512) tb1 = kTB;
  if (!(K == 5 && loss == act) || env_int("HGX_TRAIN_GENERIC", 0) == 1) tb1 = kTB;
  // K2 workgroup size: 512 threads measured best (d=128: 10.2 vs 10.6
  // us/batch at 256 and 10.5 at 1024; d=256: 12.6 vs 13.5 / 12.7)
  int tb2 = env_int("HGX_TRAIN_TB2", 512);
  if (tb2 != 512) tb2 = kTB;
  KFn k1 = nullptr, k2 = nullptr;
  HGX_CHECK(ctx, pick_kernels(L, VPL, K, loss, act, tb1, tb2, k1, k2), HGX_EUNSUP,
            "no kernel for d=%d", ctx->d);
#ifdef HGX_DEBUG_KNOBS
  {
    const int ab = env_int("HGX_TRAIN_ABLATE", 0);
    HGX_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_tab), &ab, sizeof(int)));
  }
#endif
  const char *trace_path = hgx_debug_env_str("HGX_TRAIN_TRACE");
  const int trace_nb = 256;
  struct TraceBuf {
    void *p = nullptr;
    ~TraceBuf() {
      if (p) {
#ifdef HGX_DEBUG_KNOBS
        unsigned long long *z = nullptr;
        hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &z, sizeof(z));
#endif
        hipFree(p);
      }
    }
  } tb;
  const size_t trace_bytes = sizeof(unsigned long long) * trace_nb * 2 * 1024 * 8;
  {
    unsigned long long *tp = nullptr;
    int tn = 0;
    if (trace_path && trace_path[0]) {
      HGX_HIP(ctx, hipMalloc(&tb.p, trace_bytes));
      HGX_HIP(ctx, hipMemset(tb.p, 0, trace_bytes));
      tp = (unsigned long long *)tb.p;
      tn = trace_nb;
    }
#ifdef HGX_DEBUG_KNOBS
    HGX_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &tp, sizeof(tp)));
    HGX_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_trace_nb), &tn, sizeof(tn)));
#else
    (void)tp;
    (void)tn;
#endif
  }
  const int RPB = tb1 / L;
  const int nblk1 = (batch + RPB - 1) / RPB;
  // deferred-row step: eligible geometry and batch <= kPackB records (every
  // batch of the run then takes it); else the two-kernel step for every batch
  KStepFn kf[2] = {nullptr, nullptr};  // light / MULTI pending-slot forms
  KFlushFn kfl = nullptr;
  int tbf = ctx->tune.train_tb;  // workgroup size (0: per geometry)
  int SL = 0;
  const bool fused = ctx->tune.train_fused && env_int("HGX_TRAIN_GENERIC", 0) != 1 &&
                     batch <= kPackB &&
                     pick_step(L, VPL, K, loss, act, ctx->tune.train_lanes, SL, tbf,
                               kf, kfl);
  const int prpb = fused ? tbf / SL : 0;
  const int NBF = fused ? (batch + prpb - 1) / prpb : 0;
  const int RW = R + kWX;
  const int Mmax = SB / 2 + 1;        // deferred rows per batch: <= SB / 2
  const int MX = fused ? 2 + Mmax : 0;
  HGX_CHECK(ctx, MX <= (int)kDefMask + 1, HGX_EUNSUP, "batch too large for the step");
  // (early row-0 form: one loss word per record group, float2 rows)
  const bool r0e = HGX_TRAIN_R0EARLY && fused && ctx->dp == 2 * SL;
  const int lstride = std::max(nblk1, r0e ? NBF * prpb : NBF);
  const int GPB2 = tb2 / L;
  // one unique-row task per group, plus the two padding-row workgroups
  const int grid2 = (SB + GPB2 - 1) / GPB2 + 2;
  const int64_t nbatches = (n + batch - 1) / batch;
  const int GB = kGraphBatches;
  // prep chunk: CB batches (a multiple of GB) prepared by one launch, then
  // trained (two-kernel step: by CB / GB graph replays when HGX_GRAPH=1)
  const int CB = (int)std::min<int64_t>(1024, (nbatches + GB - 1) / GB * GB);
  const int NG = CB / GB;
  const int64_t nchunks = (nbatches + CB - 1) / CB;

  // record copies padded so K1's unconditional id loads stay in bounds
  const size_t bidx_n = (size_t)CB * batch * R + (size_t)RPB * R * 2 + 64;
  const size_t btgt_n = (size_t)CB * batch * 3 + (size_t)RPB * 3 * 2 + 64;
  const size_t inv_n = (size_t)CB * SB + (size_t)RPB * R * 2 + 64;
  const size_t pg = fused ? (size_t)CB * NBF * prpb : 0;  // placed groups
  // step buffers: pfo, pidx, pcode, ptgt, scode, skey [2], sM [2], pbrk
  // (with the overlapped preparation the placed buffers pfo, pidx, pcode,
  // ptgt, pbrk twice: chunk c + 1 is placed while chunk c trains)
  const bool overlap = fused && ctx->tune.train_prep_overlap >= 1;
  const bool ahead = overlap && ctx->tune.train_prep_overlap == 2;  // one stream
  const size_t placed_ints = 2 * (size_t)CB * Mmax + pg * RW * 2 + pg * 3 + (size_t)CB + 2;
  const size_t step_ints = fused ? 2 * (size_t)CB * Mmax + pg * RW * 2 + pg * 3 +
                                       (size_t)CB * SB + 2 * (size_t)CB * Mmax +
                                       3 * (size_t)CB + 64 + (overlap ? placed_ints : 0)
                                 : 0;
  const size_t prep_ints = bidx_n + btgt_n + inv_n + (size_t)CB * SB +
                           (size_t)CB * (SB + 1) + CB + 2 * CB + 64 + step_ints;
  HGX_TRY(hgx_ensure(ctx, ctx->s1, sizeof(int) * (n + 1)));              // perm
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(float) * (size_t)SB * dp));    // gslot
  // gzero (K1 partials) | gacc [3][MX][dp] int64 | shadow [3][MX][2][dp] |
  // r0acc [3][kR0Slots][2][dp] int64 | ovf
  const size_t gz_f = (size_t)nblk1 * 2 * dp;
  const size_t gacc_f = (size_t)3 * MX * dp * 2;  // in floats
  const size_t sh_f = (size_t)3 * MX * 2 * dp;
  const size_t gp_f = (size_t)3 * kR0Slots * 2 * dp * 2;  // r0acc (int64)
  const size_t s3_f = (gz_f + 3) / 4 * 4 + gacc_f + sh_f + gp_f + 16;
  HGX_TRY(hgx_ensure(ctx, ctx->s3, sizeof(float) * s3_f));
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * (size_t)nbatches * lstride + 16));
  const bool use_graph = env_int("HGX_GRAPH", 0) == 1 && !fused;
  HGX_TRY(hgx_ensure(ctx, ctx->s5, sizeof(int) * prep_ints));
  HGX_TRY(hgx_ensure(ctx, ctx->s6, 64 + sizeof(double) * kLossBlocks));  // loss
  int *perm = ctx->s1.as<int>();
  HGX_HIP(ctx, hipMemsetAsync(ctx->s5.p, 0, sizeof(int) * prep_ints, ctx->stream));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s3.p, 0, sizeof(float) * s3_f, ctx->stream));
  TrainArgs a;
  memset(&a, 0, sizeof(a));
  a.idx = ctx->rec_idx.as<int>();
  a.tgt = ctx->rec_tgt.as<float>();
  a.perm = perm;
  a.n = n;
  a.B = batch;
  a.R = R;
  a.K = K;
  a.dp = dp;
  a.ntab = ctx->ntab.as<float>();
  a.etab = ctx->etab.as<float>();
  a.nacc = ctx->nacc.as<float>();
  a.eacc = ctx->eacc.as<float>();
  a.gslot = ctx->s2.as<float>();
  a.gzero = ctx->s3.as<float>();
  a.lossbuf = ctx->s4.as<float>();
  a.SB = SB;
  a.nblk1 = nblk1;
  a.lstride = lstride;
  a.fused = fused ? 1 : 0;
  a.prpb = prpb;
  a.RW = RW;
  a.MX = MX;
  a.Mmax = Mmax;
  {
    float *f = a.gzero + (gz_f + 3) / 4 * 4;
    a.gacc = reinterpret_cast<long long *>(f);
    f += gacc_f;
    a.shadow = f;
    f += sh_f;
    a.r0acc = reinterpret_cast<long long *>(f);
    f += gp_f;
    a.ovf = reinterpret_cast<int *>(f);
  }
  a.lr = lr;
  a.eps = eps;
  a.loss = loss;
  a.act = act;
  int *skey[2] = {nullptr, nullptr}, *sM[2] = {nullptr, nullptr};
  {
    int *q = ctx->s5.as<int>();
    a.bidx = q;
    q += bidx_n;
    a.btgt = reinterpret_cast<float *>(q);
    q += btgt_n;
    a.inv = q;
    q += inv_n;
    a.ukey = q;
    q += (size_t)CB * SB;
    a.uoff = q;
    q += (size_t)CB * (SB + 1);
    a.ucount = q;
    q += CB;
    q += ((uintptr_t)q / sizeof(int)) % 2;  // 8-B align
    a.bmeta = reinterpret_cast<int2 *>(q);
    q += 2 * CB;
    if (fused) {
      a.pfo = reinterpret_cast<int2 *>(q);
      q += 2 * (size_t)CB * Mmax;
      a.pidx = q;
      q += pg * RW;
      a.pcode = reinterpret_cast<unsigned *>(q);
      q += pg * RW;
      a.ptgt = reinterpret_cast<float *>(q);
      q += pg * 3;
      a.scode = reinterpret_cast<unsigned *>(q);
      q += (size_t)CB * SB;
      for (int i = 0; i < 2; i++) {
        skey[i] = q;
        q += (size_t)CB * Mmax;
        sM[i] = q;
        q += CB;
      }
      a.pbrk = q;
      q += CB;
    }
  }
  // placed-buffer sets by chunk parity (one set unless overlapped)
  TrainArgs ap[2] = {a, a};
  if (overlap) {
    int *q = ap[0].pbrk + CB;
    q += ((uintptr_t)q / sizeof(int)) % 2;  // 8-B align (pfo)
    ap[1].pfo = reinterpret_cast<int2 *>(q);
    q += 2 * (size_t)CB * Mmax;
    ap[1].pidx = q;
    q += pg * RW;
    ap[1].pcode = reinterpret_cast<unsigned *>(q);
    q += pg * RW;
    ap[1].ptgt = reinterpret_cast<float *>(q);
    q += pg * 3;
    ap[1].pbrk = q;
  }
  double *dloss = reinterpret_cast<double *>(ctx->s6.as<char>() + 32);
  double *dpart = reinterpret_cast<double *>(ctx->s6.as<char>() + 64);

  // records loaded by hgx_store_load: trained in the order they were
  // written (the store drew the epoch's global permutation)
  const bool in_order = !perms && ctx->rec_in_order;
  // shuffle scratch (device shuffle only)
  size_t sort_tmp = 0, sort_off = 0;
  unsigned long long *keys_in = nullptr, *keys_out = nullptr;
  int *vals_in = nullptr;
  if (!perms && !in_order) {
    HGX_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, keys_in,
                                                    keys_out, vals_in, perm, (int)n));
    sort_off = (sizeof(unsigned long long) * 2 * n + sizeof(int) * n + 255) / 256 * 256;
    HGX_TRY(hgx_ensure(ctx, ctx->s7, sort_off + sort_tmp + 256));
    char *base = ctx->s7.as<char>();
    keys_in = reinterpret_cast<unsigned long long *>(base);
    keys_out = keys_in + n;
    vals_in = reinterpret_cast<int *>(keys_out + n);
  }

  // graphs and events, released on every exit path
  struct Res {
    std::vector<hipGraph_t> graph;
    std::vector<hipGraphExec_t> gexec;
    std::vector<hipEvent_t> ev;
    ~Res() {
      for (auto g : gexec) (void)hipGraphExecDestroy(g);
      for (auto g : graph) (void)hipGraphDestroy(g);
      for (auto e : ev) (void)hipEventDestroy(e);
      if (hbrk) (void)hipHostFree(hbrk);
    }
    int *hbrk = nullptr;  // pinned: the chunk's MULTI flags (train_place)
  } res;
  if (fused)
    HGX_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&res.hbrk),
                               sizeof(int) * CB * (overlap ? 2 : 1)));
  // overlapped preparation: the batch-step stream and the preparation stream
  // (disjoint CU masks when train_prep_cus > 0), ordered after everything
  // queued on ctx->stream so far and joined back into it at the end
  hipStream_t sst = ctx->stream, spr = ctx->stream;
  if (overlap && !ahead) {
    HGX_TRY(train_streams(ctx, ctx->tune.train_prep_cus));
    sst = ctx->tstream[0];
    spr = ctx->tstream[1];
  }
  // Direct launches by default: measured as fast as hipGraph replay of the
  // same kernels (10.6 us per batch both ways at d=128) with less host time,
  // and rocprofv3 kernel tracing crashes on the replays. HGX_GRAPH=1 replays
  // captured graphs of the two-kernel step instead.
  auto launch_run = [&](const TrainArgs &ac, int cb0, int nrun) {
    for (int b = cb0; b < cb0 + nrun; b++) {
      hipLaunchKernelGGL(k1, dim3(nblk1), dim3(tb1), 0, ctx->stream, ac, b);
      hipLaunchKernelGGL(k2, dim3(grid2), dim3(tb2), 0, ctx->stream, ac, b);
    }
  };
  if (use_graph) {
    for (int g = 0; g < NG; g++) {
      hipGraph_t gr = nullptr;
      hipGraphExec_t ge = nullptr;
      HGX_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed));
      launch_run(a, g * GB, GB);
      hipError_t ce = hipStreamEndCapture(ctx->stream, &gr);
      if (ce != hipSuccess)
        return hgx_fail(ctx, HGX_EHIP, "graph capture failed: %s", hipGetErrorString(ce));
      res.graph.push_back(gr);
      ce = hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
      if (ce != hipSuccess)
        return hgx_fail(ctx, HGX_EHIP, "graph instantiate failed: %s", hipGetErrorString(ce));
      res.gexec.push_back(ge);
    }
  }
  // one event pair per prep chunk: device time of the batch kernels only
  std::vector<hipEvent_t> bev(2 * nchunks);
  for (auto &e : bev) {
    HGX_HIP(ctx, hipEventCreate(&e));
    res.ev.push_back(e);
  }
  // overlapped preparation: chunk c prepared (pev[c]), the epoch's join
  // with ctx->stream (pev[nchunks]); timing off
  std::vector<hipEvent_t> pev(overlap ? nchunks + 1 : 0);
  for (auto &e : pev) {
    HGX_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    res.ev.push_back(e);
  }
  // train_prep's dynamic LDS: keys + run classes + record ids (radix path:
  // the ids and the 16-bit classes share one region)
  const size_t prep_smem =
      P == kSortP ? ((size_t)P * 8 + std::max<size_t>(kPrepB * 4, (size_t)SB * 2) + 15) / 16 * 16
                  : (size_t)P * 12 + kPrepB * 4;
  const size_t place_smem = sizeof(int) * ((size_t)Mmax + SB);
  // Preparation of chunk c (same stream, right before its batches: the
  // records it writes are still in the Infinity Cache when they are read).
  // The step: one launch per batch, q = the batch's index in the epoch.
  auto prep_chunk = [&](int64_t c, int nbc) {
    const int cp = (int)(c & 1);
    hipLaunchKernelGGL(train_prep, dim3(CB), dim3(kTB), prep_smem, ctx->stream, a,
                       c * CB, nbc, P, skey[cp], sM[cp]);
    if (fused)
      hipLaunchKernelGGL(train_place, dim3(CB), dim3(kTB), place_smem, ctx->stream, a,
                         nbc, CB, skey[cp], sM[cp], skey[cp ^ 1], sM[cp ^ 1], c > 0 ? 1 : 0);
  };

  std::vector<int> hperm;
  int64_t nfused = 0, nsplit = 0, nmulti = 0;
  double batch_ms = 0.0;
  double best = INFINITY;
  int ep = 0;
  int rc = HGX_OK;
  HGX_HIP(ctx, hipEventRecord(ctx->ev0, ctx->stream));
  for (ep = 0; ep < max_epochs; ep++) {
    if (perms) {
      hperm.resize(n);
      const int64_t *pe = perms + (int64_t)ep * n;
      for (int64_t i = 0; i < n; i++) {
        if (pe[i] < 0 || pe[i] >= n) {
          rc = hgx_fail(ctx, HGX_EINVAL, "permutation entry out of range");
          break;
        }
        hperm[i] = (int)pe[i];
      }
      if (rc) break;
      if (hipMemcpyAsync(perm, hperm.data(), sizeof(int) * n,
                         hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
          hipStreamSynchronize(ctx->stream) != hipSuccess) {
        rc = hgx_fail(ctx, HGX_EHIP, "permutation upload failed");
        break;
      }
    } else if (in_order) {
      hipLaunchKernelGGL(iota_perm, dim3(grid_for(n, 256)), dim3(256), 0,
                         ctx->stream, n, perm);
    } else {
      hipLaunchKernelGGL(shuffle_keys, dim3(grid_for(n, 256)), dim3(256), 0,
                         ctx->stream, shuffle_seed, ep, n, keys_in, vals_in);
      size_t tmp = sort_tmp;
      if (hipcub::DeviceRadixSort::SortPairs(
              ctx->s7.as<char>() + sort_off,
              tmp, keys_in, keys_out, vals_in, perm, (int)n, 0, 64,
              ctx->stream) != hipSuccess) {
        rc = hgx_fail(ctx, HGX_EHIP, "shuffle sort failed");
        break;
      }
    }
    (void)hipMemsetAsync(dloss, 0, sizeof(double), ctx->stream);
    (void)hipMemsetAsync(a.lossbuf, 0, sizeof(float) * (size_t)nbatches * lstride,
                         ctx->stream);
    // row-0 slots start at zero every epoch (then each batch zeroes the set
    // the next one adds into)
    if (fused)
      (void)hipMemsetAsync(a.r0acc, 0, sizeof(float) * gp_f, ctx->stream);
    int last_nbc = 0;
    if (overlap) {
      // chunk c + 1 prepared on spr while chunk c trains on sst; placed set
      // c & 1 is rewritten (chunk c + 2) only after chunk c's steps are done
      if (!ahead) {
        hipEvent_t ej = pev[nchunks];
        (void)hipEventRecord(ej, ctx->stream);
        (void)hipStreamWaitEvent(sst, ej, 0);
        (void)hipStreamWaitEvent(spr, ej, 0);
      }
      // The host enqueues chunk c + 1's preparation only once chunk c - 1's
      // steps are done (it waits for them after queueing chunk c's), so the
      // preparation stream never holds a barrier packet blocked on the step
      // stream.
      auto prep_ov = [&](int64_t c) {
        const int nbc = (int)std::min<int64_t>(CB, nbatches - c * CB);
        const int cp = (int)(c & 1);
        hipLaunchKernelGGL(train_prep, dim3(CB), dim3(kTB), prep_smem, spr, a, c * CB, nbc, P,
                           skey[cp], sM[cp]);
        hipLaunchKernelGGL(train_place, dim3(CB), dim3(kTB), place_smem, spr, ap[cp], nbc, CB,
                           skey[cp], sM[cp], skey[cp ^ 1], sM[cp ^ 1], c > 0 ? 1 : 0);
        (void)hipMemcpyAsync(res.hbrk + (size_t)cp * CB, ap[cp].pbrk, sizeof(int) * nbc,
                             hipMemcpyDeviceToHost, spr);
        (void)hipEventRecord(pev[c], spr);
      };
      prep_ov(0);
      for (int64_t c = 0; c < nchunks; c++) {
        const int64_t base = c * CB;
        const int nbc = (int)std::min<int64_t>(CB, nbatches - base);
        const int cp = (int)(c & 1);
        // one stream: chunk c + 1's preparation queued ahead of chunk c's
        // batches (stream order protects placed set (c + 1) & 1, last read
        // by chunk c - 1's batches, queued before it)
        if (ahead && c + 1 < nchunks) prep_ov(c + 1);
        if (hipEventSynchronize(pev[c]) != hipSuccess) {
          rc = hgx_fail(ctx, HGX_EHIP, "batch preparation failed: %s",
                        hipGetErrorString(hipGetLastError()));
          break;
        }
        if (!ahead) (void)hipStreamWaitEvent(sst, pev[c], 0);
        (void)hipEventRecord(bev[2 * c], sst);
        const int *hb = res.hbrk + (size_t)cp * CB;
        for (int b = 0; b < nbc; b++) {
          const int64_t gbat = base + b;
          const int nrec = (int)std::min<int64_t>(batch, n - gbat * batch);
          const int multi = hb[b] && gbat > 0;
          nmulti += multi;
          hipLaunchKernelGGL(kf[multi], dim3(NBF), dim3(tbf), 0, sst, ap[cp], b, (int)gbat,
                             nrec, (int)gbat);
        }
        nfused += nbc;
        (void)hipEventRecord(bev[2 * c + 1], sst);
        last_nbc = nbc;
        if (!ahead && c + 1 < nchunks) {
          // placed set (c + 1) & 1 is free once chunk c - 1's steps are done
          if (c >= 1 && hipEventSynchronize(bev[2 * (c - 1) + 1]) != hipSuccess) {
            rc = hgx_fail(ctx, HGX_EHIP, "batch step failed: %s",
                          hipGetErrorString(hipGetLastError()));
            break;
          }
          prep_ov(c + 1);
        }
      }
    }
    for (int64_t c = 0; c < nchunks && !overlap; c++) {
      const int64_t base = c * CB;
      const int nbc = (int)std::min<int64_t>(CB, nbatches - base);
      prep_chunk(c, nbc);
      if (fused) {
        // the chunk's MULTI flags: one host wait per chunk of 1024 batches
        if (hipMemcpyAsync(res.hbrk, a.pbrk, sizeof(int) * nbc, hipMemcpyDeviceToHost,
                           ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess) {
          rc = hgx_fail(ctx, HGX_EHIP, "batch preparation failed: %s",
                        hipGetErrorString(hipGetLastError()));
          break;
        }
      }
      (void)hipEventRecord(bev[2 * c], ctx->stream);
      if (fused) {
        const int cp = (int)(c & 1);
        for (int b = 0; b < nbc; b++) {
          const int64_t gbat = base + b;
          const int nrec = (int)std::min<int64_t>(batch, n - gbat * batch);
          const int multi = res.hbrk[b] && gbat > 0;
          nmulti += multi;
          hipLaunchKernelGGL(kf[multi], dim3(NBF), dim3(tbf), 0, ctx->stream, a, b, (int)gbat,
                             nrec, (int)gbat);
        }
        nfused += nbc;
      } else if (use_graph) {
        for (int g = 0; g * GB < nbc; g++) {
          if (hipGraphLaunch(res.gexec[g], ctx->stream) != hipSuccess) {
            rc = hgx_fail(ctx, HGX_EHIP, "graph launch failed");
            break;
          }
        }
        nsplit += nbc;
      } else {
        launch_run(a, 0, nbc);
        nsplit += nbc;
      }
      (void)hipEventRecord(bev[2 * c + 1], ctx->stream);
      last_nbc = nbc;
      if (rc) break;
    }
    if (rc) break;
    if (fused) {
      // the last batch's deferred rows -> tables; gacc clean for the next
      // epoch (the last batch's entries and the one before it)
      const int cp = (int)((nchunks - 1) & 1);
      const int *ml = sM[cp] + (last_nbc - 1);
      const int *mp = last_nbc >= 2 ? sM[cp] + (last_nbc - 2)
                                    : (nchunks >= 2 ? sM[cp ^ 1] + (CB - 1) : nullptr);
      const int nlast = (int)(n - (nbatches - 1) * batch);
      hipLaunchKernelGGL(kfl, dim3(64), dim3(256), 0, sst, a,
                         skey[cp] + (size_t)(last_nbc - 1) * Mmax, ml, mp,
                         (int)(nbatches - 1), std::min(NBF, nlast));
    }
    hipLaunchKernelGGL(loss_partial, dim3(kLossBlocks), dim3(kTB), 0,
                       sst, a.lossbuf, nbatches * lstride, dpart);
    hipLaunchKernelGGL(loss_final, dim3(1), dim3(kLossBlocks), 0, sst,
                       dpart, dloss);
    double lsum = 0.0;
    int ovf = 0;
    if (hipMemcpyAsync(&lsum, dloss, sizeof(double), hipMemcpyDeviceToHost,
                       sst) != hipSuccess ||
        (fused && hipMemcpyAsync(&ovf, a.ovf, sizeof(int), hipMemcpyDeviceToHost,
                                 sst) != hipSuccess) ||
        hipStreamSynchronize(sst) != hipSuccess) {
      rc = hgx_fail(ctx, HGX_EHIP, "epoch failed: %s",
                    hipGetErrorString(hipGetLastError()));
      break;
    }
    if (ovf) {
      rc = hgx_fail(ctx, HGX_ENUMERIC,
                    "a gradient left the step's fixed-point range (|g| >= %g after "
                    "the 1/batch factor, or NaN): training diverged",
                    (double)kFixLimit);
      break;
    }
    for (int64_t c = 0; c < nchunks; c++) {
      float m = 0.f;
      if (hipEventElapsedTime(&m, bev[2 * c], bev[2 * c + 1]) == hipSuccess)
        batch_ms += m;
    }
    const double cur = lsum / (double)n;
    ctx->train_loss_sum = lsum;
    if (epoch_loss) epoch_loss[ep] = (float)cur;
    if (cur < best - (double)min_delta) {
      best = cur;
    } else {
      ep++;
      break;
    }
  }
  if (overlap) {
    // join: nothing of this call is left running on the side streams
    (void)hipStreamSynchronize(spr);
    (void)hipStreamSynchronize(sst);
  }
  hipEventRecord(ctx->ev1, ctx->stream);
  hipEventSynchronize(ctx->ev1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  if (tb.p && rc == HGX_OK) {
    std::vector<unsigned long long> h(trace_bytes / 8);
    if (hipMemcpy(h.data(), tb.p, trace_bytes, hipMemcpyDeviceToHost) == hipSuccess) {
      if (FILE *f = fopen(trace_path, "wb")) {
        fwrite(h.data(), 1, trace_bytes, f);
        fclose(f);
      }
    }
  }
  if (rc) return rc;
  HGX_LAUNCH_CHECK(ctx);
  ctx->train_ms = batch_ms;
  ctx->train_epoch_ms = ms;
  ctx->train_records = (int64_t)ep * n;
  ctx->train_batches = (int64_t)ep * nbatches;
  ctx->train_fused = nfused;
  ctx->train_split = nsplit;
  ctx->train_multi = nmulti;
  if (epochs_run) *epochs_run = ep;
  return HGX_OK;
}

extern "C" int hgx_train_last_stats(hgx_ctx *ctx, double *ms, int64_t *records,
                                    int64_t *batches) {
  if (!ctx) return HGX_EINVAL;
  if (ms) *ms = ctx->train_ms;
  if (records) *records = ctx->train_records;
  if (batches) *batches = ctx->train_batches;
  return HGX_OK;
}

extern "C" int hgx_train_last_loss(hgx_ctx *ctx, double *loss_sum) {
  if (!ctx) return HGX_EINVAL;
  if (loss_sum) *loss_sum = ctx->train_loss_sum;
  return HGX_OK;
}

extern "C" int hgx_train_multi_pending(hgx_ctx *ctx, int64_t *batches) {
  if (!ctx) return HGX_EINVAL;
  if (batches) *batches = ctx->train_multi;
  return HGX_OK;
}

extern "C" int hgx_train_path_stats(hgx_ctx *ctx, int64_t *fused_batches,
                                    int64_t *split_batches) {
  if (!ctx) return HGX_EINVAL;
  if (fused_batches) *fused_batches = ctx->train_fused;
  if (split_batches) *split_batches = ctx->train_split;
  return HGX_OK;
}
