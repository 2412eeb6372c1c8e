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
// batches in parallel (one workgroup per batch: LDS bitonic sort of the
// batch's (row, slot) keys). K1/K2 for a run of batches are captured once
// as direct launches (or hipGraphs of 64 batches, HGX_GRAPH=1), the
// chunk-local batch index passed as a kernel argument (no device counters,
// no dependent index load).
// Preparation runs once per chunk of up to 1024 batches, on the same stream:
// overlapping it with training on a second stream measured slower (the
// per-batch kernels are latency-bound and lose more to the interference
// than the preparation costs).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "hgx_internal.h"

namespace {

constexpr int kTB = 256;
constexpr int kGraphBatches = 64;  // batches per chunk buffer and per graph

// diagnostic ablation bits (HGX_TRAIN_ABLATE, timing experiments only;
// results are wrong when set): 1 empty K1, 2 empty K2, 4 K1 gathers hit
// row 0, 8 K1 skips gradient stores, 16 K2 skips slot sums, 32 K2 skips
// the table read-modify-write.
#ifdef HGX_DEBUG_KNOBS
__constant__ int g_tab = 0;  // ablation bits (diagnostic builds only)
#else
static constexpr int g_tab = 0;
#endif

// diagnostic phase trace (HGX_TRAIN_TRACE=<file>, timing experiments only):
// wave 0 of every workgroup stamps s_memrealtime (100 MHz) at phase ends
// for the first g_trace_nb batches; slots [batch][kernel][block < 1024][8].
__constant__ unsigned long long *g_trace = nullptr;
__constant__ int g_trace_nb = 0;
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
  // fused path (train_fused): records packed so that every row touched by
  // more than one slot of a batch has all its slots in ONE workgroup.
  // Per chunk-local batch: NBF workgroups x prpb groups of R ids / codes / 3
  // targets, valid groups per workgroup, and whether the batch packed.
  int fused, prpb, NBF, MS;
  int *pidx, *pcode, *pnval, *pnblk, *pfast;
  float *ptgt;
  float *r0;  // [2 parity][2 table][p, acc][dp]: padding-row state handed on
  float *gp;  // [2 parity][NBF][2 table][dp]: padding-row partials per block
};

// slot codes of the fused path (train_prep -> train_fused)
constexpr unsigned kCodeMulti = 0x80000000u;  // row has >1 slot: LDS pos
constexpr unsigned kCodeOwn = 0x40000000u;    // this slot applies the update
constexpr int kPackB = 512;                   // max records per fused batch
constexpr int kPackM = 1024;                  // max multi-slot rows per batch
constexpr int kPackNBF = 64;                  // max fused workgroups per batch
constexpr int kPrepB = 1366;  // max records per prepared batch: 8192 slots / R >= 6

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
template <int L, int TB, int NBFM>
struct Row0Loads {
  static constexpr int NC = 2 * L, TPC = TB / NC, MAXPER = (NBFM + TPC - 1) / TPC;
  float4 gv[MAXPER];
  float4 rp, ra;  // the selected row-0 state (pending or table)
};

template <int L, int TB, int NBFM>
__device__ __forceinline__ void row0_issue_state(const TrainArgs &a,
                                                 const float4 *r0src, int mode,
                                                 Row0Loads<L, TB, NBFM> &ld) {
  using RL = Row0Loads<L, TB, NBFM>;
  static_assert(TB % RL::NC == 0, "workgroup covers whole columns");
  const int col = threadIdx.x % RL::NC;
  const int tab = col / L, c = col % L;
  // the address is selected (mode is wave-uniform), not the loaded value:
  // two loads instead of four on the first round trip
  const float4 *sp = mode ? r0src + (tab * 2) * L
                          : reinterpret_cast<const float4 *>(tab ? a.etab : a.ntab);
  const float4 *sa = mode ? r0src + (tab * 2 + 1) * L
                          : reinterpret_cast<const float4 *>(tab ? a.eacc : a.nacc);
  ld.rp = sp[c];
  ld.ra = sa[c];
}

// partials [0, nmax) of gpsrc (nmax <= NBFM, the instantiation's workgroup
// cap: MAXPER = NBFM / TPC loads per thread), issued unconditionally
// (index clamped: a branch around a load makes the compiler wait for it at
// the join); row0_stage masks the clamped copies (the gp buffer is zeroed at
// hgx_train entry, so it only ever holds finite partials).
template <int L, int TB, int NBFM>
__device__ __forceinline__ void row0_issue_partials(int nmax, const float4 *gpsrc,
                                                    Row0Loads<L, TB, NBFM> &ld) {
  using RL = Row0Loads<L, TB, NBFM>;
  const int col = threadIdx.x % RL::NC, sub = threadIdx.x / RL::NC;
  const int last = max(nmax - 1, 0);
#pragma unroll
  for (int u = 0; u < RL::MAXPER; u++)
    ld.gv[u] = gpsrc[(size_t)min(sub + u * RL::TPC, last) * RL::NC + col];
}

// this thread's fixed-order partial sum of partials [0, np) -> s_red
template <int L, int TB, int NBFM>
__device__ __forceinline__ void row0_stage(int np, const Row0Loads<L, TB, NBFM> &ld,
                                           float4 (*s_red)[2 * L]) {
  using RL = Row0Loads<L, TB, NBFM>;
  const int col = threadIdx.x % RL::NC, sub = threadIdx.x / RL::NC;
  float4 g = f4(0.f);
#pragma unroll
  for (int u = 0; u < RL::MAXPER; u++) {
    const float m = (float)(sub + u * RL::TPC < np);
    const float4 v = ld.gv[u];
    g = g + make_float4(v.x * m, v.y * m, v.z * m, v.w * m);
  }
  s_red[sub][col] = g;
}

// after row0_stage: the workgroup barrier, then the column owners (sub == 0)
// add the TPC staged sums in order and apply Adagrad (mode 1)
// p0 / a0 arrive holding the selected state (mode ? pending : table),
// picked right after row0_stage: that forces the state loads' wait BEFORE the
// gathers are issued (a wait for them after the wave-uniform list-gather
// branch would be counted conservatively and drain most gathers).
template <int L, int TB, int NBFM>
__device__ __forceinline__ void row0_finish(const TrainArgs &a, int mode,
                                            float4 (*s_red)[2 * L], float4 &p0,
                                            float4 &a0) {
  using RL = Row0Loads<L, TB, NBFM>;
  const int col = threadIdx.x % RL::NC, sub = threadIdx.x / RL::NC;
  __syncthreads();
  if (sub == 0 && mode) {
    float4 gs = f4(0.f);
#pragma unroll
    for (int j = 0; j < RL::TPC; j++) gs = gs + s_red[j][col];
    adagrad4(p0, a0, gs, a.lr, a.eps);
  }
}

// Fused batch step: K1 + K2 of one batch in ONE launch (no K1 -> K2
// boundary, no per-slot gradient round trip through HBM).
//  - train_prep packed the batch so that every row with several slots has
//    them all in one workgroup; single-slot rows (most) are updated by their
//    own group right after the backward pass, multi-slot rows by their first
//    slot's group after an LDS exchange and a workgroup barrier, summing in
//    sorted-slot order like train_update.
//  - The padding row 0 (touched by nearly every record) is deferred: its
//    per-workgroup partials go to gp[q & 1]; the NEXT fused launch (q + 1)
//    folds them in (row0_issue/finish) before its gathers, train_row0_flush
//    writes the final state back after the last fused batch of a run.
// One L-lane group per record (dp == 4L), prpb = TB / L records per
// workgroup, NBF workgroups; q = position in the run of consecutive fused
// launches, mode = q > 0.
template <int L, int KMAX, int MODE, int TB, int NBFM>
__global__ __launch_bounds__(TB) void train_fused(TrainArgs a, int cb, int gb,
                                                  int nb, int np, int q,
                                                  int mode) {
  constexpr int RPB = TB / L, R = 4 + 2 * KMAX, K = KMAX;
  extern __shared__ float4 s_ms[];  // [MS][L]: gradients of multi-slot rows
  __shared__ float4 s_z[2][RPB][L];
  __shared__ float4 s_red[TB / (2 * L)][2 * L];
  __shared__ float4 s_r0[2][L];
  __shared__ float s_loss[RPB];
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g_trace) ts[0] = __builtin_amdgcn_s_memrealtime();
  const int grp = threadIdx.x / L, lane = threadIdx.x % L;
  const int NBF = a.NBF;
  if (g_tab & 64) mode = 0;  // ablation: no partial reads
  // round trip 1 (kernel arguments only): the group's record ids, slot
  // codes and targets, the workgroup's record count, the row-0 state and
  // the np padding-row partials of the previous batch (np = its workgroup
  // count, a kernel argument)
  const size_t gi = ((size_t)cb * NBF + blockIdx.x) * RPB + grp;
  const int *ri = a.pidx + gi * R;
  const unsigned *rc = reinterpret_cast<const unsigned *>(a.pcode) + gi * R;
  const float *yt = a.ptgt + gi * 3;
  int row[R];
  unsigned code[R];
  {
    // one id and one code load per lane (lane s of the group loads slot s),
    // then readlanes broadcast the group's slots: 2 load instructions
    // instead of 2R on the first round trip. L = 64: one record per wave,
    // the ids land in scalar registers; L = 32: two records per wave.
    static_assert(L == 32 || L == 64, "fused step geometry");
    const int sl = lane < R ? lane : 0;
    const int rv = ri[sl];
    const int cv = (int)rc[sl];
#pragma unroll
    for (int s = 0; s < R; s++) {
      if (L == 64) {
        row[s] = __builtin_amdgcn_readlane(rv, s);
        code[s] = (unsigned)__builtin_amdgcn_readlane(cv, s);
      } else {
        const bool hi = threadIdx.x & 32;
        const int r0 = __builtin_amdgcn_readlane(rv, s), r1 = __builtin_amdgcn_readlane(rv, 32 + s);
        const int c0 = __builtin_amdgcn_readlane(cv, s), c1 = __builtin_amdgcn_readlane(cv, 32 + s);
        row[s] = hi ? r1 : r0;
        code[s] = (unsigned)(hi ? c1 : c0);
      }
    }
  }
  // targets: at L = 64 (one record per wave) lane c < 3 loads target c and
  // readlanes broadcast them (scalar); at L = 32 three broadcast loads
  // measured faster than the two-record select
  float yt0, yt1, yt2;
  if (L == 64) {
    const int tv = __float_as_int(yt[lane < 3 ? lane : 0]);
    yt0 = __int_as_float(__builtin_amdgcn_readlane(tv, 0));
    yt1 = __int_as_float(__builtin_amdgcn_readlane(tv, 1));
    yt2 = __int_as_float(__builtin_amdgcn_readlane(tv, 2));
  } else {
    yt0 = yt[0];
    yt1 = yt[1];
    yt2 = yt[2];
  }
  const int nval = a.pnval[(size_t)cb * NBF + blockIdx.x];
  if (!mode) np = 0;
  const size_t par = (size_t)NBF * 2 * L;  // float4 per gp parity
  Row0Loads<L, TB, NBFM> r0l;
  row0_issue_state<L, TB, NBFM>(a, reinterpret_cast<const float4 *>(a.r0) + (q & 1) * 4 * L,
                                mode, r0l);
  row0_issue_partials<L, TB, NBFM>(np, reinterpret_cast<const float4 *>(a.gp) + ((q - 1) & 1) * par,
                             r0l);
  HGX_STAMP(ts[1]);
  if (nval == 0) return;  // unused workgroup of this batch
  const bool has = grp < nval;
  // staged before the gathers: frees the partials' registers
  row0_stage<L, TB, NBFM>(np, r0l, s_red);
  float4 p0 = r0l.rp, a0 = r0l.ra;
  // pin the selects here (the compiler would sink them past the gathers)
  asm volatile("" : "+v"(p0.x), "+v"(p0.y), "+v"(p0.z), "+v"(p0.w), "+v"(a0.x),
               "+v"(a0.y), "+v"(a0.z), "+v"(a0.w));
  // round trip 2: every slot's table row and owner slots' accumulator
  // rows. Per slot unconditional (row 0 / non-owner slots read row 0, a hot
  // line): a load under a per-lane branch is waited for at the join, which
  // would serialise the gathers. The neighbour-list slots 4.. are skipped by
  // a WAVE-uniform branch when no record of the wave has a list (nn / ee
  // records: all list slots are the padding row, whose value comes from
  // s_r0 below): they are 20 of a record's 28 row loads, and a CU's load
  // issue (64 B/clk) is a large part of this phase. HGX_TRAIN_ABLATE & 256
  // disables the skip.
  float4 Pv[R], Av[R];
  bool lists = false;
#pragma unroll
  for (int s = 4; s < R; s++) lists |= row[s] != 0;
  const bool wave_lists = (g_tab & 256) || __any(lists);
#pragma unroll
  for (int s = 0; s < 4; s++) {
    // every record kind has two padding slots among the first four (ne:
    // le, rn; nn: le, re; ee: ln, rn). At L = 64 (one record per wave, the
    // ids are scalar) they are skipped: their value comes from s_r0 below.
    // At L = 32 the two records of a wave may differ in kind, and the
    // per-slot branch measured slower (7.80 -> 7.90 us per batch).
    if (L == 64 && !(g_tab & 512) && row[s] == 0) {
      Pv[s] = Av[s] = f4(0.f);
      continue;
    }
    const bool edge = slot_is_edge(s, K);
    const float4 *T = reinterpret_cast<const float4 *>(edge ? a.etab : a.ntab);
    const float4 *Ac = reinterpret_cast<const float4 *>(edge ? a.eacc : a.nacc);
    const int arow = (code[s] & kCodeOwn) ? row[s] : 0;
    Pv[s] = T[(size_t)row[s] * L + lane];
    Av[s] = Ac[(size_t)arow * L + lane];
  }
  if (wave_lists) {
#pragma unroll
    for (int s = 4; s < R; s++) {
      const bool edge = slot_is_edge(s, K);
      const float4 *T = reinterpret_cast<const float4 *>(edge ? a.etab : a.ntab);
      const float4 *Ac = reinterpret_cast<const float4 *>(edge ? a.eacc : a.nacc);
      const int arow = (code[s] & kCodeOwn) ? row[s] : 0;
      Pv[s] = T[(size_t)row[s] * L + lane];
      Av[s] = Ac[(size_t)arow * L + lane];
    }
  }
  {
    row0_finish<L, TB, NBFM>(a, mode, s_red, p0, a0);
    const int col = threadIdx.x % (2 * L), sub = threadIdx.x / (2 * L);
    if (sub == 0) {
      s_r0[col / L][col % L] = p0;
      if (blockIdx.x == 0) {
        float4 *r0d = reinterpret_cast<float4 *>(a.r0) + ((q + 1) & 1) * 4 * L;
        r0d[(col / L) * 2 * L + col % L] = p0;
        r0d[((col / L) * 2 + 1) * L + col % L] = a0;
      }
    }
    __syncthreads();
  }
  HGX_STAMP(ts[2]);
  float4 zN = f4(0.f), zE = f4(0.f);
  float lrec = 0.f;
  if (has) {
#pragma unroll
    for (int s = 0; s < R; s++)
      if (row[s] == 0) Pv[s] = s_r0[slot_is_edge(s, K) ? 1 : 0][lane];
    const float inv_b = 1.0f / (float)nb;
    const float4 &Nl = Pv[0], &El = Pv[1], &Nr = Pv[2], &Er = Pv[3];
    float z1 = group_sum<L>(dot4(Nl, Nr)), z2 = group_sum<L>(dot4(El, Er));
    float za[K], zb[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      za[k] = group_sum<L>(dot4(Pv[4 + k], Nl));
      zb[k] = group_sum<L>(dot4(Pv[4 + K + k], Er));
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
    auto emit = [&](int s, float4 g) {
      if (row[s] == 0) {
        if (slot_is_edge(s, K)) zE = zE + g;
        else zN = zN + g;
      } else if (code[s] & kCodeMulti) {
        s_ms[(code[s] & 0xfffu) * L + lane] = g;
      } else if (!(g_tab & 128)) {
        const bool edge = slot_is_edge(s, K);
        float4 pv = Pv[s], av = Av[s];
        adagrad4_hw(pv, av, f4(0.f) + g, a.lr, a.eps);
        reinterpret_cast<float4 *>(edge ? a.etab : a.ntab)[(size_t)row[s] * L + lane] = pv;
        reinterpret_cast<float4 *>(edge ? a.eacc : a.nacc)[(size_t)row[s] * L + lane] = av;
      }
    };
    float4 gln = fma4(dz1, Nr, f4(0.f)), gre = fma4(dz2, El, f4(0.f));
#pragma unroll
    for (int k = 0; k < K; k++) {
      const float da = dP * act_d(act, za[k], sa[k]);
      const float db = dQ * act_d(act, zb[k], sb[k]);
      gln = fma4(da, Pv[4 + k], gln);
      gre = fma4(db, Pv[4 + K + k], gre);
      emit(4 + k, fma4(da, Nl, f4(0.f)));
      emit(4 + K + k, fma4(db, Er, f4(0.f)));
    }
    emit(0, gln);
    emit(3, gre);
    emit(2, fma4(dz1, Nl, f4(0.f)));
    emit(1, fma4(dz2, Er, f4(0.f)));
    HGX_STAMP(ts[4]);
  }
  s_z[0][grp][lane] = zN;
  s_z[1][grp][lane] = zE;
  if (lane == 0) s_loss[grp] = lrec;
  __syncthreads();
  if (has) {
#pragma unroll
    for (int s = 0; s < R; s++) {
      const unsigned cd = code[s];
      if (row[s] != 0 && (cd & kCodeMulti) && (cd & kCodeOwn)) {
        const int pos = cd & 0xfffu, cnt = (cd >> 12) & 0xfffu;
        float4 g = f4(0.f);
        for (int j = 0; j < cnt; j++) g = g + s_ms[(pos + j) * L + lane];
        const bool edge = slot_is_edge(s, K);
        float4 pv = Pv[s], av = Av[s];
        adagrad4_hw(pv, av, g, a.lr, a.eps);
        reinterpret_cast<float4 *>(edge ? a.etab : a.ntab)[(size_t)row[s] * L + lane] = pv;
        reinterpret_cast<float4 *>(edge ? a.eacc : a.nacc)[(size_t)row[s] * L + lane] = av;
      }
    }
  }
  HGX_STAMP(ts[5]);
  float4 *gpd = reinterpret_cast<float4 *>(a.gp) + (q & 1) * par;
  for (int t = threadIdx.x; t < 2 * L; t += TB) {
    const int tab = t / L, j = t % L;
    float4 sz = f4(0.f);
    for (int g = 0; g < RPB; g++) sz = sz + s_z[tab][g][j];
    gpd[((size_t)blockIdx.x * 2 + tab) * L + j] = sz;
  }
  if (threadIdx.x == 0) {
    float sl = 0.f;
    for (int g = 0; g < RPB; g++) sl += s_loss[g];
    a.lossbuf[(size_t)gb * a.lstride + blockIdx.x] = sl;
  }
  HGX_STAMP(ts[6]);
  trace_put(gb, 0, 7, ts);
}

// After the last launch q of a fused run: the pending padding-row update ->
// row 0 of both tables and accumulators.
template <int L, int TB, int NBFM>
__global__ __launch_bounds__(TB) void train_row0_flush(TrainArgs a, int cb, int q) {
  __shared__ float4 s_red[TB / (2 * L)][2 * L];
  const size_t par = (size_t)a.NBF * 2 * L;
  Row0Loads<L, TB, NBFM> r0l;
  row0_issue_state<L, TB, NBFM>(a, reinterpret_cast<const float4 *>(a.r0) + ((q + 1) & 1) * 4 * L,
                                1, r0l);
  row0_issue_partials<L, TB, NBFM>(a.NBF, reinterpret_cast<const float4 *>(a.gp) + (q & 1) * par,
                             r0l);
  row0_stage<L, TB, NBFM>(a.pnblk[cb], r0l, s_red);
  float4 p0 = r0l.rp, a0 = r0l.ra;
  row0_finish<L, TB, NBFM>(a, 1, s_red, p0, a0);
  const int col = threadIdx.x % (2 * L), sub = threadIdx.x / (2 * L);
  if (sub == 0) {
    const int tab = col / L, c = col % L;
    reinterpret_cast<float4 *>(tab ? a.etab : a.ntab)[c] = p0;
    reinterpret_cast<float4 *>(tab ? a.eacc : a.nacc)[c] = a0;
  }
}

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

// Fused-path packing of one batch (tail of train_prep, same workgroup, the
// batch's (row, slot) keys sorted in LDS).
//  1. Records that share a non-padding row are connected; components by
//     min-label propagation with pointer jumping (bounded; no convergence ->
//     the batch takes the two-kernel path).
//  2. Components are placed whole, in order of their first record, into
//     workgroups of prpb groups with at most MS multi-slot rows' slots each
//     (first fit in sequence; a component too large for one workgroup, or
//     more than NBF workgroups -> two-kernel path).
//  3. Each slot gets a code: single-slot row -> kCodeOwn (its group applies
//     Adagrad directly); multi-slot row -> kCodeMulti | LDS position, the
//     row's slots on consecutive positions in sorted-slot order, the first
//     also kCodeOwn | count << 12 (it sums them in that order and applies
//     Adagrad: the same order and arithmetic as train_update).
// Every serial step runs on thread 0 in record / sorted order: the packing is
// a deterministic function of the batch.
__device__ void pack_batch(const TrainArgs &a, int cb, int nb, int V, int P,
                           const unsigned long long *s_key, int *s_ws) {
  __shared__ int s_lab[kPackB], s_csz[kPackB], s_cms[kPackB], s_cblk[kPackB],
      s_cmoff[kPackB], s_grp[kPackB];
  __shared__ int s_mrun[kPackM], s_mlen[kPackM], s_mbase[kPackM];
  __shared__ int s_bfill[kPackNBF], s_bshort[kPackNBF];
  __shared__ unsigned char s_short[kPackB];
  __shared__ int s_flag[2], s_ok;
  const int R = a.R, RPB = a.prpb, NBF = a.NBF, MS = a.MS;
  volatile int *lab = s_lab;
  auto rowkey = [&](int t) { return (unsigned)(s_key[t] >> 32); };
  auto slotof = [&](int t) { return (int)(unsigned)(s_key[t] & 0xffffffffu); };
  for (int i = threadIdx.x; i < nb; i += kTB) {
    s_lab[i] = i;
    s_csz[i] = 0;
    s_cms[i] = 0;
  }
  if (threadIdx.x == 0) {
    s_flag[0] = s_flag[1] = 0;
    s_ok = nb <= kPackB;
  }
  __syncthreads();
  if (!s_ok) {
    if (threadIdx.x == 0) a.pfast[cb] = 0;
    return;
  }
  int conv = 0;
  for (int it = 0; it < 64; it++) {
    for (int t = 1 + threadIdx.x; t < V; t += kTB) {
      if (rowkey(t) == rowkey(t - 1)) {
        const int ra = slotof(t - 1) / R, rb = slotof(t) / R;
        const int la = lab[ra], lb = lab[rb];
        if (la != lb) {
          const int m = min(la, lb);
          atomicMin(&s_lab[ra], m);
          atomicMin(&s_lab[rb], m);
          s_flag[it & 1] = 1;
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_flag[(it + 1) & 1] = 0;
    for (int i = threadIdx.x; i < nb; i += kTB) {
      const int l = lab[i];
      const int ll = lab[l];
      if (ll < l) atomicMin(&s_lab[i], ll);
    }
    __syncthreads();
    if (!s_flag[it & 1]) {
      conv = 1;
      break;
    }
  }
  // component sizes and multi-slot counts
  for (int i = threadIdx.x; i < nb; i += kTB) atomicAdd(&s_csz[lab[i]], 1);
  const int per = P / kTB, t0 = threadIdx.x * per;
  int nm = 0;
  for (int t = t0; t < t0 + per && t < V; t++) {
    const bool prev = t > 0 && rowkey(t) == rowkey(t - 1);
    const bool next = t + 1 < V && rowkey(t + 1) == rowkey(t);
    if (prev || next) atomicAdd(&s_cms[lab[slotof(t) / R]], 1);
    if (!prev && next) nm++;
  }
  int M = 0;
  int m0 = block_exclusive_scan(nm, &M, s_ws);
  if (M <= kPackM) {
    for (int t = t0; t < t0 + per && t < V; t++) {
      const bool prev = t > 0 && rowkey(t) == rowkey(t - 1);
      const bool next = t + 1 < V && rowkey(t + 1) == rowkey(t);
      if (!prev && next) {
        int c = 2;
        while (t + c < V && rowkey(t + c) == rowkey(t)) c++;
        s_mrun[m0] = t;
        s_mlen[m0] = c;
        m0++;
      }
    }
  }
  // records without neighbour lists (nn / ee): placed first in their
  // workgroup so that whole waves skip the list-slot gathers in train_fused
  // (from the batch-ordered copies train_prep wrote: contiguous, no
  // dependent record-id load)
  const int *bidx = a.bidx + (size_t)cb * a.B * R;
  const float *btgt = a.btgt + (size_t)cb * a.B * 3;
  for (int i = threadIdx.x; i < nb; i += kTB) {
    const int *ri = bidx + i * R;
    int any = 0;
    for (int s2 = 4; s2 < R; s2++) any |= ri[s2];
    s_short[i] = any == 0;
  }
  __syncthreads();
  // Component placement, first fit in record order. The scan is sequential,
  // so wave 0 runs it in scalar registers: every record's packed
  // (size | multi-slot count << 10, 0 for a non-root) sits in a VGPR of its
  // lane and is read by a wave-uniform readlane; the results go back into
  // the root's lane by a lane-select. No LDS round trip sits on the chain (one
  // thread walking LDS arrays took most of train_prep's time).
  if (threadIdx.x < 64) {
    constexpr int U = kPackB / 64;
    const int lane = threadIdx.x;
    int pk[U], rb[U], ro[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int i = u * 64 + lane;
      pk[u] = (i < nb && lab[i] == i) ? (s_csz[i] | (s_cms[i] << 10)) : 0;
      rb[u] = ro[u] = 0;
    }
    int ok = conv && M <= kPackM && NBF <= kPackNBF;
    int fill = 0, msf = 0, blk = 0;
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (u * 64 >= nb) break;
      for (int l = 0; l < 64 && ok; l++) {
        const int v = __builtin_amdgcn_readlane(pk[u], l);
        if (v == 0) continue;
        const int sz = v & 1023, q = v >> 10;
        if (sz > RPB || q > MS) {
          ok = 0;
          break;
        }
        if (fill + sz > RPB || msf + q > MS) {
          if (lane == 0) s_bfill[blk] = fill;
          blk++;
          fill = msf = 0;
        }
        if (blk >= NBF) {
          ok = 0;
          break;
        }
        if (lane == l) {
          rb[u] = blk;
          ro[u] = msf;
        }
        fill += sz;
        msf += q;
      }
    }
    if (ok) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (pk[u] != 0) {
          s_cblk[u * 64 + lane] = rb[u];
          s_cmoff[u * 64 + lane] = ro[u];
        }
      }
    }
    if (lane == 0) {
      if (ok) s_bfill[blk] = fill;
      s_ok = ok;
      s_flag[0] = blk + 1;
      a.pfast[cb] = ok;
      a.pnblk[cb] = ok ? blk + 1 : 0;
    }
  }
  __syncthreads();
  if (!s_ok) return;
  {
    // positions inside a workgroup: records without lists first, then the
    // others, each in record order (the workgroup of a record, and so the
    // packing, is unchanged; multi-slot codes index LDS, not positions).
    // s_csz now holds each record's key = block * 2 + no-list flag; s_mlen
    // gets its run's component in the upper half.
    const int nblk = s_flag[0];
    for (int j = threadIdx.x; j < NBF; j += kTB) {
      if (j < nblk) s_bshort[j] = 0;
      else s_bfill[j] = 0;
    }
    for (int i = threadIdx.x; i < nb; i += kTB) s_csz[i] = s_cblk[lab[i]] * 2 + s_short[i];
    for (int k = threadIdx.x; k < M; k += kTB)
      s_mlen[k] |= lab[slotof(s_mrun[k]) / R] << 16;
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += kTB)
      if (s_short[i]) atomicAdd(&s_bshort[s_csz[i] >> 1], 1);
    __syncthreads();
    // rank among the earlier records of the same key; a multi-slot run's
    // base = its component's offset + the runs of that component before it
    for (int i = threadIdx.x; i < nb; i += kTB) {
      const int key = s_csz[i], b = key >> 1;
      int r = 0;
      for (int j = 0; j < i; j++) r += s_csz[j] == key;
      s_grp[i] = b * RPB + ((key & 1) ? r : s_bshort[b] + r);
    }
    for (int k = threadIdx.x; k < M; k += kTB) {
      const int comp = s_mlen[k] >> 16;
      int base = s_cmoff[comp];
      for (int j = 0; j < k; j++)
        if ((s_mlen[j] >> 16) == comp) base += s_mlen[j] & 0xffff;
      s_mbase[k] = base;
    }
  }
  const int G = NBF * RPB;
  int *pidx = a.pidx + (size_t)cb * G * R;
  unsigned *pcode = reinterpret_cast<unsigned *>(a.pcode) + (size_t)cb * G * R;
  float *ptgt = a.ptgt + (size_t)cb * G * 3;
  for (int t = threadIdx.x; t < G * R; t += kTB) {
    pidx[t] = 0;
    pcode[t] = 0u;
  }
  for (int t = threadIdx.x; t < G * 3; t += kTB) ptgt[t] = 0.f;
  for (int j = threadIdx.x; j < NBF; j += kTB) a.pnval[(size_t)cb * NBF + j] = s_bfill[j];
  __syncthreads();  // zero fill before the scattered writes (same workgroup)
  // 8 loads per thread in flight before the stores (a global store between
  // two loads would make each load wait for the previous one)
  for (int t0 = threadIdx.x; t0 < nb * R; t0 += 8 * kTB) {
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int t = t0 + u * kTB;
      v[u] = t < nb * R ? bidx[t] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int t = t0 + u * kTB;
      if (t < nb * R) {
        const int i = t / R;
        pidx[s_grp[i] * R + (t - i * R)] = v[u];
      }
    }
  }
  for (int t = threadIdx.x; t < nb * 3; t += kTB) {
    const int i = t / 3, c = t - i * 3;
    ptgt[s_grp[i] * 3 + c] = btgt[t];
  }
  for (int t = threadIdx.x; t < V; t += kTB) {
    const bool prev = t > 0 && rowkey(t) == rowkey(t - 1);
    const bool next = t + 1 < V && rowkey(t + 1) == rowkey(t);
    if (!prev && !next) {
      const int sl = slotof(t), i = sl / R;
      pcode[s_grp[i] * R + (sl - i * R)] = kCodeOwn;
    }
  }
  for (int k = threadIdx.x; k < M; k += kTB) {
    const int t = s_mrun[k], c = s_mlen[k] & 0xffff, base = s_mbase[k];
    for (int j = 0; j < c; j++) {
      const int sl = slotof(t + j), i = sl / R;
      unsigned code = kCodeMulti | (unsigned)(base + j);
      if (j == 0) code |= kCodeOwn | ((unsigned)c << 12);
      pcode[s_grp[i] * R + (sl - i * R)] = code;
    }
  }
}

// One workgroup per batch of the chunk: sorted unique (table,row) keys of
// the non-padding slots and, per key, its slot ids in ascending order.
__global__ __launch_bounds__(kTB) void train_prep(TrainArgs a, int64_t base,
                                                  int nbc, int P) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_key[];
  __shared__ int s_ws[kTB / 64];
  const int cb = blockIdx.x;
  if (cb >= nbc) {  // graph nodes past the last batch find no work
    if (threadIdx.x == 0) a.bmeta[cb] = make_int2(0, 0);
    return;
  }
  const int64_t r0 = (base + cb) * a.B;
  const int nb = (int)min((int64_t)a.B, a.n - r0);
  if (threadIdx.x == 0) a.bmeta[cb] = make_int2(nb, (int)(base + cb));
  const int R = a.R, K = a.K;
  const int S = nb * R;
  int *bidx = a.bidx + (size_t)cb * a.B * R;
  float *btgt = a.btgt + (size_t)cb * a.B * 3;
  // the batch's record ids once into LDS, then every gather below has one
  // round trip; slot rows 8 per thread in flight before the stores
  __shared__ int s_perm[kPrepB];
  for (int i = threadIdx.x; i < nb; i += kTB) s_perm[i] = a.perm[r0 + i];
  __syncthreads();
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
  block_exclusive_scan(valid, &V, s_ws);
  int *ukey = a.ukey + (size_t)cb * a.SB;
  int *uoff = a.uoff + (size_t)cb * (a.SB + 1);
  int *inv = a.inv + (size_t)cb * a.SB;
  for (int t = t0; t < t0 + per; t++) {
    const unsigned long long x = s_key[t];
    if (x == ~0ull) break;
    inv[x & 0xffffffffu] = t;
    if (t == 0 || (unsigned)(s_key[t - 1] >> 32) != (unsigned)(x >> 32)) {
      ukey[u] = (int)(x >> 32);
      uoff[u] = t;
      u++;
    }
  }
  if (threadIdx.x == 0) {
    uoff[U] = V;
    a.ucount[cb] = U;
  }
  if (a.fused) pack_batch(a, cb, nb, V, P, s_key, s_ws);
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

using KFusedFn = void (*)(TrainArgs, int, int, int, int, int, int);
using KFlushFn = void (*)(TrainArgs, int, int);

// fused one-launch step: d in (64, 256] (one float4 per lane, L = 32 or 64),
// K = 5 with the FOBE (sigmoid/KLD) or HOBE (relu/MSE) heads. NBFM = the
// workgroup cap of the instantiation (40 when the batch packs into at most
// 40 workgroups, else kPackNBF): every workgroup of the next launch loads
// ceil(NBFM / TPC) padding-row partials per thread.
template <int L, int TB, int NBFM>
void fused_fns(int loss, KFusedFn &kf, KFlushFn &kfl) {
  kf = loss == 0 ? train_fused<L, 5, 1, TB, NBFM> : train_fused<L, 5, 2, TB, NBFM>;
  kfl = train_row0_flush<L, TB, NBFM>;
}
bool pick_fused(int L, int VPL, int K, int loss, int act, int nbfm, KFusedFn &kf,
                KFlushFn &kfl, int &tb) {
  if (VPL != 1 || K != 5 || loss != act) return false;
  if (L == 32) {
    tb = 256;
    if (nbfm <= 40) fused_fns<32, 256, 40>(loss, kf, kfl);
    else fused_fns<32, 256, kPackNBF>(loss, kf, kfl);
    return true;
  }
  if (L == 64) {
    tb = 512;
    if (nbfm <= 40) fused_fns<64, 512, 40>(loss, kf, kfl);
    else fused_fns<64, 512, kPackNBF>(loss, kf, kfl);
    return true;
  }
  return false;
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

// ---------------------------------------------------------------------------
// fit
// ---------------------------------------------------------------------------
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
        unsigned long long *z = nullptr;
        hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &z, sizeof(z));
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
    HGX_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &tp, sizeof(tp)));
    HGX_HIP(ctx, hipMemcpyToSymbol(HIP_SYMBOL(g_trace_nb), &tn, sizeof(tn)));
  }
  const int RPB = tb1 / L;
  const int nblk1 = (batch + RPB - 1) / RPB;
  // fused step: eligible geometry, batch <= kPackB records, NBF workgroups
  // (packing leaves holes: nblk1 + 50% + 2, at most kPackNBF)
  KFusedFn kf = nullptr;
  KFlushFn kfl = nullptr;
  int tbf = 0;
  // train_fused tuning 0: off; else HGX_TRAIN_FUSED (debug builds): 0 off,
  // 1 only d in (64, 128] (L = 32), 2 (default)
  // also d in (128, 256] (L = 64; r01: 12.7 vs 12.7 us/batch with the wide
  // workgroup cap, 11.3 vs 12.7 with the 40-workgroup cap and the list-gather
  // skip)
  const int fz = ctx->tune.train_fused ? env_int("HGX_TRAIN_FUSED", 2) : 0;
  // workgroups per fused batch: the records' lane groups plus headroom for
  // packing holes (components placed whole, first fit): +8 when that stays
  // within 40 (the NBFM = 40 instantiation, fewer padding-row partial loads
  // per workgroup; HGX_TRAIN_NBF_WIDE=1 keeps the wide cap), else 50% + 2 up
  // to kPackNBF. A batch that needs more takes the two-kernel step.
  const int tb_f = L == 64 ? 512 : 256;
  const int prpb0 = tb_f / L;
  const int need0 = (batch + prpb0 - 1) / prpb0;
  const bool narrow_nbf = need0 + 8 <= 40 && env_int("HGX_TRAIN_NBF_WIDE", 0) != 1;
  const int nbf_target = narrow_nbf ? need0 + 8 : std::min(kPackNBF, need0 + need0 / 2 + 2);
  bool fused = fz != 0 && (L == 32 || fz == 2) &&
               env_int("HGX_TRAIN_GENERIC", 0) != 1 &&
               pick_fused(L, VPL, K, loss, act, nbf_target, kf, kfl, tbf) &&
               batch <= kPackB;
  const int prpb = fused ? tbf / L : 0;
  const int nbf_need = fused ? (batch + prpb - 1) / prpb : 0;
  const int NBF = fused ? nbf_target : 0;
  if (fused && NBF < nbf_need) fused = false;
  const int MS = 48;  // LDS rows for multi-slot gradients per workgroup
  const int lstride = std::max(nblk1, NBF);
  const int GPB2 = tb2 / L;
  // one unique-row task per group, plus the two padding-row workgroups
  const int grid2 = (SB + GPB2 - 1) / GPB2 + 2;
  const int64_t nbatches = (n + batch - 1) / batch;
  const int GB = kGraphBatches;
  // prep chunk: CB batches (a multiple of GB) prepared by one launch, then
  // trained by CB / GB graph replays (graph g holds chunk-local batches
  // [g*GB, (g+1)*GB), their indices baked into the node arguments)
  const int CB = (int)std::min<int64_t>(1024, (nbatches + GB - 1) / GB * GB);
  const int NG = CB / GB;
  const int64_t nchunks = (nbatches + CB - 1) / CB;

  // record copies padded so K1's unconditional id loads stay in bounds
  const size_t bidx_n = (size_t)CB * batch * R + (size_t)RPB * R * 2 + 64;
  const size_t btgt_n = (size_t)CB * batch * 3 + (size_t)RPB * 3 * 2 + 64;
  const size_t inv_n = (size_t)CB * SB + (size_t)RPB * R * 2 + 64;
  const size_t pg = fused ? (size_t)CB * NBF * prpb : 0;  // packed groups
  const size_t pack_ints = fused ? pg * R * 2 + pg * 3 + (size_t)CB * NBF + 2 * CB + 64 : 0;
  const size_t prep_ints = bidx_n + btgt_n + inv_n + (size_t)CB * SB +
                           (size_t)CB * (SB + 1) + CB + 2 * CB + 64 + pack_ints;
  HGX_TRY(hgx_ensure(ctx, ctx->s1, sizeof(int) * (n + 1)));              // perm
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(float) * (size_t)SB * dp));    // gslot
  // gzero (K1 partials) | r0 [2][2][2][dp] | gp [2][NBF][2][dp]
  const size_t s3_f = (size_t)nblk1 * 2 * dp + 8 * (size_t)dp + (size_t)2 * NBF * 2 * dp;
  HGX_TRY(hgx_ensure(ctx, ctx->s3, sizeof(float) * s3_f));
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * (size_t)nbatches * lstride + 16));
  // chunk buffers in two parities: train_prep of chunk c + 1 runs on a side
  // stream while chunk c trains (graph replay bakes parity 0: one parity)
  const bool use_graph = env_int("HGX_GRAPH", 0) == 1 && !fused;
  // HGX_TRAIN_PIPE: 0 (default) = one parity, prep of chunk c + 1 queued
  // right after chunk c (the host waits for it with the GPU idle, ~0.1 ms per
  // 1024 batches); 1 = two parities, prep of chunk c + 1 queued on the same
  // stream BEFORE chunk c's batches (no host bubble); 2 = two parities, prep
  // on a side stream beside the batches. Measured r01 at d=128 (4M records):
  // 8.61 / 8.90 / 9.45 us per batch. The packed records a prep has just
  // written sit in the Infinity Cache when the batches right behind it read
  // them; preparing a chunk ahead lets 9 ms of training traffic evict them,
  // and a second active stream also slows every batch launch.
  const int pipe = use_graph ? 0 : env_int("HGX_TRAIN_PIPE", 0);
  const int NPAR = pipe == 0 ? 1 : 2;
  HGX_TRY(hgx_ensure(ctx, ctx->s5, sizeof(int) * prep_ints * NPAR));
  HGX_TRY(hgx_ensure(ctx, ctx->s6, 64 + sizeof(double) * kLossBlocks));  // loss
  int *perm = ctx->s1.as<int>();
  HGX_HIP(ctx, hipMemsetAsync(ctx->s5.p, 0, sizeof(int) * prep_ints * NPAR, ctx->stream));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s3.p, 0, sizeof(float) * s3_f, ctx->stream));
  TrainArgs a;
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
  a.NBF = NBF;
  a.MS = MS;
  a.r0 = a.gzero + (size_t)nblk1 * 2 * dp;
  a.gp = a.r0 + 8 * (size_t)dp;
  a.lr = lr;
  a.eps = eps;
  a.loss = loss;
  a.act = act;
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
    a.pidx = q;
    q += pg * R;
    a.pcode = q;
    q += pg * R;
    a.ptgt = reinterpret_cast<float *>(q);
    q += pg * 3;
    a.pnval = q;
    q += (size_t)CB * NBF;
    a.pnblk = q;
    q += CB;
    a.pfast = q;
  }
  // parity 1: the same layout shifted by prep_ints
  TrainArgs ap[2] = {a, a};
  if (NPAR == 2) {
    const size_t sh = prep_ints;
    TrainArgs &b = ap[1];
    b.bidx += sh;
    b.btgt += sh;
    b.inv += sh;
    b.ukey += sh;
    b.uoff += sh;
    b.ucount += sh;
    b.bmeta = reinterpret_cast<int2 *>(reinterpret_cast<int *>(b.bmeta) + sh);
    b.pidx += sh;
    b.pcode += sh;
    b.ptgt += sh;
    b.pnval += sh;
    b.pnblk += sh;
    b.pfast += sh;
  }
  double *dloss = reinterpret_cast<double *>(ctx->s6.as<char>() + 32);
  double *dpart = reinterpret_cast<double *>(ctx->s6.as<char>() + 64);

  // shuffle scratch (device shuffle only)
  size_t sort_tmp = 0, sort_off = 0;
  unsigned long long *keys_in = nullptr, *keys_out = nullptr;
  int *vals_in = nullptr;
  if (!perms) {
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
      if (side) (void)hipStreamDestroy(side);
      if (hflags) (void)hipHostFree(hflags);
    }
    hipStream_t side = nullptr;
    int *hflags = nullptr;  // pinned [NPAR][2][CB]: pfast, pnblk per parity
  } res;
  // Direct launches by default: measured as fast as hipGraph replay of the
  // same kernels (10.6 us per batch both ways at d=128) with less host time,
  // and rocprofv3 kernel tracing crashes on the replays. HGX_GRAPH=1 replays
  // captured graphs instead.
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

  // prep pipeline: side stream, per parity "prep done + flags copied" and
  // "chunk trained" events
  hipEvent_t ev_prep[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr},
             ev_perm = nullptr;
  if (pipe == 2) HGX_HIP(ctx, hipStreamCreateWithFlags(&res.side, hipStreamNonBlocking));
  hipStream_t ps = pipe == 2 ? res.side : ctx->stream;  // prep stream
  HGX_HIP(ctx, hipHostMalloc(reinterpret_cast<void **>(&res.hflags),
                             sizeof(int) * 4 * (size_t)CB));
  for (int i = 0; i < 2; i++) {
    HGX_HIP(ctx, hipEventCreateWithFlags(&ev_prep[i], hipEventDisableTiming));
    res.ev.push_back(ev_prep[i]);
    HGX_HIP(ctx, hipEventCreateWithFlags(&ev_free[i], hipEventDisableTiming));
    res.ev.push_back(ev_free[i]);
  }
  HGX_HIP(ctx, hipEventCreateWithFlags(&ev_perm, hipEventDisableTiming));
  res.ev.push_back(ev_perm);
  // both parities start free
  for (int i = 0; i < 2; i++) HGX_HIP(ctx, hipEventRecord(ev_free[i], ctx->stream));
  // train_prep of chunk c into parity c % NPAR on the side stream, after the
  // epoch's permutation and after the parity's previous chunk trained; then
  // its packing flags to pinned host memory
  auto issue_prep = [&](int64_t c) -> int {
    const int par = (int)(c % NPAR);
    const TrainArgs &ac = ap[par];
    const int64_t base = c * CB;
    const int nbc = (int)std::min<int64_t>(CB, nbatches - base);
    if (ps != ctx->stream) {
      HGX_HIP(ctx, hipStreamWaitEvent(ps, ev_perm, 0));
      HGX_HIP(ctx, hipStreamWaitEvent(ps, ev_free[par], 0));
    }
    hipLaunchKernelGGL(train_prep, dim3(CB), dim3(kTB),
                       (size_t)P * sizeof(unsigned long long), ps, ac,
                       base, nbc, P);
    HGX_LAUNCH_CHECK(ctx);
    if (fused) {
      int *hf = res.hflags + (size_t)par * 2 * CB;
      HGX_HIP(ctx, hipMemcpyAsync(hf, ac.pfast, sizeof(int) * nbc,
                                  hipMemcpyDeviceToHost, ps));
      HGX_HIP(ctx, hipMemcpyAsync(hf + CB, ac.pnblk, sizeof(int) * nbc,
                                  hipMemcpyDeviceToHost, ps));
    }
    HGX_HIP(ctx, hipEventRecord(ev_prep[par], ps));
    return HGX_OK;
  };

  std::vector<int> hperm;
  int64_t nfused = 0, nsplit = 0;
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
    if (hipEventRecord(ev_perm, ctx->stream) != hipSuccess ||
        (rc = issue_prep(0)) != HGX_OK) {
      if (!rc) rc = hgx_fail(ctx, HGX_EHIP, "prep pipeline failed");
      break;
    }
    for (int64_t c = 0; c < nchunks && rc == HGX_OK; c++) {
      const int par = (int)(c % NPAR);
      const TrainArgs &ac = ap[par];
      const int64_t base = c * CB;
      const int nbc = (int)std::min<int64_t>(CB, nbatches - base);
      const int *hfast = res.hflags + (size_t)par * 2 * CB;
      const int *hnblk = hfast + CB;
      // which batches packed: one host wait per chunk, normally long done
      // (prep c ran beside chunk c - 1)
      if (hipEventSynchronize(ev_prep[par]) != hipSuccess ||
          (ps != ctx->stream &&
           hipStreamWaitEvent(ctx->stream, ev_prep[par], 0) != hipSuccess)) {
        rc = hgx_fail(ctx, HGX_EHIP, "batch preparation failed: %s",
                      hipGetErrorString(hipGetLastError()));
        break;
      }
      if (NPAR == 1 && c + 1 < nchunks) {
        // one parity: chunk c + 1's prep must follow chunk c (queued below)
      } else if (c + 1 < nchunks && (rc = issue_prep(c + 1)) != HGX_OK) {
        break;
      }
      (void)hipEventRecord(bev[2 * c], ctx->stream);
      if (fused) {
        int qrun = 0;  // position in the current run of fused launches
        for (int b = 0; b < nbc; b++) {
          if (hfast[b]) {
            const int64_t gbat = base + b;
            const int nrec = (int)std::min<int64_t>(batch, n - gbat * batch);
            hipLaunchKernelGGL(kf, dim3(NBF), dim3(tbf),
                               (size_t)MS * L * sizeof(float4), ctx->stream, ac,
                               b, (int)gbat, nrec, qrun > 0 ? hnblk[b - 1] : 0,
                               qrun, qrun > 0 ? 1 : 0);
            qrun++;
            nfused++;
          } else {
            if (qrun > 0)
              hipLaunchKernelGGL(kfl, dim3(1), dim3(tbf), 0, ctx->stream, ac,
                                 b - 1, qrun - 1);
            qrun = 0;
            launch_run(ac, b, 1);
            nsplit++;
          }
        }
        if (qrun > 0)
          hipLaunchKernelGGL(kfl, dim3(1), dim3(tbf), 0, ctx->stream, ac,
                             nbc - 1, qrun - 1);
      } else if (use_graph) {
        for (int g = 0; g * GB < nbc; g++) {
          if (hipGraphLaunch(res.gexec[g], ctx->stream) != hipSuccess) {
            rc = hgx_fail(ctx, HGX_EHIP, "graph launch failed");
            break;
          }
        }
      } else {
        launch_run(ac, 0, nbc);
        nsplit += nbc;
      }
      (void)hipEventRecord(bev[2 * c + 1], ctx->stream);
      (void)hipEventRecord(ev_free[par], ctx->stream);
      if (NPAR == 1 && c + 1 < nchunks && (rc = issue_prep(c + 1)) != HGX_OK) break;
    }
    if (rc) break;
    hipLaunchKernelGGL(loss_partial, dim3(kLossBlocks), dim3(kTB), 0,
                       ctx->stream, a.lossbuf, nbatches * lstride, dpart);
    hipLaunchKernelGGL(loss_final, dim3(1), dim3(kLossBlocks), 0, ctx->stream,
                       dpart, dloss);
    double lsum = 0.0;
    if (hipMemcpyAsync(&lsum, dloss, sizeof(double), hipMemcpyDeviceToHost,
                       ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
      rc = hgx_fail(ctx, HGX_EHIP, "epoch failed: %s",
                    hipGetErrorString(hipGetLastError()));
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

extern "C" int hgx_train_path_stats(hgx_ctx *ctx, int64_t *fused_batches,
                                    int64_t *split_batches) {
  if (!ctx) return HGX_EINVAL;
  if (fused_batches) *fused_batches = ctx->train_fused;
  if (split_batches) *split_batches = ctx->train_split;
  return HGX_OK;
}
