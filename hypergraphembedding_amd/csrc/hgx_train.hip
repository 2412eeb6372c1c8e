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
// in a hipGraph and replayed; the batch index lives in device counters
// (K1 reads ctr[0] and publishes ctr[1]; K2 reads ctr[1] and advances
// ctr[0]), so the graph needs no per-batch arguments.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "hgx_internal.h"

namespace {

constexpr int kTB = 256;
constexpr int kGraphBatches = 64;

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
  int *ctr;  // [0] K1 batch, [1] K2 batch, [2] chunk base batch, [3] chunk nb
  int SB, nblk1;
  float lr, eps;
  int loss, act;
};

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

template <int L, int VPL, int KMAX>
__global__ __launch_bounds__(kTB) void train_fwd_bwd(TrainArgs a) {
  constexpr int RPB = kTB / L;
  __shared__ float4 s_z[2][RPB][L * VPL];
  __shared__ float s_loss[RPB];
  const int cb = a.ctr[0];
  // publish before the tail check: a tail K2 must see cb >= nb and exit
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctr[1] = cb;
  if (cb >= a.ctr[3]) return;
  const int64_t gb = (int64_t)a.ctr[2] + cb;
  const int64_t r0 = gb * a.B;
  const int nb = (int)min((int64_t)a.B, a.n - r0);
  const float inv_b = 1.0f / (float)nb;
  const int grp = threadIdx.x / L, lane = threadIdx.x % L;
  const int rib = blockIdx.x * RPB + grp;
  const int K = a.K, R = a.R, dp = a.dp;
  float4 zN[VPL], zE[VPL];
#pragma unroll
  for (int v = 0; v < VPL; v++) zN[v] = zE[v] = f4(0.f);
  float lrec = 0.f;
  if (rib < nb) {
    const int *ri = a.bidx + ((size_t)cb * a.B + rib) * R;
    const float *yt = a.btgt + ((size_t)cb * a.B + rib) * 3;
    const int *pos = a.inv + (size_t)cb * a.SB + (size_t)rib * R;
    const int ln = ri[0], le = ri[1], rn = ri[2], re = ri[3];
    int nnk[KMAX], nek[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      nnk[k] = k < K ? ri[4 + k] : 0;
      nek[k] = k < K ? ri[4 + K + k] : 0;
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
    const int act = a.act;
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
    head_loss(a.loss, y1, yt[0], l1, g1);
    head_loss(a.loss, y2, yt[1], l2, g2);
    head_loss(a.loss, y3, yt[2], l3, g3);
    lrec = l1 + l2 + l3;
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
      } else {
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
  }
  // padding-row partials and loss: reduce over the record groups
#pragma unroll
  for (int v = 0; v < VPL; v++) {
    s_z[0][grp][v * L + lane] = zN[v];
    s_z[1][grp][v * L + lane] = zE[v];
  }
  if (lane == 0) s_loss[grp] = lrec;
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * L * VPL; t += kTB) {
    const int tab = t / (L * VPL), j = t % (L * VPL);
    float4 s = f4(0.f);
    for (int g = 0; g < RPB; g++) s = s + s_z[tab][g][j];
    reinterpret_cast<float4 *>(a.gzero + ((size_t)blockIdx.x * 2 + tab) * dp)[j] = s;
  }
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int g = 0; g < RPB; g++) s += s_loss[g];
    a.lossbuf[(size_t)cb * a.nblk1 + blockIdx.x] = s;
  }
}

template <int L, int VPL>
__global__ __launch_bounds__(kTB) void train_update(TrainArgs a) {
  constexpr int GPB = kTB / L;
  const int cb = a.ctr[1];
  if (cb >= a.ctr[3]) return;
  const int U = a.ucount[cb];
  const int *ukey = a.ukey + (size_t)cb * a.SB;
  const int *uoff = a.uoff + (size_t)cb * (a.SB + 1);
  const int grp = threadIdx.x / L, lane = threadIdx.x % L;
  const int dp = a.dp;
  for (int it = blockIdx.x * GPB + grp; it < U + 2; it += gridDim.x * GPB) {
    float4 g[VPL];
#pragma unroll
    for (int v = 0; v < VPL; v++) g[v] = f4(0.f);
    int table, row;
    if (it < U) {
      const int key = ukey[it];
      table = key >> 30;
      row = key & 0x3fffffff;
      // this row's slot gradients are contiguous (prep sorted them)
      const int j1 = uoff[it + 1];
      for (int j = uoff[it]; j < j1; j++) {
        const float4 *p = reinterpret_cast<const float4 *>(a.gslot + (size_t)j * dp);
#pragma unroll
        for (int v = 0; v < VPL; v++) g[v] = g[v] + p[v * L + lane];
      }
    } else {
      table = it - U;
      row = 0;
      // padding row: one partial per K1 workgroup, 8 loads in flight
      const float4 *base = reinterpret_cast<const float4 *>(a.gzero + (size_t)table * dp);
      const size_t bstride = (size_t)2 * dp / 4;
      int b = 0;
      for (; b + 8 <= a.nblk1; b += 8) {
#pragma unroll
        for (int v = 0; v < VPL; v++) {
          float4 t[8];
#pragma unroll
          for (int q = 0; q < 8; q++) t[q] = base[(b + q) * bstride + v * L + lane];
#pragma unroll
          for (int q = 0; q < 8; q++) g[v] = g[v] + t[q];
        }
      }
      for (; b < a.nblk1; b++) {
#pragma unroll
        for (int v = 0; v < VPL; v++) g[v] = g[v] + base[b * bstride + v * L + lane];
      }
    }
    float4 *P = reinterpret_cast<float4 *>((table ? a.etab : a.ntab) + (size_t)row * dp);
    float4 *A = reinterpret_cast<float4 *>((table ? a.eacc : a.nacc) + (size_t)row * dp);
#pragma unroll
    for (int v = 0; v < VPL; v++) {
      const int j = v * L + lane;
      float4 p = P[j], ac = A[j];
      const float4 gg = g[v];
      float *pp = &p.x, *aa = &ac.x;
      const float *gv = &gg.x;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const float na = __fadd_rn(aa[c], __fmul_rn(gv[c], gv[c]));
        aa[c] = na;
        pp[c] = __fsub_rn(pp[c], __fdiv_rn(__fmul_rn(a.lr, gv[c]),
                                           __fadd_rn(sqrtf(na), a.eps)));
      }
      P[j] = p;
      A[j] = ac;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.ctr[0] = cb + 1;
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

// One workgroup per batch of the chunk: sorted unique (table,row) keys of
// the non-padding slots and, per key, its slot ids in ascending order.
__global__ __launch_bounds__(kTB) void train_prep(TrainArgs a, int64_t base,
                                                  int nbc, int P) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long s_key[];
  __shared__ int s_ws[kTB / 64];
  const int cb = blockIdx.x;
  if (cb >= nbc) return;
  const int64_t r0 = (base + cb) * a.B;
  const int nb = (int)min((int64_t)a.B, a.n - r0);
  const int R = a.R, K = a.K;
  const int S = nb * R;
  int *bidx = a.bidx + (size_t)cb * a.B * R;
  float *btgt = a.btgt + (size_t)cb * a.B * 3;
  for (int t = threadIdx.x; t < nb * 3; t += kTB) {
    const int i = t / 3;
    btgt[t] = a.tgt[(int64_t)a.perm[r0 + i] * 3 + (t - 3 * i)];
  }
  for (int t = threadIdx.x; t < P; t += kTB) {
    unsigned long long key = ~0ull;
    if (t < S) {
      const int i = t / R, s = t % R;
      const int rec = a.perm[r0 + i];
      const int row = a.idx[(int64_t)rec * R + s];
      bidx[t] = row;
      if (row != 0) {
        const unsigned k32 = ((unsigned)slot_is_edge(s, K) << 30) | (unsigned)row;
        key = ((unsigned long long)k32 << 32) | (unsigned)t;
      }
    }
    s_key[t] = key;
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
}

__global__ void set_ctr(int *ctr, int base, int nbc) {
  ctr[0] = 0;
  ctr[1] = 0;
  ctr[2] = base;
  ctr[3] = nbc;
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

using KFn = void (*)(TrainArgs);

template <int L, int VPL>
KFn fwd_for_k(int K) {
  if (K <= 2) return train_fwd_bwd<L, VPL, 2>;
  if (K <= 5) return train_fwd_bwd<L, VPL, 5>;
  if (K <= 8) return train_fwd_bwd<L, VPL, 8>;
  return train_fwd_bwd<L, VPL, 16>;
}

bool pick_kernels(int L, int VPL, int K, KFn &k1, KFn &k2) {
#define HGX_CASE(LL, VV)                                                     \
  if (L == LL && VPL == VV) {                                                \
    k1 = fwd_for_k<LL, VV>(K);                                               \
    k2 = train_update<LL, VV>;                                               \
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
  KFn k1 = nullptr, k2 = nullptr;
  HGX_CHECK(ctx, pick_kernels(L, VPL, K, k1, k2), HGX_EUNSUP,
            "no kernel for d=%d", ctx->d);
  const int RPB = kTB / L;
  const int nblk1 = (batch + RPB - 1) / RPB;
  const int GPB2 = kTB / L;
  const int grid2 = std::max(1, std::min(256, (SB + 2 + GPB2 - 1) / GPB2));
  const int64_t nbatches = (n + batch - 1) / batch;
  // chunk of batches whose unique-row lists are prepared together (<=~1 GB)
  const int64_t per_batch = (int64_t)SB * 4 + 3 * batch + 2;
  const int CB = (int)std::max<int64_t>(
      1, std::min<int64_t>(nbatches, (int64_t)(256ll << 20) / per_batch));

  // buffers
  HGX_TRY(hgx_ensure(ctx, ctx->s1, sizeof(int) * (n + 1)));              // perm
  HGX_TRY(hgx_ensure(ctx, ctx->s2, sizeof(float) * (size_t)SB * dp));    // gslot
  HGX_TRY(hgx_ensure(ctx, ctx->s3, sizeof(float) * (size_t)nblk1 * 2 * dp));
  HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(float) * (size_t)CB * nblk1 + 16));
  HGX_TRY(hgx_ensure(ctx, ctx->s5, sizeof(int) * ((size_t)CB * per_batch + 8)));
  HGX_TRY(hgx_ensure(ctx, ctx->s6, 64 + sizeof(double) * kLossBlocks));  // ctr, loss
  int *perm = ctx->s1.as<int>();
  int *prep = ctx->s5.as<int>();
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
  a.bidx = prep;                                         // CB*SB
  a.inv = prep + (size_t)CB * SB;                        // CB*SB
  a.ukey = prep + (size_t)CB * SB * 2;                   // CB*SB
  a.uoff = prep + (size_t)CB * SB * 3;                   // CB*(SB+1)
  a.btgt = reinterpret_cast<float *>(prep + (size_t)CB * (4 * (size_t)SB + 1));  // CB*B*3
  a.ucount = prep + (size_t)CB * (4 * (size_t)SB + 1 + 3 * (size_t)batch);      // CB
  a.ctr = ctx->s6.as<int>();
  double *dloss = reinterpret_cast<double *>(ctx->s6.as<char>() + 32);
  double *dpart = reinterpret_cast<double *>(ctx->s6.as<char>() + 64);
  a.SB = SB;
  a.nblk1 = nblk1;
  a.lr = lr;
  a.eps = eps;
  a.loss = loss;
  a.act = act;

  // shuffle scratch (device shuffle only)
  size_t sort_tmp = 0, sort_off = 0;
  unsigned long long *keys_in = nullptr, *keys_out = nullptr;
  int *vals_in = nullptr;
  if (!perms) {
    hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, keys_in, keys_out,
                                       vals_in, perm, (int)n);
    sort_off = (sizeof(unsigned long long) * 2 * n + sizeof(int) * n + 255) / 256 * 256;
    HGX_TRY(hgx_ensure(ctx, ctx->s7, sort_off + sort_tmp + 256));
    char *base = ctx->s7.as<char>();
    keys_in = reinterpret_cast<unsigned long long *>(base);
    keys_out = keys_in + n;
    vals_in = reinterpret_cast<int *>(keys_out + n);
  }

  // graph: kGraphBatches x [K1, K2]. HGX_NO_GRAPH=1 launches the same
  // kernels directly (profilers that mishandle graph replay).
  const int GB = (int)std::min<int64_t>(kGraphBatches, CB);
  const char *nog = getenv("HGX_NO_GRAPH");
  const bool use_graph = !(nog && nog[0] == '1');
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  if (use_graph) {
    HGX_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed));
    for (int b = 0; b < GB; b++) {
      hipLaunchKernelGGL(k1, dim3(nblk1), dim3(kTB), 0, ctx->stream, a);
      hipLaunchKernelGGL(k2, dim3(grid2), dim3(kTB), 0, ctx->stream, a);
    }
    hipError_t ce = hipStreamEndCapture(ctx->stream, &graph);
    if (ce != hipSuccess)
      return hgx_fail(ctx, HGX_EHIP, "graph capture failed: %s", hipGetErrorString(ce));
    ce = hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0);
    if (ce != hipSuccess) {
      hipGraphDestroy(graph);
      return hgx_fail(ctx, HGX_EHIP, "graph instantiate failed: %s", hipGetErrorString(ce));
    }
  }

  std::vector<int> hperm;
  // device time of the per-batch kernels only (K1+K2 replays), per chunk
  std::vector<hipEvent_t> bev;
  double batch_ms = 0.0;
  auto flush_events = [&]() {
    for (size_t i = 0; i + 1 < bev.size(); i += 2) {
      float m = 0.f;
      if (hipEventElapsedTime(&m, bev[i], bev[i + 1]) == hipSuccess) batch_ms += m;
    }
    for (hipEvent_t e : bev) hipEventDestroy(e);
    bev.clear();
  };
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
    hipMemsetAsync(dloss, 0, sizeof(double), ctx->stream);
    for (int64_t base = 0; base < nbatches; base += CB) {
      const int nbc = (int)std::min<int64_t>(CB, nbatches - base);
      hipLaunchKernelGGL(set_ctr, dim3(1), dim3(1), 0, ctx->stream, a.ctr,
                         (int)base, nbc);
      hipLaunchKernelGGL(train_prep, dim3(nbc), dim3(kTB),
                         (size_t)P * sizeof(unsigned long long), ctx->stream, a,
                         base, nbc, P);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      bev.push_back(e0);
      bev.push_back(e1);
      hipEventRecord(e0, ctx->stream);
      if (use_graph) {
        for (int g = 0; g < nbc; g += GB) {
          if (hipGraphLaunch(gexec, ctx->stream) != hipSuccess) {
            rc = hgx_fail(ctx, HGX_EHIP, "graph launch failed");
            break;
          }
        }
      } else {
        for (int g = 0; g < nbc; g++) {
          hipLaunchKernelGGL(k1, dim3(nblk1), dim3(kTB), 0, ctx->stream, a);
          hipLaunchKernelGGL(k2, dim3(grid2), dim3(kTB), 0, ctx->stream, a);
        }
      }
      hipEventRecord(e1, ctx->stream);
      if (rc) break;
      hipLaunchKernelGGL(loss_partial, dim3(kLossBlocks), dim3(kTB), 0,
                         ctx->stream, a.lossbuf, (int64_t)nbc * nblk1, dpart);
      hipLaunchKernelGGL(loss_final, dim3(1), dim3(kLossBlocks), 0,
                         ctx->stream, dpart, dloss);
    }
    if (rc) break;
    double lsum = 0.0;
    if (hipMemcpyAsync(&lsum, dloss, sizeof(double), hipMemcpyDeviceToHost,
                       ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
      rc = hgx_fail(ctx, HGX_EHIP, "epoch failed: %s",
                    hipGetErrorString(hipGetLastError()));
      break;
    }
    flush_events();
    const double cur = lsum / (double)n;
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
  flush_events();
  float ms = 0.f;
  hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1);
  if (gexec) hipGraphExecDestroy(gexec);
  if (graph) hipGraphDestroy(graph);
  if (rc) return rc;
  HGX_LAUNCH_CHECK(ctx);
  ctx->train_ms = batch_ms;
  ctx->train_epoch_ms = ms;
  ctx->train_records = (int64_t)ep * n;
  ctx->train_batches = (int64_t)ep * nbatches;
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
