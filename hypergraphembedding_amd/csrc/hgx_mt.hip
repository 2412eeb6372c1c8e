// numpy-seeded FOBE / HOBE sampling (rng = "mt19937"): the reference's
// record stream bit for bit, continuing numpy's global RandomState.
//
// Reference: hg2v_sample.py:49-51 (_sample_neighbors), :53-86
// (_sample_adj_matrix), :125-242 (BooleanSamples), :632-717
// (AlgebraicDistanceSamples with run_in_parallel=False: the node-edge
// neighbour draws run in the one forked Pool worker, i.e. on a copy of the
// parent's stream after its last pair draw; the parent's stream does not
// see them). Every draw the reference makes comes from numpy's global legacy
// RandomState (MT19937):
//   * np.random.choice(cols, m, replace=False) = cols[permutation(|cols|)
//     [:m]]: a reversed Fisher-Yates over arange(|cols|) with one
//     masked-rejection random_interval(i) per position i = |cols|-1 .. 1,
//     made whatever m is (also m = 0);
//   * np.random.choice(cols, K, replace=True) = cols[randint(0, |cols|, K)]
//     (masked-rejection bounded draws; none for |cols| = 1);
//   * np.random.randint(ncols, size=q) for the negatives (:73-75).
// The columns of a row of a pattern product (A A^T, A^T A, A A^T A,
// A^T A A^T, hg2v_sample.py:154,167,659,679,698,703) are in scipy's SMMP
// order (csr_matmat: the reverse of first discovery over the row's
// expansion, the product of a product expanded through the inner product's
// own SMMP rows); 1-hop rows (A, A^T) in CSR order.
//
// Host / device split. The MT19937 stream is sequential: how many 32-bit
// words a bounded draw consumes depends on the words themselves. The host
// walks the stream once, in the reference's order, and keeps only the
// accepted value of every bounded draw (~3 ns a draw). Everything that turns
// those values into records runs on the device, in parallel over rows:
//   * mt_smmp: the SMMP column order of every 2- / 3-hop row (one workgroup
//     per row: the first path reaching each column found with atomicMax of
//     ~path on a per-workgroup column slice, the first-discovery list
//     compacted by block scans; counted once for the offsets, then written);
//   * mt_fisher_yates: per row, the Fisher-Yates swaps of the row's draws and
//     the first m = min(q, |row|) columns;
//   * mt_emit / mt_neighbors: the SamplesToModelInput records (ids + 1) and
//     their neighbour columns; HOBE probabilities by hgx_hobe_fill_probs.
// What the host needs back: each pattern row's length (its draws' bounds)
// and the sampled node-edge pairs (the bounds of their neighbour draws).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <new>
#include <vector>

#include "hgx_internal.h"

int hgx_hobe_prepare(hgx_ctx *ctx);
int hgx_hobe_fill_probs(hgx_ctx *ctx, int kind, int64_t b, int64_t e);

namespace {

// ---- host: numpy's legacy RandomState stream (MT19937) ---------------------
constexpr int kMtN = 624, kMtM = 397;

struct Mt {
  uint32_t key[kMtN];  // numpy's state: the untempered key block
  int pos;
  uint32_t tw[kMtN];   // the block's tempered outputs (the draws' words)
};

void mt_twist(Mt &s) {
  uint32_t *m = s.key;
  auto mix = [](uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  };
  int i = 0;
  for (; i < kMtN - kMtM; i++) m[i] = mix(m[i], m[i + 1], m[i + kMtM]);
  for (; i < kMtN - 1; i++) m[i] = mix(m[i], m[i + 1], m[i + kMtM - kMtN]);
  m[kMtN - 1] = mix(m[kMtN - 1], m[0], m[kMtM - 1]);
  s.pos = 0;
}

// the tempered outputs of the current key block, all at once (vectorises)
void mt_temper(Mt &s) {
  for (int i = 0; i < kMtN; i++) {
    uint32_t y = s.key[i];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    s.tw[i] = y ^ (y >> 18);
  }
}

inline void mt_refill(Mt &s) {
  mt_twist(s);
  mt_temper(s);
}

inline uint32_t mt_next(Mt &s) {
  if (s.pos >= kMtN) mt_refill(s);
  return s.tw[s.pos++];
}

inline uint32_t mask_of(uint32_t v) {
  v |= v >> 1;
  v |= v >> 2;
  v |= v >> 4;
  v |= v >> 8;
  return v | (v >> 16);
}

// The draws random_interval(i) for i = hi, hi - 1, ..., lo, which share one
// mask (lo = 2^b <= hi < 2^(b+1)), appended to out: numpy's
// random_interval (masked rejection: the first word & mask <= i) one draw
// after another, without its data-dependent branch: every word is
// masked, stored at out and kept (out advances, i counts down) iff it is
// <= i; only the loop's exit is a branch. ~3x faster on the host.
inline void mt_interval_run(Mt &s, uint32_t hi, uint32_t lo, uint32_t mask,
                            uint32_t *&out) {
  uint32_t i = hi;
  while (i >= lo) {
    if (s.pos >= kMtN) mt_refill(s);
    const uint32_t *w = s.tw + s.pos;
    const int n = kMtN - s.pos;
    uint32_t *o = out;
    int j = 0;
    while (j < n && i >= lo) {
      const uint32_t v = w[j++] & mask;
      const uint32_t keep = v <= i;
      *o = v;
      o += keep;
      i -= keep;
    }
    out = o;
    s.pos += j;
  }
}

// a Fisher-Yates row of length L: random_interval(i), i = L-1 .. 1
inline void mt_permutation_draws(Mt &s, uint32_t L, uint32_t *&out) {
  uint32_t hi = L - 1;
  while (hi >= 1) {
    const uint32_t lo = 1u << (31 - __builtin_clz(hi));
    mt_interval_run(s, hi, lo, 2 * lo - 1, out);
    hi = lo - 1;
  }
}

// One masked-rejection draw (v = word & mask, first v <= max), looking at
// the next four words at once: the first acceptable one is picked by its
// bit (almost always one is: each word is accepted with probability
// > 1/2), so the data-dependent branch of the rejection loop becomes a
// well-predicted one. Same value, same words consumed.
inline uint32_t mt_bounded(Mt &s, uint32_t max, uint32_t mask) {
  if (s.pos + 4 <= kMtN) {
    const uint32_t *w = s.tw + s.pos;
    const uint32_t v[4] = {w[0] & mask, w[1] & mask, w[2] & mask, w[3] & mask};
    const unsigned ok = (unsigned)(v[0] <= max) | (unsigned)(v[1] <= max) << 1 |
                        (unsigned)(v[2] <= max) << 2 | (unsigned)(v[3] <= max) << 3;
    if (ok) {
      const int f = __builtin_ctz(ok);
      s.pos += f + 1;
      return v[f];
    }
    s.pos += 4;
  }
  uint32_t x;
  while ((x = (mt_next(s) & mask)) > max) {
  }
  return x;
}

// legacy randint(0, n), n <= 2^32 (masked bounded draw of rng = n - 1)
inline uint32_t mt_randint(Mt &s, uint64_t n) {
  const uint64_t rng = n - 1;
  if (rng == 0) return 0;
  if (rng == 0xffffffffull) return mt_next(s);
  return mt_bounded(s, (uint32_t)rng, mask_of((uint32_t)rng));
}

// ---- device ---------------------------------------------------------------
constexpr int kMB = 256;  // workgroup of the SMMP pass

struct Csr {
  const int *rp, *col;
};

__device__ int mt_scan_excl(int v, int *total, int *s_ws) {
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
#pragma unroll
  for (int w = 0; w < kMB / 64; w++) {
    const int x = s_ws[w];
    if (w < wave) base += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

__device__ __forceinline__ int mt_upper_find(const int *off, int n, int w) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= w) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// L1-bypassing accesses of the per-workgroup slices (written by atomics and
// by other waves of the workgroup)
__device__ __forceinline__ unsigned ld_agent(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_agent_i(const int *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned *p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent_i(int *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct SmmpShared {
  int ws[kMB / 64];
  int id[kMB], off[kMB];
  int base;  // reps found so far (mode 1)
};

enum WalkMode { W_MARK = 0, W_LIST = 1, W_CLEAR = 2 };

// One pass over the expansion of a source list through CSR B: path s runs
// over (i < ns, j < |B row src(i)|) in that order, reaching column
// c = B.col[B.rp[src(i)] + j]. F[c] holds ~(first path reaching c) (0 =
// unreached, so atomicMax keeps the smallest path).
//   W_MARK:  atomicMax(F[c], ~s)
//   W_LIST:  path s is c's first: out[rank] = c in path order (out may be
//            null: count only); returns the count
//   W_CLEAR: F[c] = 0 (the slice is clean for the next row)
// `src(i)` reads the source id: from a CSR row (ascending) or, for the
// 3-hop patterns, from the inner product's SMMP row (the reverse of its
// first-discovery list `mid`, L2 entries).
template <class Src>
__device__ int smmp_walk(const Src &src, int ns, Csr B, unsigned *F, int mode,
                         int *out, SmmpShared &S, int *err) {
  const int tid = threadIdx.x;
  unsigned sbase = 0;  // paths before this chunk
  if (tid == 0) S.base = 0;
  __syncthreads();
  for (int c1 = 0; c1 < ns; c1 += kMB) {
    const int i1 = c1 + tid;
    int id = -1, sz = 0;
    if (i1 < ns) {
      id = src(i1);
      sz = B.rp[id + 1] - B.rp[id];
    }
    int W;
    const int o = mt_scan_excl(sz, &W, S.ws);
    S.id[tid] = id;
    S.off[tid] = o;
    __syncthreads();
    const int n1 = min(kMB, ns - c1);
    if ((uint64_t)sbase + (uint64_t)W >= 0xfffffffeull) {
      if (tid == 0) atomicOr(err, 1);
      return 0;
    }
    for (int w0 = 0; w0 < W; w0 += kMB) {
      const int w = w0 + tid;
      int c = -1;
      if (w < W) {
        const int j = mt_upper_find(S.off, n1, w);
        const int m = S.id[j];
        c = B.col[B.rp[m] + (w - S.off[j])];
      }
      const unsigned ns_ = ~(sbase + (unsigned)w);
      if (mode == W_MARK) {
        if (c >= 0) atomicMax(&F[c], ns_);
      } else if (mode == W_CLEAR) {
        if (c >= 0) st_agent(&F[c], 0u);
      } else {
        const int rep = (c >= 0 && ld_agent(&F[c]) == ns_) ? 1 : 0;
        int tot;
        const int r = mt_scan_excl(rep, &tot, S.ws);
        if (rep && out) st_agent_i(&out[S.base + r], c);
        __syncthreads();
        if (tid == 0) S.base += tot;
        __syncthreads();
      }
    }
    sbase += (unsigned)W;
    __syncthreads();
  }
  const int found = S.base;  // read by every thread before the next walk resets it
  __syncthreads();
  return found;
}

struct CsrRow {
  const int *col;
  __device__ int operator()(int i) const { return col[i]; }
};
// the inner product's SMMP row: reverse of its first-discovery list
struct RevList {
  const int *list;
  int n;
  __device__ int operator()(int i) const { return ld_agent_i(&list[n - 1 - i]); }
};

struct SmmpArgs {
  int levels;  // 2: l1 -> l2; 3: (l1 -> l2) -> l3
  int nrows;
  Csr l1, l2, l3;
  int ncol_mid;        // column space of the 2-hop list (levels 3)
  int ncol;            // column space of the output
  unsigned *first_g;   // per workgroup: ncol_mid + ncol
  int *mid_g;          // per workgroup: ncol_mid (levels 3)
  int *len;            // count pass: row lengths
  const int64_t *coff; // write pass: row offsets into out (null: count pass)
  int *out;            // write pass: each row's columns in first-discovery order
  int *err;
};

__global__ __launch_bounds__(kMB) void mt_smmp(SmmpArgs A) {
  __shared__ SmmpShared S;
  const size_t slice = (size_t)(A.levels == 3 ? A.ncol_mid : 0) + A.ncol;
  unsigned *F2 = A.first_g + blockIdx.x * slice;
  unsigned *F = F2 + (A.levels == 3 ? A.ncol_mid : 0);
  int *mid = A.levels == 3 ? A.mid_g + (size_t)blockIdx.x * A.ncol_mid : nullptr;
  for (int r = blockIdx.x; r < A.nrows; r += gridDim.x) {
    const int b1 = A.l1.rp[r], n1 = A.l1.rp[r + 1] - b1;
    int *out = A.coff ? A.out + A.coff[r] : nullptr;
    int L = 0;
    if (A.levels == 2) {
      const CsrRow src{A.l1.col + b1};
      smmp_walk(src, n1, A.l2, F, W_MARK, nullptr, S, A.err);
      L = smmp_walk(src, n1, A.l2, F, W_LIST, out, S, A.err);
      smmp_walk(src, n1, A.l2, F, W_CLEAR, nullptr, S, A.err);
    } else {
      const CsrRow src{A.l1.col + b1};
      smmp_walk(src, n1, A.l2, F2, W_MARK, nullptr, S, A.err);
      const int L2 = smmp_walk(src, n1, A.l2, F2, W_LIST, mid, S, A.err);
      smmp_walk(src, n1, A.l2, F2, W_CLEAR, nullptr, S, A.err);
      const RevList src2{mid, L2};
      smmp_walk(src2, L2, A.l3, F, W_MARK, nullptr, S, A.err);
      L = smmp_walk(src2, L2, A.l3, F, W_LIST, out, S, A.err);
      smmp_walk(src2, L2, A.l3, F, W_CLEAR, nullptr, S, A.err);
    }
    if (!A.coff && threadIdx.x == 0) A.len[r] = L;
    __syncthreads();
  }
}

// Per row r (one lane): arr = arange(L); for i = L-1 .. 1 swap arr[i] and
// arr[d_i] (d = the row's accepted random_interval(i) values, in stream
// order); the first m = min(q, L) positions name the chosen columns: the
// SMMP column at position p is the first-discovery list's entry L-1-p
// (asc != null), or the CSR row's entry p.
__global__ void mt_fisher_yates(int nrows, const int *len, const int *quota,
                                const int64_t *doff, const uint32_t *D,
                                const int64_t *coff, int *arr, const int *asc,
                                Csr one, const int64_t *roff, int *out) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < nrows;
       r += gridDim.x * blockDim.x) {
    const int L = len[r];
    const int m = min(quota[r], L);
    if (m <= 0) continue;
    int *a = arr + coff[r];
    for (int i = 0; i < L; i++) a[i] = i;
    const uint32_t *d = D + doff[r];
    for (int i = L - 1; i >= 1; i--) {
      const int j = (int)d[L - 1 - i];
      const int t = a[j];
      a[j] = a[i];
      a[i] = t;
    }
    int *o = out + roff[r];
    for (int t = 0; t < m; t++) {
      const int p = a[t];
      o[t] = asc ? asc[coff[r] + L - 1 - p] : one.col[one.rp[r] + p];
    }
  }
}

using hgx::REC_NN;
using hgx::REC_EE;
using hgx::REC_NE_NODE;
using hgx::REC_NE_EDGE;

// records base + roff[r] + t of row r: (row, cols[roff[r] + t]) in the
// kind's id columns, target `prob` in the kind's slot
__global__ void mt_emit(int kind, int nrows, const int64_t *roff, const int *cols,
                        int64_t base, int R, int *idx, float *tgt, float prob) {
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int64_t b = roff[r], m = roff[r + 1] - b;
    for (int64_t t = threadIdx.x; t < m; t += blockDim.x) {
      const int64_t rec = base + b + t;
      int *ri = idx + rec * R;
      for (int s = 0; s < R; s++) ri[s] = 0;
      const int c = cols[b + t];
      if (kind == REC_NN) { ri[0] = r + 1; ri[2] = c + 1; }
      else if (kind == REC_EE) { ri[1] = r + 1; ri[3] = c + 1; }
      else if (kind == REC_NE_NODE) { ri[0] = r + 1; ri[3] = c + 1; }
      else { ri[0] = c + 1; ri[3] = r + 1; }
      float *tt = tgt + rec * 3;
      tt[0] = tt[1] = tt[2] = 0.f;
      tt[kind == REC_NN ? 0 : kind == REC_EE ? 1 : 2] = prob;
    }
  }
}

// neighbour columns of node-edge records [b, b + n): per record 2K accepted
// draws, K edges of its node (positions in A's row) then K nodes of its
// edge (positions in A^T's row) (hg2v_sample.py:184-187, 604-605)
__global__ void mt_neighbors(int64_t b, int64_t n, int K, int R, int *idx,
                             const uint32_t *vals, Csr A, Csr AT) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    int *ri = idx + (b + t) * R;
    const int v = ri[0] - 1, e = ri[3] - 1;
    const uint32_t *x = vals + t * 2 * K;
    for (int k = 0; k < K; k++) {
      ri[4 + K + k] = A.col[A.rp[v] + (int)x[k]] + 1;
      ri[4 + k] = AT.col[AT.rp[e] + (int)x[K + k]] + 1;
    }
  }
}

int grid_of(int64_t work, int per, int cap = 65536) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((work + per - 1) / per, cap));
}

// host vector -> device buffer; complete on return (callers' vectors are
// often locals that die right after)
template <class T>
int upload(hgx_ctx *ctx, DevBuf &b, const std::vector<T> &h) {
  HGX_TRY(hgx_ensure(ctx, b, sizeof(T) * (h.size() + 1)));
  if (!h.empty()) {
    HGX_HIP(ctx, hipMemcpyAsync(b.p, h.data(), sizeof(T) * h.size(),
                                hipMemcpyHostToDevice, ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return HGX_OK;
}

enum MtPattern { P_A = 0, P_AT, P_NN, P_EE, P_NNE, P_EEN };

// entries (= draws + rows) of one pattern held at once: 8.6e9 x 12 B of
// device memory and 34 GB of host memory at most
constexpr int64_t kMaxPatternEntries = int64_t(1) << 33;

// One pattern's sample: per row the chosen columns (packed by roff) on the
// device, plus what the host knows (row lengths, counts).
struct MtPat {
  int pattern = 0, nrows = 0;
  std::vector<int> len;
  std::vector<int64_t> roff;  // nrows + 1: exclusive scan of min(q, len)
  DevBuf dlen, droff, cols;
  int64_t total() const { return roff.empty() ? 0 : roff.back(); }
  ~MtPat() {
    hgx_release(dlen);
    hgx_release(droff);
    hgx_release(cols);
  }
};

struct MtRun {
  hgx_ctx *ctx;
  std::vector<int> rp_n, rp_e;  // host copies of the row pointers
  Csr A, AT;
};

// The SMMP pass of a 2- / 3-hop pattern: with coff null the row lengths
// (into dlen), else the rows' first-discovery column lists packed by coff
// (into asc).
int smmp_pass(MtRun &M, const MtPat &p, int *dlen, const int64_t *coff, int *asc) {
  hgx_ctx *ctx = M.ctx;
  const int N = ctx->N, E = ctx->E;
  SmmpArgs a{};
  a.nrows = p.nrows;
  switch (p.pattern) {
    case P_NN: a.levels = 2; a.l1 = M.A; a.l2 = M.AT; a.ncol = N; break;
    case P_EE: a.levels = 2; a.l1 = M.AT; a.l2 = M.A; a.ncol = E; break;
    case P_NNE:
      a.levels = 3; a.l1 = M.A; a.l2 = M.AT; a.l3 = M.A; a.ncol_mid = N; a.ncol = E;
      break;
    default:
      a.levels = 3; a.l1 = M.AT; a.l2 = M.A; a.l3 = M.AT; a.ncol_mid = E; a.ncol = N;
      break;
  }
  // per-workgroup column slices, <= ~2 GB in all
  const size_t fwords = (size_t)a.ncol_mid + a.ncol;
  const size_t per_wg = sizeof(unsigned) * fwords + sizeof(int) * (size_t)a.ncol_mid;
  int nwg = 1024;
  while (nwg > 32 && (double)nwg * per_wg > 2e9) nwg /= 2;
  nwg = std::max(1, std::min(nwg, p.nrows));
  DevBuf first, mid, err;
  auto done = [&](int rc) {
    hgx_release(first);
    hgx_release(mid);
    hgx_release(err);
    return rc;
  };
  int rc;
  if ((rc = hgx_ensure(ctx, first, sizeof(unsigned) * nwg * fwords + 16)) ||
      (rc = hgx_ensure(ctx, mid, sizeof(int) * nwg * (size_t)a.ncol_mid + 16)) ||
      (rc = hgx_ensure(ctx, err, 16)))
    return done(rc);
  a.first_g = first.as<unsigned>();
  a.mid_g = mid.as<int>();
  a.len = dlen;
  a.coff = coff;
  a.out = asc;
  a.err = err.as<int>();
  int e = 0;
  if (hipMemsetAsync(first.p, 0, sizeof(unsigned) * nwg * fwords, ctx->stream) != hipSuccess ||
      hipMemsetAsync(err.p, 0, 16, ctx->stream) != hipSuccess)
    return done(hgx_fail(ctx, HGX_EHIP, "SMMP pass setup failed"));
  if (p.nrows > 0) {
    hipLaunchKernelGGL(mt_smmp, dim3(nwg), dim3(kMB), 0, ctx->stream, a);
    if (hipGetLastError() != hipSuccess)
      return done(hgx_fail(ctx, HGX_EHIP, "mt_smmp launch failed"));
  }
  if (hipMemcpyAsync(&e, err.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return done(hgx_fail(ctx, HGX_EHIP, "SMMP pass failed"));
  if (e) return done(hgx_fail(ctx, HGX_EUNSUP, "a pattern row's expansion exceeds 2^32 - 2 paths"));
  return done(HGX_OK);
}

// row lengths of a pattern: A / A^T from the row pointers, 2- / 3-hop by
// the device's count pass
int pattern_lengths(MtRun &M, MtPat &p) {
  hgx_ctx *ctx = M.ctx;
  p.nrows = (p.pattern == P_A || p.pattern == P_NN || p.pattern == P_NNE) ? ctx->N : ctx->E;
  p.len.assign(p.nrows, 0);
  if (p.pattern == P_A || p.pattern == P_AT) {
    const std::vector<int> &rp = p.pattern == P_A ? M.rp_n : M.rp_e;
    for (int r = 0; r < p.nrows; r++) p.len[r] = rp[r + 1] - rp[r];
    return upload(ctx, p.dlen, p.len);
  }
  HGX_TRY(hgx_ensure(ctx, p.dlen, sizeof(int) * (p.nrows + 1)));
  HGX_TRY(smmp_pass(M, p, p.dlen.as<int>(), nullptr, nullptr));
  HGX_HIP(ctx, hipMemcpyAsync(p.len.data(), p.dlen.p, sizeof(int) * p.nrows,
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

// Pattern p with per-row quotas q: its draws from `st` (host), then the
// device's SMMP lists + Fisher-Yates -> p.cols / p.roff.
int sample_pattern(MtRun &M, MtPat &p, Mt &st, const std::vector<int> &q) {
  hgx_ctx *ctx = M.ctx;
  HGX_TRY(pattern_lengths(M, p));
  const int R = p.nrows;
  // host: every row with |row| > 1 draws random_interval(i), i = |row|-1..1
  std::vector<int64_t> doff(R + 1), coff(R + 1);
  p.roff.assign(R + 1, 0);
  for (int r = 0; r < R; r++) {
    const int L = p.len[r];
    doff[r + 1] = doff[r] + std::max(L - 1, 0);
    coff[r + 1] = coff[r] + L;
    p.roff[r + 1] = p.roff[r] + std::min(q[r], L);
  }
  // every draw of the pattern is held on the host, then on the device with
  // the rows' column lists and Fisher-Yates scratch (12 B per draw): the
  // mode is for the graphs the reference itself can sample (C4's 2-hop
  // patterns have ~1e12 entries)
  HGX_CHECK(ctx, coff[R] <= kMaxPatternEntries, HGX_EUNSUP,
            "rng=mt19937: pattern %d has %lld entries, above the %lld this mode "
            "holds (the reference materialises the same rows)",
            p.pattern, (long long)coff[R], (long long)kMaxPatternEntries);
  // (one slack word: mt_interval_run stores every word it looks at)
  std::vector<uint32_t> D((size_t)doff[R] + 1);
  uint32_t *dp = D.data();
  for (int r = 0; r < R; r++)
    if (p.len[r] > 1) mt_permutation_draws(st, (uint32_t)p.len[r], dp);
  D.pop_back();
  const bool hop1 = p.pattern == P_A || p.pattern == P_AT;
  DevBuf dD, ddoff, dcoff, dq, arr, asc;
  auto done = [&](int rc) {
    for (DevBuf *b : {&dD, &ddoff, &dcoff, &dq, &arr, &asc}) hgx_release(*b);
    return rc;
  };
  int rc;
  if ((rc = upload(ctx, dD, D)) || (rc = upload(ctx, ddoff, doff)) ||
      (rc = upload(ctx, dcoff, coff)) || (rc = upload(ctx, dq, q)) ||
      (rc = upload(ctx, p.droff, p.roff)) ||
      (rc = hgx_ensure(ctx, arr, sizeof(int) * (size_t)(coff[R] + 1))) ||
      (rc = hgx_ensure(ctx, p.cols, sizeof(int) * (size_t)(p.total() + 1))))
    return done(rc);
  if (!hop1) {
    if ((rc = hgx_ensure(ctx, asc, sizeof(int) * (size_t)(coff[R] + 1))) ||
        (rc = smmp_pass(M, p, nullptr, dcoff.as<int64_t>(), asc.as<int>())))
      return done(rc);
  }
  const Csr one = p.pattern == P_A ? M.A : M.AT;
  hipLaunchKernelGGL(mt_fisher_yates, dim3(grid_of(R, 64)), dim3(64), 0, ctx->stream, R,
                     p.dlen.as<int>(), dq.as<int>(), ddoff.as<int64_t>(), dD.as<uint32_t>(),
                     dcoff.as<int64_t>(), arr.as<int>(), hop1 ? nullptr : asc.as<int>(), one,
                     p.droff.as<int64_t>(), p.cols.as<int>());
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess)
    return done(hgx_fail(ctx, HGX_EHIP, "Fisher-Yates pass failed"));
  return done(HGX_OK);
}

// Negatives (hg2v_sample.py:73-75): q[r] draws randint(ncols) per row, all
// on the host (the accepted values are the columns).
int sample_negatives(MtRun &M, MtPat &p, Mt &st, const std::vector<int> &q, int ncols) {
  p.nrows = (int)q.size();
  p.roff.assign(p.nrows + 1, 0);
  for (int r = 0; r < p.nrows; r++) p.roff[r + 1] = p.roff[r] + q[r];
  std::vector<int> cols((size_t)p.total());
  size_t k = 0;
  for (int r = 0; r < p.nrows; r++)
    for (int t = 0; t < q[r]; t++) cols[k++] = (int)mt_randint(st, (uint64_t)ncols);
  HGX_TRY(upload(M.ctx, p.droff, p.roff));
  HGX_TRY(upload(M.ctx, p.cols, cols));
  return HGX_OK;
}

int emit(MtRun &M, int kind, const MtPat &p, int64_t base, float prob) {
  hgx_ctx *ctx = M.ctx;
  if (p.total() == 0) return HGX_OK;
  hipLaunchKernelGGL(mt_emit, dim3(grid_of(p.nrows, 1)), dim3(64), 0, ctx->stream, kind,
                     p.nrows, p.droff.as<int64_t>(), p.cols.as<int>(), base, 4 + 2 * ctx->K,
                     ctx->rec_idx.as<int>(), ctx->rec_tgt.as<float>(), prob);
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

// (v, e) of every record of the node-edge blocks `nr` (node rows) then `er`
// (edge rows, swapped), in record order
int ne_pairs(MtRun &M, const MtPat &nr, const MtPat &er, std::vector<int> &v,
             std::vector<int> &e) {
  hgx_ctx *ctx = M.ctx;
  const int64_t n1 = nr.total(), n2 = er.total();
  v.resize(n1 + n2);
  e.resize(n1 + n2);
  std::vector<int> c1(n1), c2(n2);
  if (n1)
    HGX_HIP(ctx, hipMemcpyAsync(c1.data(), nr.cols.p, sizeof(int) * n1, hipMemcpyDeviceToHost,
                                ctx->stream));
  if (n2)
    HGX_HIP(ctx, hipMemcpyAsync(c2.data(), er.cols.p, sizeof(int) * n2, hipMemcpyDeviceToHost,
                                ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (int r = 0; r < nr.nrows; r++)
    for (int64_t t = nr.roff[r]; t < nr.roff[r + 1]; t++) {
      v[t] = r;
      e[t] = c1[t];
    }
  for (int r = 0; r < er.nrows; r++)
    for (int64_t t = er.roff[r]; t < er.roff[r + 1]; t++) {
      v[n1 + t] = c2[t];
      e[n1 + t] = r;
    }
  return HGX_OK;
}

// _sample_neighbors of records [b, b + |v|): K randint(deg v) then K
// randint(|e|) per record, in record order, from `st`; written on device
int neighbors(MtRun &M, int64_t b, const std::vector<int> &v, const std::vector<int> &e,
              Mt &st) {
  hgx_ctx *ctx = M.ctx;
  const int K = ctx->K;
  const int64_t n = (int64_t)v.size();
  if (n == 0) return HGX_OK;
  std::vector<uint32_t> vals((size_t)n * 2 * K);
  for (int64_t t = 0; t < n; t++) {
    const int dv = M.rp_n[v[t] + 1] - M.rp_n[v[t]];
    const int de = M.rp_e[e[t] + 1] - M.rp_e[e[t]];
    HGX_CHECK(ctx, dv > 0 && de > 0, HGX_EVALUE,
              "a cannot be empty unless no samples are taken (_sample_neighbors "
              "on a node without edges or an edge without nodes, "
              "hg2v_sample.py:49-51)");
    uint32_t *x = vals.data() + t * 2 * K;
    for (int k = 0; k < K; k++) x[k] = mt_randint(st, (uint64_t)dv);
    for (int k = 0; k < K; k++) x[K + k] = mt_randint(st, (uint64_t)de);
  }
  DevBuf dv;
  int rc = upload(ctx, dv, vals);
  if (rc == HGX_OK) {
    hipLaunchKernelGGL(mt_neighbors, dim3(grid_of(n, 256)), dim3(256), 0, ctx->stream, b, n, K,
                       4 + 2 * K, ctx->rec_idx.as<int>(), dv.as<uint32_t>(), M.A, M.AT);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess)
      rc = hgx_fail(ctx, HGX_EHIP, "neighbour pass failed");
  }
  hgx_release(dv);
  return rc;
}

int mt_begin(hgx_ctx *ctx, MtRun &M, const uint32_t *key, const int32_t *pos, Mt &st, int K) {
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, key && pos, HGX_EINVAL, "null MT19937 state");
  HGX_CHECK(ctx, *pos >= 0 && *pos <= kMtN, HGX_EINVAL, "MT19937 position %d outside [0, 624]",
            *pos);
  HGX_CHECK(ctx, K >= 1 && K <= 16, HGX_EUNSUP, "num_neighbors %d outside [1,16]", K);
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  std::copy(key, key + kMtN, st.key);
  st.pos = *pos;
  mt_temper(st);  // the words left in numpy's current block
  M.ctx = ctx;
  M.rp_n.resize(ctx->N + 1);
  M.rp_e.resize(ctx->E + 1);
  HGX_HIP(ctx, hipMemcpyAsync(M.rp_n.data(), ctx->rp_n.p, sizeof(int) * (ctx->N + 1),
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(M.rp_e.data(), ctx->rp_e.p, sizeof(int) * (ctx->E + 1),
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  M.A = Csr{ctx->rp_n.as<int>(), ctx->col_n.as<int>()};
  M.AT = Csr{ctx->rp_e.as<int>(), ctx->col_e.as<int>()};
  ctx->sample_union_rows = ctx->sample_fallback_rows = ctx->sample_uniform_rows = 0;
  return HGX_OK;
}

int mt_alloc(hgx_ctx *ctx, int64_t n, int K) {
  const int R = 4 + 2 * K;
  HGX_CHECK(ctx, n < (int64_t)INT32_MAX, HGX_EUNSUP,
            "%lld records exceed the 2^31 record limit", (long long)n);
  HGX_TRY(hgx_ensure(ctx, ctx->rec_idx, sizeof(int32_t) * (n * R + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->rec_tgt, sizeof(float) * (n * 3 + 1)));
  ctx->n_rec = n;
  ctx->K = K;
  ctx->rec_in_order = false;
  ctx->store_carry = 0;
  // not a keyed sampler stream: the record store cannot re-derive its
  // neighbour draws, so hgx_store_append refuses it
  ctx->smp_family = -1;
  return HGX_OK;
}

std::vector<int> quota_vec(const int32_t *q, int n) { return std::vector<int>(q, q + n); }

int check_quota(hgx_ctx *ctx, const int32_t *q, int n, const char *what) {
  HGX_CHECK(ctx, q, HGX_EINVAL, "%s quota is null", what);
  for (int i = 0; i < n; i++)
    HGX_CHECK(ctx, q[i] >= 0, HGX_EINVAL, "%s quota[%d] < 0", what, i);
  return HGX_OK;
}

void put_state(const Mt &st, uint32_t *key, int32_t *pos) {
  std::copy(st.key, st.key + kMtN, key);
  *pos = st.pos;
}

}  // namespace

static int hgx_sample_fobe_mt_impl(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                                  const int32_t *node_quota, const int32_t *edge_quota,
                                  const int32_t *neg_node_quota,
                                  const int32_t *neg_edge_quota, int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  MtRun M;
  Mt st;
  HGX_TRY(mt_begin(ctx, M, mt_key, mt_pos, st, K));
  HGX_CHECK(ctx, (neg_node_quota == nullptr) == (neg_edge_quota == nullptr), HGX_EINVAL,
            "give both negative quotas or neither");
  HGX_TRY(check_quota(ctx, node_quota, ctx->N, "node"));
  HGX_TRY(check_quota(ctx, edge_quota, ctx->E, "edge"));
  if (neg_node_quota) {
    HGX_TRY(check_quota(ctx, neg_node_quota, ctx->N, "negative node"));
    HGX_TRY(check_quota(ctx, neg_edge_quota, ctx->E, "negative edge"));
  }
  const std::vector<int> qn = quota_vec(node_quota, ctx->N), qe = quota_vec(edge_quota, ctx->E);
  // BooleanSamples (hg2v_sample.py:156-194): nn, ee, node-edge of node rows,
  // of edge rows (swapped), then their neighbour draws
  MtPat nn, ee, ne_n, ne_e;
  nn.pattern = P_NN;
  ee.pattern = P_EE;
  ne_n.pattern = P_A;
  ne_e.pattern = P_AT;
  HGX_TRY(sample_pattern(M, nn, st, qn));
  HGX_TRY(sample_pattern(M, ee, st, qe));
  HGX_TRY(sample_pattern(M, ne_n, st, qn));
  HGX_TRY(sample_pattern(M, ne_e, st, qe));
  std::vector<int> pv, pe;
  HGX_TRY(ne_pairs(M, ne_n, ne_e, pv, pe));
  const int64_t o_ee = nn.total(), o_ne = o_ee + ee.total();
  const int64_t o_en = o_ne + ne_n.total(), o_neg = o_en + ne_e.total();
  // negatives (:198-240): nn, ee, the repeated ee block (:215-221), node-edge
  // of node rows, of edge rows; their counts are the quotas
  std::vector<int> gqn, gqe;
  int64_t sn = 0, se = 0;
  if (neg_node_quota) {
    gqn = quota_vec(neg_node_quota, ctx->N);
    gqe = quota_vec(neg_edge_quota, ctx->E);
    for (int x : gqn) sn += x;
    for (int x : gqe) se += x;
  }
  const int64_t o_gee = o_neg + sn, o_gee2 = o_gee + se, o_gne = o_gee2 + se;
  const int64_t o_gen = o_gne + sn, total = o_gen + se;
  HGX_TRY(mt_alloc(ctx, total, K));
  HGX_TRY(emit(M, REC_NN, nn, 0, 1.f));
  HGX_TRY(emit(M, REC_EE, ee, o_ee, 1.f));
  HGX_TRY(emit(M, REC_NE_NODE, ne_n, o_ne, 1.f));
  HGX_TRY(emit(M, REC_NE_EDGE, ne_e, o_en, 1.f));
  HGX_TRY(neighbors(M, o_ne, pv, pe, st));
  if (neg_node_quota) {
    // after the positives' neighbour draws in the stream
    MtPat gnn, gee, gee2, gne_n, gne_e;
    HGX_TRY(sample_negatives(M, gnn, st, gqn, ctx->N));
    HGX_TRY(sample_negatives(M, gee, st, gqe, ctx->E));
    HGX_TRY(sample_negatives(M, gee2, st, gqe, ctx->E));
    HGX_TRY(sample_negatives(M, gne_n, st, gqn, ctx->E));
    HGX_TRY(sample_negatives(M, gne_e, st, gqe, ctx->N));
    HGX_TRY(emit(M, REC_NN, gnn, o_neg, 0.f));
    HGX_TRY(emit(M, REC_EE, gee, o_gee, 0.f));
    HGX_TRY(emit(M, REC_EE, gee2, o_gee2, 0.f));
    HGX_TRY(emit(M, REC_NE_NODE, gne_n, o_gne, 0.f));
    HGX_TRY(emit(M, REC_NE_EDGE, gne_e, o_gen, 0.f));
    std::vector<int> gv, ge;
    HGX_TRY(ne_pairs(M, gne_n, gne_e, gv, ge));
    HGX_TRY(neighbors(M, o_gne, gv, ge, st));
    const int64_t b[10] = {0, o_ee, o_ne, o_en, o_neg, o_gee, o_gee2, o_gne, o_gen, total};
    for (int i = 0; i <= 9; i++) ctx->rec_bounds[i] = b[i];
    ctx->n_rec_blocks = 9;
  } else {
    const int64_t b[5] = {0, o_ee, o_ne, o_en, total};
    for (int i = 0; i <= 4; i++) ctx->rec_bounds[i] = b[i];
    ctx->n_rec_blocks = 4;
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  put_state(st, mt_key, mt_pos);
  if (n_records) *n_records = total;
  return HGX_OK;
}

extern "C" int hgx_sample_fobe_mt(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                                  const int32_t *node_quota, const int32_t *edge_quota,
                                  const int32_t *neg_node_quota,
                                  const int32_t *neg_edge_quota, int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  try {
    return hgx_sample_fobe_mt_impl(ctx, mt_key, mt_pos, K, node_quota, edge_quota,
                                   neg_node_quota, neg_edge_quota, n_records);
  } catch (const std::bad_alloc &) {
    return hgx_fail(ctx, HGX_ENOMEM, "rng=mt19937: host allocation failed");
  }
}

namespace {

// AlgebraicDistanceSamples / WeightedJaccardSamples (run_in_parallel=False)
// pair blocks drawing the stream: nn, ee, A A^T A of node rows, A^T A A^T of
// edge rows (swapped) in the parent (hg2v_sample.py:658-705, 432-503), the
// records emitted with targets 0, then the node-edge neighbour draws on the
// forked worker's copy of the stream (:604-605, 371-372): `st` stays the
// parent's. off = block bounds {0, o_ee, o_ne, o_en, total}.
int pairs4_mt(MtRun &M, Mt &st, const std::vector<int> &qn, const std::vector<int> &qe,
              int K, int64_t off[5]) {
  hgx_ctx *ctx = M.ctx;
  MtPat nn, ee, ne_n, ne_e;
  nn.pattern = P_NN;
  ee.pattern = P_EE;
  ne_n.pattern = P_NNE;
  ne_e.pattern = P_EEN;
  HGX_TRY(sample_pattern(M, nn, st, qn));
  HGX_TRY(sample_pattern(M, ee, st, qe));
  HGX_TRY(sample_pattern(M, ne_n, st, qn));
  HGX_TRY(sample_pattern(M, ne_e, st, qe));
  std::vector<int> pv, pe;
  HGX_TRY(ne_pairs(M, ne_n, ne_e, pv, pe));
  off[0] = 0;
  off[1] = nn.total();
  off[2] = off[1] + ee.total();
  off[3] = off[2] + ne_n.total();
  off[4] = off[3] + ne_e.total();
  HGX_TRY(mt_alloc(ctx, off[4], K));
  HGX_TRY(emit(M, REC_NN, nn, off[0], 0.f));
  HGX_TRY(emit(M, REC_EE, ee, off[1], 0.f));
  HGX_TRY(emit(M, REC_NE_NODE, ne_n, off[2], 0.f));
  HGX_TRY(emit(M, REC_NE_EDGE, ne_e, off[3], 0.f));
  Mt worker = st;
  HGX_TRY(neighbors(M, off[2], pv, pe, worker));
  for (int i = 0; i <= 4; i++) ctx->rec_bounds[i] = off[i];
  ctx->n_rec_blocks = 4;
  return HGX_OK;
}

}  // namespace

int hgx_jaccard_fill(hgx_ctx *ctx, int64_t o_ee, int64_t o_ne, int64_t total);

static int hgx_sample_hobe_mt_impl(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                                  int S, int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  MtRun M;
  Mt st;
  HGX_TRY(mt_begin(ctx, M, mt_key, mt_pos, st, K));
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE, "HOBE needs the algebraic-distance coords on device");
  HGX_CHECK(ctx, S >= 0, HGX_EINVAL, "num_samples must be >= 0 (hg2v_sample.py:647)");
  // AlgebraicDistanceSamples: quota S on every row (hg2v_sample.py:659-703)
  const std::vector<int> qn(ctx->N, S), qe(ctx->E, S);
  int64_t off[5];
  HGX_TRY(pairs4_mt(M, st, qn, qe, K, off));
  HGX_TRY(hgx_hobe_prepare(ctx));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 0, off[0], off[1]));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 1, off[1], off[2]));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 2, off[2], off[4]));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  put_state(st, mt_key, mt_pos);
  if (n_records) *n_records = off[4];
  return HGX_OK;
}

extern "C" int hgx_sample_hobe_mt(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                                  int S, int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  try {
    return hgx_sample_hobe_mt_impl(ctx, mt_key, mt_pos, K, S, n_records);
  } catch (const std::bad_alloc &) {
    return hgx_fail(ctx, HGX_ENOMEM, "rng=mt19937: host allocation failed");
  }
}

static int hgx_sample_jaccard_mt_impl(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                                     const int32_t *node_quota, const int32_t *edge_quota,
                                     int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  MtRun M;
  Mt st;
  HGX_TRY(mt_begin(ctx, M, mt_key, mt_pos, st, K));
  HGX_CHECK(ctx, ctx->features_ok, HGX_ESTATE, "hgx_features_set not called");
  HGX_TRY(check_quota(ctx, node_quota, ctx->N, "node"));
  HGX_TRY(check_quota(ctx, edge_quota, ctx->E, "edge"));
  // WeightedJaccardSamples: quotas int(weight * S) (hg2v_sample.py:419-422)
  int64_t off[5];
  HGX_TRY(pairs4_mt(M, st, quota_vec(node_quota, ctx->N), quota_vec(edge_quota, ctx->E), K,
                    off));
  HGX_TRY(hgx_jaccard_fill(ctx, off[1], off[2], off[4]));
  put_state(st, mt_key, mt_pos);
  if (n_records) *n_records = off[4];
  return HGX_OK;
}

extern "C" int hgx_sample_jaccard_mt(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                                     const int32_t *node_quota, const int32_t *edge_quota,
                                     int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  try {
    return hgx_sample_jaccard_mt_impl(ctx, mt_key, mt_pos, K, node_quota, edge_quota, n_records);
  } catch (const std::bad_alloc &) {
    return hgx_fail(ctx, HGX_ENOMEM, "rng=mt19937: host allocation failed");
  }
}
