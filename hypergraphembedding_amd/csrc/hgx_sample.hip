// FOBE / HOBE samplers on MI355X.
//
// Reference: hg2v_sample.py:53-86 (_sample_adj_matrix: per row, min(q, |row|)
// DISTINCT columns uniformly without replacement, or q uniform columns with
// replacement for negatives), :49-51 (_sample_neighbors: K draws with
// replacement), :125-242 (BooleanSamples), :632-717 (AlgebraicDistanceSamples),
// :751-797 (SamplesToModelInput layout, ids +1, 0 = absent).
//
// The reference samples rows of explicit sparse products (A*A^T, A^T*A,
// A*A^T*A, A^T*A*A^T built with scipy SpGEMM). Here no product is
// materialised: one workgroup per row walks the 1/2/3-hop CSR expansion
// with LDS block scans + binary search (one path endpoint per thread),
// de-duplicates endpoints with a test-and-set bitmap (LDS when the column
// space fits, else a per-workgroup slice in HBM) into a distinct list, and
// picks an exactly uniform m-subset (m = min(q, distinct)) as the m smallest
// 64-bit keys (hash(seed,row,col) << 32 | col) by an 8-pass LDS radix
// select. The chosen columns are written sorted (deterministic for a seed).
// The uniform draws come from a counter-based hash, so the sampled SET has
// the reference's distribution but not numpy's MT19937 stream.
//
// Large 2-hop rows (A*A^T, A^T*A with more than `reject_w` expansion paths,
// e.g. every node of a power-law edge with 1e6 members) are not expanded.
// They are sampled from the union U = U_m S_m (S_m = row m of the second
// factor, m over row r of the first) by Karp-Luby rejection:
//   1. draw a path uniformly: m with probability |S_m| / W, c uniform in S_m;
//   2. accept iff m is the FIRST set holding c, i.e.
//      m == min(row r of l1 ∩ row c of l1) (for both patterns the second
//      factor is the transpose of the first);
//   3. distinct accepted columns are kept in draw order until q are held.
// Step 2 makes every c in U equally likely per draw; step 3 (sequential
// draws, repeats rejected) yields a uniform q-subset, which is the
// distribution of np.random.choice(U, q, replace=False). Draws are processed
// in rounds of 256 in thread order, so the result is deterministic for a
// seed. A row whose union turns out smaller than q (no progress for 32
// rounds) falls back to expansion.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "hgx_internal.h"

namespace {

constexpr int kSB = 256;      // sampler workgroup
constexpr int kSelCap = 2048; // LDS sort capacity for the chosen columns

enum Pattern { PAT_A = 0, PAT_AT, PAT_NN, PAT_EE, PAT_NNE, PAT_EEN };

struct Csr {
  const int *rp, *col;
};

struct SampleArgs {
  int pattern;
  int nrows, ncols;
  Csr l1, l2, l3;            // CSR used at each expansion level
  int levels;
  const int *quota;          // per row (nullptr -> quota_all)
  int quota_all;
  const int64_t *cap_off;    // exclusive scan of quotas
  int *out_cols;             // capacity buffer
  int *out_cnt;              // chosen per row
  unsigned *bitmap_g;        // per-WG bitmap slices (global mode)
  int *list_g;               // per-WG distinct lists
  int64_t list_cap;          // per-WG list capacity
  int *row_ctr;              // dynamic row queue
  uint64_t seed;
  int lds_bitmap;            // 1 -> bitmap in dynamic LDS
  int64_t reject_w;          // 2-hop rows with more paths: rejection sampling
  int *stats;                // [0] rows sampled by rejection, [1] fallbacks
};

__device__ int block_scan_excl(int v, int *total, int *s_ws) {
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
  for (int w = 0; w < kSB / 64; w++) {
    const int x = s_ws[w];
    if (w < wave) base += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// index i of the last entry with off[i] <= w (off ascending, n entries)
__device__ __forceinline__ int upper_find(const int *off, int n, int w) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= w) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ unsigned long long composite(uint64_t seed, int pat,
                                                        int row, int col) {
  const uint32_t h = (uint32_t)(hgx::rand64(seed, 0x100 + pat,
                                            ((uint64_t)(uint32_t)row << 32) |
                                                (uint32_t)col) >> 32);
  return ((unsigned long long)h << 32) | (unsigned)col;
}

struct SharedState {
  int cnt;
  int nsel;
  int ws[kSB / 64];
  int a_id[kSB], a_off[kSB];
  int b_id[kSB], b_off[kSB];
  int hist[256];
  unsigned long long prefix;
  int need;
  int sel[kSelCap];
};

// Insert column c into the distinct set.
__device__ __forceinline__ void insert_col(int c, unsigned *bm, int *list,
                                           int64_t list_cap, int *cnt) {
  const unsigned bit = 1u << (c & 31);
  const unsigned old = atomicOr(&bm[c >> 5], bit);
  if (!(old & bit)) {
    const int pos = atomicAdd(cnt, 1);
    if (pos < list_cap) list[pos] = c;
  }
}

// Walk every endpoint of row r's expansion and insert it.
__device__ void expand_row(const SampleArgs &A, int r, unsigned *bm, int *list,
                           SharedState &S) {
  const int tid = threadIdx.x;
  const int b1 = A.l1.rp[r], e1 = A.l1.rp[r + 1];
  if (A.levels == 1) {
    for (int t = b1 + tid; t < e1; t += kSB)
      insert_col(A.l1.col[t], bm, list, A.list_cap, &S.cnt);
    return;
  }
  for (int c1 = b1; c1 < e1; c1 += kSB) {
    // level-1 chunk: ids and level-2 row sizes
    const int i1 = c1 + tid;
    int id1 = -1, sz = 0;
    if (i1 < e1) {
      id1 = A.l1.col[i1];
      sz = A.l2.rp[id1 + 1] - A.l2.rp[id1];
    }
    int W2;
    const int o1 = block_scan_excl(sz, &W2, S.ws);
    S.a_id[tid] = id1;
    S.a_off[tid] = o1;
    __syncthreads();
    const int n1 = min(kSB, e1 - c1);
    if (A.levels == 2) {
      for (int w = tid; w < W2; w += kSB) {
        const int j = upper_find(S.a_off, n1, w);
        const int id = S.a_id[j];
        insert_col(A.l2.col[A.l2.rp[id] + (w - S.a_off[j])], bm, list,
                   A.list_cap, &S.cnt);
      }
    } else {
      for (int w2 = 0; w2 < W2; w2 += kSB) {
        const int w = w2 + tid;
        int id2 = -1, sz2 = 0;
        if (w < W2) {
          const int j = upper_find(S.a_off, n1, w);
          const int id = S.a_id[j];
          id2 = A.l2.col[A.l2.rp[id] + (w - S.a_off[j])];
          sz2 = A.l3.rp[id2 + 1] - A.l3.rp[id2];
        }
        int W3;
        const int o2 = block_scan_excl(sz2, &W3, S.ws);
        S.b_id[tid] = id2;
        S.b_off[tid] = o2;
        __syncthreads();
        const int n2 = min(kSB, W2 - w2);
        for (int x = tid; x < W3; x += kSB) {
          const int j = upper_find(S.b_off, n2, x);
          const int id = S.b_id[j];
          insert_col(A.l3.col[A.l3.rp[id] + (x - S.b_off[j])], bm, list,
                     A.list_cap, &S.cnt);
        }
        __syncthreads();
      }
    }
    __syncthreads();
  }
}

__device__ void bitonic_sort_int(int *a, int n) {
  int P = 1;
  while (P < n) P <<= 1;
  for (int t = n + threadIdx.x; t < P; t += kSB) a[t] = 0x7fffffff;
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += kSB) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const bool up = (lo & size) == 0;
        const int x = a[lo], y = a[hi];
        if ((x > y) == up) {
          a[lo] = y;
          a[hi] = x;
        }
      }
      __syncthreads();
    }
  }
}

// smallest element of sorted a[0..na) that is also in sorted b[0..nb)
// (INT_MAX if none): walk the shorter list, binary-search the longer one
__device__ int first_common(const int *a, int na, const int *b, int nb) {
  if (na > nb) {
    const int *t = a;
    a = b;
    b = t;
    const int tn = na;
    na = nb;
    nb = tn;
  }
  int lo = 0;
  for (int i = 0; i < na; i++) {
    const int x = a[i];
    int hi = nb;
    while (lo < hi) {  // first b[j] >= x, from the previous position on
      const int mid = (lo + hi) >> 1;
      if (b[mid] < x) lo = mid + 1;
      else hi = mid;
    }
    if (lo == nb) return INT_MAX;
    if (b[lo] == x) return x;
  }
  return INT_MAX;
}

struct RejState {
  unsigned long long key[kSB];
  int flag[kSB];
  int cand[kSB];
  int wsum_ws[kSB / 64];
  long long wtot;
  int wmax;
};

// Karp-Luby union sampling of row r (see the header). Fills S.sel[0..q) and
// sets their bitmap bits; returns false if the union looks smaller than q.
__device__ bool reject_row(const SampleArgs &A, int r, int q, unsigned *bm,
                           SharedState &S, RejState &J, long long W, int wmax) {
  const int tid = threadIdx.x;
  const int b1 = A.l1.rp[r], e1 = A.l1.rp[r + 1], n1 = e1 - b1;
  const bool small = n1 <= kSB;
  if (small) {  // exact path draws: prefix of |S_m| over row r in LDS
    const int i1 = b1 + tid;
    int id1 = -1, sz = 0;
    if (tid < n1) {
      id1 = A.l1.col[i1];
      sz = A.l2.rp[id1 + 1] - A.l2.rp[id1];
    }
    int tot;
    const int o1 = block_scan_excl(sz, &tot, S.ws);
    S.a_id[tid] = id1;
    S.a_off[tid] = o1;
  }
  if (tid == 0) S.nsel = 0;
  __syncthreads();
  int stall = 0;
  for (int round = 0; round < 4096; round++) {
    const uint64_t base = ((uint64_t)(uint32_t)r << 32) ^ ((uint64_t)round << 12);
    const uint64_t h = hgx::rand64(A.seed, 0x300 + A.pattern, base + tid);
    const uint64_t h2 = hgx::mix64(h ^ 0x51ed27ull);
    int m = -1, c = -1;
    if (small) {
      const int w = (int)hgx::bounded(h, (uint32_t)W);
      const int j = upper_find(S.a_off, n1, w);
      m = S.a_id[j];
      c = A.l2.col[A.l2.rp[m] + (w - S.a_off[j])];
    } else {  // m uniform, accepted with |S_m| / max |S_m|
      m = A.l1.col[b1 + (int)hgx::bounded(h, (uint32_t)n1)];
      const int sz = A.l2.rp[m + 1] - A.l2.rp[m];
      if ((uint32_t)(h2 >> 32) % (uint32_t)wmax < (uint32_t)sz)
        c = A.l2.col[A.l2.rp[m] + (int)hgx::bounded(h2, (uint32_t)sz)];
    }
    int cand = INT_MAX;
    if (c >= 0 && !(bm[c >> 5] & (1u << (c & 31)))) {
      const int f = first_common(A.l1.col + b1, n1, A.l1.col + A.l1.rp[c],
                                 A.l1.rp[c + 1] - A.l1.rp[c]);
      if (f == m) cand = c;
    }
    // repeats inside the round: keep the lowest thread (sort (col, tid))
    J.key[tid] = ((unsigned long long)(unsigned)cand << 32) | (unsigned)tid;
    __syncthreads();
    for (int size = 2; size <= kSB; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const int t = tid;
        if (t < kSB / 2) {
          const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
          const bool up = (lo & size) == 0;
          const unsigned long long x = J.key[lo], y = J.key[hi];
          if ((x > y) == up) {
            J.key[lo] = y;
            J.key[hi] = x;
          }
        }
        __syncthreads();
      }
    }
    {
      const unsigned long long k = J.key[tid];
      const int col = (int)(k >> 32);
      const bool fresh = col != INT_MAX &&
                         (tid == 0 || (int)(J.key[tid - 1] >> 32) != col);
      J.flag[(int)(k & 0xffffffffu)] = fresh ? 1 : 0;
    }
    __syncthreads();
    int total;
    const int rank = block_scan_excl(J.flag[tid], &total, S.ws);
    const int need = q - S.nsel;
    if (J.flag[tid] && rank < need) {
      S.sel[S.nsel + rank] = cand;
      atomicOr(&bm[cand >> 5], 1u << (cand & 31));
    }
    __syncthreads();
    const int got = min(total, need);
    if (tid == 0) S.nsel += got;
    __syncthreads();
    if (S.nsel >= q) return true;
    stall = got ? 0 : stall + 1;
    if (stall >= 32) break;
  }
  // give back the bits and let expansion handle the row
  for (int i = tid; i < S.nsel; i += kSB) {
    const int c = S.sel[i];
    bm[c >> 5] = 0u;
  }
  __syncthreads();
  return false;
}

__global__ __launch_bounds__(kSB) void sample_rows(SampleArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned s_dyn[];
  __shared__ SharedState S;
  __shared__ RejState J;
  __shared__ long long s_rw[kSB / 64];
  __shared__ int s_rm[kSB / 64];
  __shared__ int s_row;
  const int tid = threadIdx.x;
  const int nwords = (A.ncols + 31) >> 5;
  unsigned *bm = A.lds_bitmap ? s_dyn : A.bitmap_g + (size_t)blockIdx.x * nwords;
  int *list = A.list_g + (size_t)blockIdx.x * A.list_cap;
  for (int w = tid; w < nwords; w += kSB) bm[w] = 0u;
  __syncthreads();
  while (true) {
    if (tid == 0) {
      s_row = atomicAdd(A.row_ctr, 1);
      S.cnt = 0;
      S.nsel = 0;
    }
    __syncthreads();
    const int r = s_row;
    if (r >= A.nrows) break;
    const int q = A.quota ? A.quota[r] : A.quota_all;
    int *out = A.out_cols + A.cap_off[r];
    if (q <= 0) {
      if (tid == 0) A.out_cnt[r] = 0;
      __syncthreads();
      continue;
    }
    if (A.levels == 2 && q <= kSelCap && A.reject_w > 0) {
      // path count W and max |S_m| of the row (block reductions)
      const int b1 = A.l1.rp[r], e1 = A.l1.rp[r + 1];
      long long w = 0;
      int wm = 0;
      for (int t = b1 + tid; t < e1; t += kSB) {
        const int id = A.l1.col[t];
        const int sz = A.l2.rp[id + 1] - A.l2.rp[id];
        w += sz;
        wm = max(wm, sz);
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        w += __shfl_xor(w, off);
        wm = max(wm, __shfl_xor(wm, off));
      }
      if ((tid & 63) == 0) {
        s_rw[tid >> 6] = w;
        s_rm[tid >> 6] = wm;
      }
      __syncthreads();
      long long W = 0;
      int wmax = 0;
#pragma unroll
      for (int i = 0; i < kSB / 64; i++) {
        W += s_rw[i];
        wmax = max(wmax, s_rm[i]);
      }
      __syncthreads();
      if (W > A.reject_w && W < (1ll << 31) && reject_row(A, r, q, bm, S, J, W, wmax)) {
        if (tid == 0) atomicAdd(&A.stats[0], 1);
        bitonic_sort_int(S.sel, q);
        for (int i = tid; i < q; i += kSB) out[i] = S.sel[i];
        if (tid == 0) A.out_cnt[r] = q;
        for (int i = tid; i < q; i += kSB) {
          const int c = S.sel[i];
          bm[c >> 5] = 0u;
        }
        __syncthreads();
        continue;
      }
      if (W > A.reject_w && tid == 0) atomicAdd(&A.stats[1], 1);
      if (tid == 0) S.nsel = 0;
      __syncthreads();
    }
    expand_row(A, r, bm, list, S);
    __syncthreads();
    if (tid == 0 && S.cnt > A.list_cap) atomicOr(&A.stats[2], 1);
    const int cnt = (int)min((int64_t)S.cnt, A.list_cap);
    const int m = min(q, cnt);
    if (m < cnt) {
      // m smallest composite keys: 8-pass radix select -> exact threshold
      if (tid == 0) {
        S.prefix = 0ull;
        S.need = m;
      }
      for (int p = 7; p >= 0; p--) {
        S.hist[tid] = 0;
        __syncthreads();
        const unsigned long long hm = p == 7 ? 0ull : ~((1ull << (8 * (p + 1))) - 1);
        const unsigned long long pre = S.prefix;
        for (int i = tid; i < cnt; i += kSB) {
          const unsigned long long c = composite(A.seed, A.pattern, r, list[i]);
          if ((c & hm) == (pre & hm)) atomicAdd(&S.hist[(c >> (8 * p)) & 255], 1);
        }
        __syncthreads();
        if (tid < 64) {
          // wave 0 finds the digit holding the need-th key
          int h[4], s4 = 0;
#pragma unroll
          for (int q4 = 0; q4 < 4; q4++) {
            h[q4] = S.hist[tid * 4 + q4];
            s4 += h[q4];
          }
          int inc = s4;
#pragma unroll
          for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(inc, off);
            if (tid >= off) inc += o;
          }
          const int need = S.need;
          int before = inc - s4;
          if (before < need && inc >= need) {
            int digit = tid * 4;
#pragma unroll
            for (int q4 = 0; q4 < 4; q4++) {
              if (before + h[q4] >= need) break;
              before += h[q4];
              digit++;
            }
            S.need = need - before;
            S.prefix = pre | ((unsigned long long)digit << (8 * p));
          }
        }
        __syncthreads();
      }
      const unsigned long long T = S.prefix;
      for (int i = tid; i < cnt; i += kSB) {
        const int c = list[i];
        if (composite(A.seed, A.pattern, r, c) <= T) {
          const int pos = atomicAdd(&S.nsel, 1);
          if (m <= kSelCap) S.sel[pos] = c;
          else out[pos] = c;
        }
      }
    } else {
      for (int i = tid; i < cnt; i += kSB) {
        if (m <= kSelCap) S.sel[i] = list[i];
        else out[i] = list[i];
      }
    }
    __syncthreads();
    if (m <= kSelCap) {
      bitonic_sort_int(S.sel, m);
      for (int i = tid; i < m; i += kSB) out[i] = S.sel[i];
    }
    if (tid == 0) A.out_cnt[r] = m;
    // clear exactly the bits that were set
    for (int i = tid; i < cnt; i += kSB) {
      const int c = list[i];
      bm[c >> 5] = 0u;
    }
    __syncthreads();
  }
}

// ---- record materialisation ----------------------------------------------
enum RecKind { REC_NN = 0, REC_EE, REC_NE_NODE, REC_NE_EDGE };

// one thread per (row, j < cnt[row]): write record rec_base + off[row] + j
__global__ void emit_records(int kind, int nrows, const int *cnt,
                             const int64_t *cap_off, const int64_t *rec_off,
                             const int *cols, int64_t rec_base, int R,
                             int *idx, float *tgt, float prob) {
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int m = cnt[r];
    const int *src = cols + cap_off[r];
    for (int j = threadIdx.x; j < m; j += blockDim.x) {
      const int64_t rec = rec_base + rec_off[r] + j;
      int *ri = idx + rec * R;
      for (int s = 0; s < R; s++) ri[s] = 0;
      const int c = src[j];
      if (kind == REC_NN) { ri[0] = r + 1; ri[2] = c + 1; }
      else if (kind == REC_EE) { ri[1] = r + 1; ri[3] = c + 1; }
      else if (kind == REC_NE_NODE) { ri[0] = r + 1; ri[3] = c + 1; }
      else { ri[0] = c + 1; ri[3] = r + 1; }
      float *t = tgt + rec * 3;
      t[0] = t[1] = t[2] = 0.f;
      t[kind == REC_NN ? 0 : kind == REC_EE ? 1 : 2] = prob;
    }
  }
}

// negatives: q[row] uniform columns WITH replacement (hg2v_sample.py:73-75)
__global__ void emit_negatives(int kind, int nrows, int ncols, const int *q,
                               const int64_t *off, int64_t rec_base, int R,
                               int *idx, float *tgt, uint64_t seed,
                               uint64_t stream) {
  for (int r = blockIdx.x; r < nrows; r += gridDim.x) {
    const int m = q[r];
    for (int j = threadIdx.x; j < m; j += blockDim.x) {
      const int64_t rec = rec_base + off[r] + j;
      const int c = (int)hgx::bounded(
          hgx::rand64(seed, stream, ((uint64_t)r << 32) | (uint32_t)j),
          (uint32_t)ncols);
      int *ri = idx + rec * R;
      for (int s = 0; s < R; s++) ri[s] = 0;
      if (kind == REC_NN) { ri[0] = r + 1; ri[2] = c + 1; }
      else if (kind == REC_EE) { ri[1] = r + 1; ri[3] = c + 1; }
      else if (kind == REC_NE_NODE) { ri[0] = r + 1; ri[3] = c + 1; }
      else { ri[0] = c + 1; ri[3] = r + 1; }
      float *t = tgt + rec * 3;
      t[0] = t[1] = t[2] = 0.f;
    }
  }
}

// _sample_neighbors for node-edge records [b, e): nn_k from N(re-1),
// ne_k from E(ln-1), K draws with replacement each.
__global__ void draw_neighbors(int64_t b, int64_t e, int K, int R, int *idx,
                               const int *rp_n, const int *col_n,
                               const int *rp_e, const int *col_e,
                               uint64_t seed, uint64_t stream) {
  for (int64_t rec = b + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; rec < e;
       rec += (int64_t)gridDim.x * blockDim.x) {
    int *ri = idx + rec * R;
    const int v = ri[0] - 1, ed = ri[3] - 1;
    const int nb = rp_e[ed], nl = rp_e[ed + 1] - nb;
    const int eb = rp_n[v], el = rp_n[v + 1] - eb;
    for (int k = 0; k < K; k++) {
      const uint64_t h = hgx::rand64(seed, stream, (uint64_t)rec * 64 + k);
      const uint64_t h2 = hgx::rand64(seed, stream + 1, (uint64_t)rec * 64 + k);
      // an isolated endpoint (possible only for negatives) keeps padding 0;
      // the reference raises there (np.random.choice on an empty row)
      ri[4 + k] = nl ? col_e[nb + hgx::bounded(h, (uint32_t)nl)] + 1 : 0;
      ri[4 + K + k] = el ? col_n[eb + hgx::bounded(h2, (uint32_t)el)] + 1 : 0;
    }
  }
}

int grid_for(int64_t work, int per_block, int cap = 4096) {
  int64_t g = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

struct ToI64 {
  __host__ __device__ int64_t operator()(int x) const { return (int64_t)x; }
};

int excl_scan_i32_to_i64(hgx_ctx *ctx, const int *in, int64_t *out, int n,
                         int64_t *total) {
  // out has n+1 entries; out[n] = total; accumulate in int64
  hipcub::TransformInputIterator<int64_t, ToI64, const int *> it(in, ToI64());
  size_t tmp = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, out, n + 1, ctx->stream);
  HGX_TRY(hgx_ensure(ctx, ctx->s7, tmp + 256));
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(ctx->s7.p, tmp, it, out, n + 1,
                                                ctx->stream));
  HGX_HIP(ctx, hipMemcpyAsync(total, out + n, sizeof(int64_t),
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

// Result of sampling one pattern: per-row chosen columns (capacity layout)
struct PatOut {
  int nrows = 0;
  DevBuf q;        // int quota[nrows + 1] (last = 0 for the scan)
  DevBuf cap_off;  // int64[nrows + 1]
  DevBuf cols;     // int[sum q]
  DevBuf cnt;      // int[nrows + 1]
  DevBuf rec_off;  // int64[nrows + 1]
  int64_t total = 0;
  ~PatOut() {
    hgx_release(q);
    hgx_release(cap_off);
    hgx_release(cols);
    hgx_release(cnt);
    hgx_release(rec_off);
  }
};

__global__ void fill_quota(int *q, int n, int v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i <= n;
       i += gridDim.x * blockDim.x)
    q[i] = i < n ? v : 0;
}

int run_pattern(hgx_ctx *ctx, int pattern, const int32_t *host_quota,
                int quota_all, uint64_t seed, PatOut &po) {
  const int N = ctx->N, E = ctx->E;
  const Csr A{ctx->rp_n.as<int>(), ctx->col_n.as<int>()};
  const Csr AT{ctx->rp_e.as<int>(), ctx->col_e.as<int>()};
  SampleArgs a{};
  a.pattern = pattern;
  switch (pattern) {
    case PAT_A: a.nrows = N; a.ncols = E; a.l1 = A; a.levels = 1; break;
    case PAT_AT: a.nrows = E; a.ncols = N; a.l1 = AT; a.levels = 1; break;
    case PAT_NN: a.nrows = N; a.ncols = N; a.l1 = A; a.l2 = AT; a.levels = 2; break;
    case PAT_EE: a.nrows = E; a.ncols = E; a.l1 = AT; a.l2 = A; a.levels = 2; break;
    case PAT_NNE: a.nrows = N; a.ncols = E; a.l1 = A; a.l2 = AT; a.l3 = A; a.levels = 3; break;
    default: a.nrows = E; a.ncols = N; a.l1 = AT; a.l2 = A; a.l3 = AT; a.levels = 3; break;
  }
  const int R = a.nrows;
  po.nrows = R;
  HGX_TRY(hgx_ensure(ctx, po.q, sizeof(int) * (R + 1)));
  if (host_quota) {
    HGX_HIP(ctx, hipMemcpyAsync(po.q.p, host_quota, sizeof(int) * R,
                                hipMemcpyHostToDevice, ctx->stream));
    HGX_HIP(ctx, hipMemsetAsync(po.q.as<int>() + R, 0, sizeof(int), ctx->stream));
  } else {
    hipLaunchKernelGGL(fill_quota, dim3(grid_for(R + 1, 256)), dim3(256), 0,
                       ctx->stream, po.q.as<int>(), R, quota_all);
  }
  HGX_TRY(hgx_ensure(ctx, po.cap_off, sizeof(int64_t) * (R + 1)));
  int64_t cap_total = 0;
  HGX_TRY(excl_scan_i32_to_i64(ctx, po.q.as<int>(), po.cap_off.as<int64_t>(), R,
                               &cap_total));
  HGX_TRY(hgx_ensure(ctx, po.cols, sizeof(int) * (cap_total + 1)));
  HGX_TRY(hgx_ensure(ctx, po.cnt, sizeof(int) * (R + 1)));
  HGX_HIP(ctx, hipMemsetAsync(po.cnt.p, 0, sizeof(int) * (R + 1), ctx->stream));
  // workgroups and their scratch
  const int nwords = (a.ncols + 31) / 32;
  const bool lds = (size_t)nwords * 4 <= 48 * 1024;
  int nwg = 1024;
  {
    // 2-hop rows with more expansion paths than this are union-sampled
    // (HGX_SAMPLE_REJECT_W overrides; 0 disables)
    const char *e = getenv("HGX_SAMPLE_REJECT_W");
    a.reject_w = e ? atoll(e) : (int64_t)1 << 15;
  }
  // the distinct list only serves expanded rows: with union sampling on,
  // 2-hop rows expand at most reject_w paths (a fallback row that does not
  // fit is reported, never truncated)
  const int64_t list_cap =
      (a.levels == 2 && a.reject_w > 0)
          ? std::min<int64_t>(a.ncols, std::max<int64_t>(2 * a.reject_w, 65536))
          : a.ncols;
  while (nwg > 64 && (double)nwg * (list_cap * 4 + (lds ? 0 : nwords * 4)) > 4e9)
    nwg /= 2;
  HGX_TRY(hgx_ensure(ctx, ctx->s3, sizeof(int) * (size_t)nwg * list_cap + 16));
  if (!lds) HGX_TRY(hgx_ensure(ctx, ctx->s4, sizeof(unsigned) * (size_t)nwg * nwords));
  HGX_TRY(hgx_ensure(ctx, ctx->s0, 16));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s0.p, 0, 16, ctx->stream));
  a.quota = po.q.as<int>();
  a.quota_all = quota_all;
  a.cap_off = po.cap_off.as<int64_t>();
  a.out_cols = po.cols.as<int>();
  a.out_cnt = po.cnt.as<int>();
  a.bitmap_g = lds ? nullptr : ctx->s4.as<unsigned>();
  a.list_g = ctx->s3.as<int>();
  a.list_cap = list_cap;
  a.row_ctr = ctx->s0.as<int>();
  a.seed = seed;
  a.lds_bitmap = lds;
  a.stats = ctx->s0.as<int>() + 1;  // [0] union-sampled rows, [1] fallbacks, [2] overflow
  hipLaunchKernelGGL(sample_rows, dim3(nwg), dim3(kSB),
                     lds ? (size_t)nwords * 4 : 0, ctx->stream, a);
  HGX_LAUNCH_CHECK(ctx);
  {
    int st[3] = {0, 0, 0};
    HGX_HIP(ctx, hipMemcpyAsync(st, a.stats, sizeof(st), hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ctx->sample_union_rows += st[0];
    ctx->sample_fallback_rows += st[1];
    HGX_CHECK(ctx, st[2] == 0, HGX_EUNSUP,
              "a sampled row has more than %lld distinct columns "
              "(raise HGX_SAMPLE_REJECT_W or disable union sampling)",
              (long long)list_cap);
  }
  HGX_TRY(hgx_ensure(ctx, po.rec_off, sizeof(int64_t) * (R + 1)));
  HGX_TRY(excl_scan_i32_to_i64(ctx, po.cnt.as<int>(), po.rec_off.as<int64_t>(),
                               R, &po.total));
  return HGX_OK;
}

int alloc_records(hgx_ctx *ctx, int64_t n, int K) {
  const int R = 4 + 2 * K;
  HGX_CHECK(ctx, n < (int64_t)INT32_MAX, HGX_EUNSUP,
            "%lld records exceed the 2^31 record limit", (long long)n);
  HGX_TRY(hgx_ensure(ctx, ctx->rec_idx, sizeof(int32_t) * (n * R + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->rec_tgt, sizeof(float) * (n * 3 + 1)));
  ctx->n_rec = n;
  ctx->K = K;
  return HGX_OK;
}

int emit(hgx_ctx *ctx, int kind, const PatOut &po, int64_t base, float prob) {
  if (po.total == 0) return HGX_OK;
  hipLaunchKernelGGL(emit_records, dim3(grid_for(po.nrows, 1, 65536)), dim3(64),
                     0, ctx->stream, kind, po.nrows, po.cnt.as<int>(),
                     po.cap_off.as<int64_t>(), po.rec_off.as<int64_t>(),
                     po.cols.as<int>(), base, 4 + 2 * ctx->K,
                     ctx->rec_idx.as<int>(), ctx->rec_tgt.as<float>(), prob);
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

int neighbors(hgx_ctx *ctx, int64_t b, int64_t e, uint64_t seed,
              uint64_t stream) {
  if (e <= b) return HGX_OK;
  hipLaunchKernelGGL(draw_neighbors, dim3(grid_for(e - b, 256)), dim3(256), 0,
                     ctx->stream, b, e, ctx->K, 4 + 2 * ctx->K,
                     ctx->rec_idx.as<int>(), ctx->rp_n.as<int>(),
                     ctx->col_n.as<int>(), ctx->rp_e.as<int>(),
                     ctx->col_e.as<int>(), seed, stream);
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

struct NegOut {
  DevBuf q, off;
  int64_t total = 0;
  int nrows = 0;
  ~NegOut() {
    hgx_release(q);
    hgx_release(off);
  }
};

int neg_prepare(hgx_ctx *ctx, const int32_t *host_q, int nrows, NegOut &no) {
  no.nrows = nrows;
  HGX_TRY(hgx_ensure(ctx, no.q, sizeof(int) * (nrows + 1)));
  HGX_HIP(ctx, hipMemcpyAsync(no.q.p, host_q, sizeof(int) * nrows,
                              hipMemcpyHostToDevice, ctx->stream));
  HGX_HIP(ctx, hipMemsetAsync(no.q.as<int>() + nrows, 0, sizeof(int), ctx->stream));
  HGX_TRY(hgx_ensure(ctx, no.off, sizeof(int64_t) * (nrows + 1)));
  return excl_scan_i32_to_i64(ctx, no.q.as<int>(), no.off.as<int64_t>(), nrows,
                              &no.total);
}

int neg_emit(hgx_ctx *ctx, int kind, const NegOut &no, int ncols, int64_t base,
             uint64_t seed, uint64_t stream) {
  if (no.total == 0) return HGX_OK;
  hipLaunchKernelGGL(emit_negatives, dim3(grid_for(no.nrows, 1, 65536)),
                     dim3(64), 0, ctx->stream, kind, no.nrows, ncols,
                     no.q.as<int>(), no.off.as<int64_t>(), base,
                     4 + 2 * ctx->K, ctx->rec_idx.as<int>(),
                     ctx->rec_tgt.as<float>(), seed, stream);
  HGX_LAUNCH_CHECK(ctx);
  return HGX_OK;
}

int check_quota(hgx_ctx *ctx, const int32_t *q, int n, const char *what) {
  HGX_CHECK(ctx, q, HGX_EINVAL, "%s quota is null", what);
  for (int i = 0; i < n; i++)
    HGX_CHECK(ctx, q[i] >= 0, HGX_EINVAL, "%s quota[%d] < 0", what, i);
  return HGX_OK;
}

}  // namespace

// HOBE probability kernels live in hgx_hobe.hip
int hgx_hobe_fill_probs(hgx_ctx *ctx, int kind, int64_t b, int64_t e);

extern "C" int hgx_sample_fobe(hgx_ctx *ctx, uint64_t seed, int K,
                               const int32_t *node_quota,
                               const int32_t *edge_quota,
                               const int32_t *neg_node_quota,
                               const int32_t *neg_edge_quota,
                               int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, K >= 1 && K <= 16, HGX_EUNSUP, "num_neighbors %d outside [1,16]", K);
  HGX_CHECK(ctx, (neg_node_quota == nullptr) == (neg_edge_quota == nullptr),
            HGX_EINVAL, "give both negative quotas or neither");
  HGX_TRY(check_quota(ctx, node_quota, ctx->N, "node"));
  HGX_TRY(check_quota(ctx, edge_quota, ctx->E, "edge"));
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  ctx->sample_union_rows = ctx->sample_fallback_rows = 0;
  // BooleanSamples order (hg2v_sample.py:156-194): nn, ee, ne(node rows),
  // ne(edge rows, swapped); then negatives (:198-240).
  PatOut nn, ee, ne_n, ne_e;
  HGX_TRY(run_pattern(ctx, PAT_NN, node_quota, 0, seed, nn));
  HGX_TRY(run_pattern(ctx, PAT_EE, edge_quota, 0, seed, ee));
  HGX_TRY(run_pattern(ctx, PAT_A, node_quota, 0, seed, ne_n));
  HGX_TRY(run_pattern(ctx, PAT_AT, edge_quota, 0, seed, ne_e));
  NegOut gnn, gee, gne_n, gne_e;
  if (neg_node_quota) {
    HGX_TRY(check_quota(ctx, neg_node_quota, ctx->N, "negative node"));
    HGX_TRY(check_quota(ctx, neg_edge_quota, ctx->E, "negative edge"));
    HGX_TRY(neg_prepare(ctx, neg_node_quota, ctx->N, gnn));
    HGX_TRY(neg_prepare(ctx, neg_edge_quota, ctx->E, gee));
    HGX_TRY(neg_prepare(ctx, neg_node_quota, ctx->N, gne_n));
    HGX_TRY(neg_prepare(ctx, neg_edge_quota, ctx->E, gne_e));
  }
  const int64_t o_ee = nn.total, o_ne = o_ee + ee.total;
  const int64_t o_en = o_ne + ne_n.total, o_neg = o_en + ne_e.total;
  const int64_t o_gee = o_neg + gnn.total, o_gee2 = o_gee + gee.total;
  const int64_t o_gne = o_gee2 + gee.total, o_gen = o_gne + gne_n.total;
  const int64_t total = o_gen + gne_e.total;
  HGX_TRY(alloc_records(ctx, total, K));
  HGX_TRY(emit(ctx, REC_NN, nn, 0, 1.f));
  HGX_TRY(emit(ctx, REC_EE, ee, o_ee, 1.f));
  HGX_TRY(emit(ctx, REC_NE_NODE, ne_n, o_ne, 1.f));
  HGX_TRY(emit(ctx, REC_NE_EDGE, ne_e, o_en, 1.f));
  HGX_TRY(neighbors(ctx, o_ne, o_neg, seed, 0x200));
  if (neg_node_quota) {
    HGX_TRY(neg_emit(ctx, REC_NN, gnn, ctx->N, o_neg, seed, 0x300));
    HGX_TRY(neg_emit(ctx, REC_EE, gee, ctx->E, o_gee, seed, 0x301));
    // the reference's "Node-Edge Negatives" block repeats edge-edge
    // sampling (hg2v_sample.py:215-221); kept for parity of counts
    HGX_TRY(neg_emit(ctx, REC_EE, gee, ctx->E, o_gee2, seed, 0x302));
    HGX_TRY(neg_emit(ctx, REC_NE_NODE, gne_n, ctx->E, o_gne, seed, 0x303));
    HGX_TRY(neg_emit(ctx, REC_NE_EDGE, gne_e, ctx->N, o_gen, seed, 0x304));
    HGX_TRY(neighbors(ctx, o_gne, total, seed, 0x400));
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (n_records) *n_records = total;
  return HGX_OK;
}

extern "C" int hgx_sample_hobe(hgx_ctx *ctx, uint64_t seed, int K, int S,
                               int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE,
            "HOBE needs the algebraic-distance coords on device");
  HGX_CHECK(ctx, K >= 1 && K <= 16, HGX_EUNSUP, "num_neighbors %d outside [1,16]", K);
  HGX_CHECK(ctx, S >= 0, HGX_EINVAL, "num_samples must be >= 0 (hg2v_sample.py:647)");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  ctx->sample_union_rows = ctx->sample_fallback_rows = 0;
  // AlgebraicDistanceSamples order (hg2v_sample.py:658-715)
  PatOut nn, ee, ne_n, ne_e;
  HGX_TRY(run_pattern(ctx, PAT_NN, nullptr, S, seed, nn));
  HGX_TRY(run_pattern(ctx, PAT_EE, nullptr, S, seed, ee));
  HGX_TRY(run_pattern(ctx, PAT_NNE, nullptr, S, seed, ne_n));
  HGX_TRY(run_pattern(ctx, PAT_EEN, nullptr, S, seed, ne_e));
  const int64_t o_ee = nn.total, o_ne = o_ee + ee.total;
  const int64_t o_en = o_ne + ne_n.total, total = o_en + ne_e.total;
  HGX_TRY(alloc_records(ctx, total, K));
  HGX_TRY(emit(ctx, REC_NN, nn, 0, 0.f));
  HGX_TRY(emit(ctx, REC_EE, ee, o_ee, 0.f));
  HGX_TRY(emit(ctx, REC_NE_NODE, ne_n, o_ne, 0.f));
  HGX_TRY(emit(ctx, REC_NE_EDGE, ne_e, o_en, 0.f));
  HGX_TRY(neighbors(ctx, o_ne, total, seed, 0x500));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 0, 0, o_ee));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 1, o_ee, o_ne));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 2, o_ne, total));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (n_records) *n_records = total;
  return HGX_OK;
}

// WeightedJaccardSamples pair blocks (hg2v_sample.py:436-505): nn (node
// quotas), ee (edge quotas), ne from A A^T A rows (node quotas) then
// A^T A A^T rows swapped (edge quotas); records allocated and emitted,
// ne neighbours drawn; probabilities are left to the caller (hgx_jaccard).
int hgx_sample_pairs4(hgx_ctx *ctx, uint64_t seed, int K, const int32_t *node_q,
                      const int32_t *edge_q, int64_t *o_ee_out,
                      int64_t *o_ne_out, int64_t *total_out) {
  HGX_TRY(check_quota(ctx, node_q, ctx->N, "node"));
  HGX_TRY(check_quota(ctx, edge_q, ctx->E, "edge"));
  ctx->sample_union_rows = ctx->sample_fallback_rows = 0;
  PatOut nn, ee, ne_n, ne_e;
  HGX_TRY(run_pattern(ctx, PAT_NN, node_q, 0, seed, nn));
  HGX_TRY(run_pattern(ctx, PAT_EE, edge_q, 0, seed, ee));
  HGX_TRY(run_pattern(ctx, PAT_NNE, node_q, 0, seed, ne_n));
  HGX_TRY(run_pattern(ctx, PAT_EEN, edge_q, 0, seed, ne_e));
  const int64_t o_ee = nn.total, o_ne = o_ee + ee.total;
  const int64_t o_en = o_ne + ne_n.total, total = o_en + ne_e.total;
  HGX_TRY(alloc_records(ctx, total, K));
  HGX_TRY(emit(ctx, REC_NN, nn, 0, 0.f));
  HGX_TRY(emit(ctx, REC_EE, ee, o_ee, 0.f));
  HGX_TRY(emit(ctx, REC_NE_NODE, ne_n, o_ne, 0.f));
  HGX_TRY(emit(ctx, REC_NE_EDGE, ne_e, o_en, 0.f));
  HGX_TRY(neighbors(ctx, o_ne, total, seed, 0x600));
  *o_ee_out = o_ee;
  *o_ne_out = o_ne;
  *total_out = total;
  return HGX_OK;
}

extern "C" int hgx_sample_last_stats(hgx_ctx *ctx, int64_t *union_rows,
                                     int64_t *fallback_rows) {
  if (!ctx) return HGX_EINVAL;
  if (union_rows) *union_rows = ctx->sample_union_rows;
  if (fallback_rows) *fallback_rows = ctx->sample_fallback_rows;
  return HGX_OK;
}
