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
// materialised. Rows with a quota are listed, then sampled in two passes:
//
// 1. `reject_rows` (2- and 3-hop patterns): rows whose expansion has more
//    than `reject_w` paths are sampled from the union of the pattern row by
//    rejection, never expanded. A workgroup draws 256 candidates per round
//    and keeps the distinct accepted ones in draw order until q are held
//    (an LDS hash set de-duplicates); sequential draws with repeats
//    rejected give a uniform q-subset, the distribution of
//    np.random.choice(row, q, replace=False). Rounds are processed in
//    thread order, so the result is deterministic for a seed. Proposals:
//      * 2-hop (Karp-Luby over paths r -> m -> c): m with probability
//        |S_m| / W, c uniform in S_m; accept iff m is the FIRST set holding
//        c, m == min(row_r(l1) ∩ row_c(l1)) (the second factor is the
//        transpose of the first);
//      * 3-hop, paths (Karp-Luby over r -> m1 -> m2 -> c): a uniform path
//        (m1 weighted by its path count, m2 by |row m2 of l3| through a
//        scan of l2's incidences), accepted iff (m1, m2) is the
//        lexicographically first path to c;
//      * 3-hop, uniform columns: c uniform over all columns, accepted iff
//        (v, e) is in A A^T A, i.e. some e' in E(v) shares a node with e,
//        probed from the smaller edge against each member's sorted edge
//        list. Used when the path count exceeds the column count, where
//        its acceptance rate |row| / ncols beats |row| / W.
//    Rows with at most `reject_w` paths, rows with q > 2048 and rows whose
//    rejection stalls (a union smaller than q) are deferred to pass 2.
// 2. `expand_rows`: one workgroup per row walks the 1/2/3-hop CSR expansion
//    with LDS block scans + binary search (one path endpoint per thread),
//    de-duplicates endpoints with a test-and-set bitmap (LDS when the column
//    space fits, else a per-workgroup slice in HBM) into a distinct list,
//    and picks an exactly uniform m-subset (m = min(q, distinct)) as the m
//    smallest 64-bit keys (hash(seed,row,col) << 32 | col) by an 8-pass LDS
//    radix select. 1-hop rows are their own distinct list.
// Chosen columns are written sorted (the reference's row order). The
// uniform draws come from a counter-based hash, so the sampled SET has the
// reference's distribution but not numpy's MT19937 stream.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <initializer_list>
#include <climits>
#include <vector>

#include "hgx_internal.h"

namespace {

constexpr int kSB = 256;      // sampler workgroup
constexpr int kSelCap = 2048; // LDS capacity for the chosen columns
constexpr int kHashBits = 12; // LDS hash set of the chosen columns
constexpr int kHash = 1 << kHashBits;

enum Pattern { PAT_A = 0, PAT_AT, PAT_NN, PAT_EE, PAT_NNE, PAT_EEN };

struct Csr {
  const int *rp, *col;
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

__device__ long long block_scan_excl64(long long v, long long *total,
                                       long long *s_ws) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  long long inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const long long o = __shfl_up(inc, off);
    if (lane >= off) inc += o;
  }
  if (lane == 63) s_ws[wave] = inc;
  __syncthreads();
  long long base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kSB / 64; w++) {
    const long long x = s_ws[w];
    if (w < wave) base += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

// index i of the last entry with off[i] <= w (off ascending, n entries)
template <class T>
__device__ __forceinline__ int upper_find(const T *off, int n, T w) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= w) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// position of x in sorted col[b, e), or -1
__device__ __forceinline__ int find_sorted(const int *col, int b, int e, int x) {
  int lo = b, hi = e;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (col[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return (lo < e && col[lo] == x) ? lo : -1;
}

__device__ __forceinline__ unsigned long long composite(uint64_t seed, int pat,
                                                        int row, int col) {
  const uint32_t h = (uint32_t)(hgx::rand64(seed, 0x100 + pat,
                                            ((uint64_t)(uint32_t)row << 32) |
                                                (uint32_t)col) >> 32);
  return ((unsigned long long)h << 32) | (unsigned)col;
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

// ---- 3-hop membership (A: node -> edges, AT: edge -> nodes) --------------
// Smallest node in members(x) ∩ members(y) (INT_MAX if none): the smaller
// edge's members in ascending order, each probed for the other edge in its
// own sorted edge list; the first hit is the minimum. Eight members are
// probed at once (their binary searches interleaved step by step): a lone
// thread's probe is a chain of ~6 dependent loads, and the walk over two
// disjoint mid-size power-law edges (thousands of members) was that chain
// thousands of times. C4 2% slice (tools/sample_c4_probe.py): sampling
// 2.39 s one at a time, 1.66 s four, 1.53 s eight, 2.84 s sixteen (register
// pressure). A merge of the two sorted member lists measured slower (one
// dependent load per step over both lists): 3.0 s.
constexpr int kProbeWays = 8;
constexpr int kBloomWays = 8;

// Blocked Bloom filters of the edges' member sets (built once per incidence,
// ensure_bloom): per edge a power of two of 64-byte blocks, >= 16 bits per
// member; a member sets 3 bits of one block chosen by its hash. A member
// whose 3 bits are not all set is not in the edge, so its binary search is
// skipped (~0.5-1 % false positives): a chunk of 8 probes then costs two
// round trips (ids, filter words) instead of ~7. The answer is the exact
// one (a positive still takes the search).
struct Bloom {
  const long long *off;  // first 32-bit word of edge e's filter, E + 1
  const unsigned *bits;
};
__device__ __forceinline__ uint64_t bloom_hash(int u) {
  return hgx::mix64((uint64_t)(uint32_t)u ^ 0x426c6f6f6d4d656dull);
}

__device__ int edges_min_common(const Csr &A, const Csr &AT, int x, int y,
                                const Bloom &B = Bloom{nullptr, nullptr}) {
  if (x == y) return AT.rp[x + 1] > AT.rp[x] ? AT.col[AT.rp[x]] : INT_MAX;
  if (AT.rp[x + 1] - AT.rp[x] > AT.rp[y + 1] - AT.rp[y]) {
    const int t = x;
    x = y;
    y = t;
  }
  const unsigned *fy = nullptr;
  unsigned bmask = 0;
  if (B.bits) {
    const long long o = B.off[y];
    fy = B.bits + o;
    bmask = (unsigned)((B.off[y + 1] - o) / 16 - 1);  // blocks - 1
  }
  const int xe = AT.rp[x + 1];
  if (fy) {
    // kBloomWays members filtered at once (ids, then their filter words),
    // the rare positives searched one by one in ascending order (C4 2%
    // slice: 0.94 s at 4, 0.89 s at 8, 0.975 s at 16 -- register pressure)
    for (int t = AT.rp[x]; t < xe; t += kBloomWays) {
      int u[kBloomWays];
#pragma unroll
      for (int k = 0; k < kBloomWays; k++) u[k] = t + k < xe ? AT.col[t + k] : -1;
      unsigned pass = 0;
      unsigned w0[kBloomWays], w1[kBloomWays], w2[kBloomWays];
      unsigned s0[kBloomWays], s1[kBloomWays], s2[kBloomWays];
#pragma unroll
      for (int k = 0; k < kBloomWays; k++) {
        const uint64_t h = bloom_hash(u[k]);
        const unsigned *blk = fy + 16 * ((unsigned)(h >> 40) & bmask);
        s0[k] = (unsigned)h & 511;
        s1[k] = (unsigned)(h >> 9) & 511;
        s2[k] = (unsigned)(h >> 18) & 511;
        w0[k] = u[k] >= 0 ? blk[s0[k] >> 5] : 0u;
        w1[k] = u[k] >= 0 ? blk[s1[k] >> 5] : 0u;
        w2[k] = u[k] >= 0 ? blk[s2[k] >> 5] : 0u;
      }
#pragma unroll
      for (int k = 0; k < kBloomWays; k++)
        pass |= ((w0[k] >> (s0[k] & 31)) & (w1[k] >> (s1[k] & 31)) & (w2[k] >> (s2[k] & 31)) &
                 1u) << k;
      while (pass) {
        const int k = __builtin_ctz(pass);
        pass &= pass - 1;
        int uk = 0;
#pragma unroll
        for (int j = 0; j < kBloomWays; j++)
          if (j == k) uk = u[j];
        if (find_sorted(A.col, A.rp[uk], A.rp[uk + 1], y) >= 0) return uk;
      }
    }
    return INT_MAX;
  }
  for (int t = AT.rp[x]; t < xe; t += kProbeWays) {
    int u[kProbeWays], lo[kProbeWays], hi[kProbeWays], end[kProbeWays];
#pragma unroll
    for (int k = 0; k < kProbeWays; k++) u[k] = t + k < xe ? AT.col[t + k] : -1;
#pragma unroll
    for (int k = 0; k < kProbeWays; k++) {
      lo[k] = u[k] >= 0 ? A.rp[u[k]] : 0;
      end[k] = u[k] >= 0 ? A.rp[u[k] + 1] : 0;
      hi[k] = end[k];
    }
    // lower bound of y in each member's edge list, in lockstep
    while (true) {
      bool live = false;
      int v[kProbeWays];
#pragma unroll
      for (int k = 0; k < kProbeWays; k++) {
        v[k] = lo[k] < hi[k] ? A.col[(lo[k] + hi[k]) >> 1] : 0;
        live |= lo[k] < hi[k];
      }
      if (!live) break;
#pragma unroll
      for (int k = 0; k < kProbeWays; k++) {
        if (lo[k] < hi[k]) {
          const int mid = (lo[k] + hi[k]) >> 1;
          if (v[k] < y) lo[k] = mid + 1;
          else hi[k] = mid;
        }
      }
    }
    int hit[kProbeWays];
#pragma unroll
    for (int k = 0; k < kProbeWays; k++) hit[k] = lo[k] < end[k] ? A.col[lo[k]] : -1;
#pragma unroll
    for (int k = 0; k < kProbeWays; k++)
      if (hit[k] == y) return u[k];
  }
  return INT_MAX;
}

// (v, e) in A A^T A (equivalently (e, v) in A^T A A^T): some edge of v
// shares a node with e. E(v) is walked in ascending id order.
__device__ bool ne3_member(const Csr &A, const Csr &AT, int v, int e,
                           const Bloom &B = Bloom{nullptr, nullptr}) {
  for (int t = A.rp[v]; t < A.rp[v + 1]; t++)
    if (edges_min_common(A, AT, A.col[t], e, B) != INT_MAX) return true;
  return false;
}

// ---- pass 2: expansion ----------------------------------------------------
struct ExpandArgs {
  int pattern;
  int nrows, ncols;
  Csr l1, l2, l3;            // CSR used at each expansion level
  int levels;
  const int *quota;          // per row
  const int64_t *cap_off;    // exclusive scan of quotas
  int *out_cols;             // capacity buffer
  int *out_cnt;              // chosen per row
  const int *rows;           // rows to expand
  int nlist;
  unsigned *bitmap_g;        // per-WG bitmap slices (global mode)
  int *list_g;               // per-WG distinct lists
  int64_t list_cap;          // per-WG list capacity
  int *row_ctr;              // dynamic queue over `rows`
  uint64_t seed;
  int lds_bitmap;            // 1 -> bitmap in dynamic LDS
  int *overflow;             // set when a row has more than list_cap columns
};

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

// Walk every endpoint of row r's 2- or 3-hop expansion and insert it.
__device__ void expand_row(const ExpandArgs &A, int r, unsigned *bm, int *list,
                           SharedState &S) {
  const int tid = threadIdx.x;
  const int b1 = A.l1.rp[r], e1 = A.l1.rp[r + 1];
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

__global__ __launch_bounds__(kSB) void expand_rows(ExpandArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned s_dyn[];
  __shared__ SharedState S;
  __shared__ int s_idx;
  const int tid = threadIdx.x;
  const int nwords = (A.ncols + 31) >> 5;
  unsigned *bm = nullptr;
  int *list = nullptr;
  if (A.levels > 1) {
    bm = A.lds_bitmap ? s_dyn : A.bitmap_g + (size_t)blockIdx.x * nwords;
    list = A.list_g + (size_t)blockIdx.x * A.list_cap;
    for (int w = tid; w < nwords; w += kSB) bm[w] = 0u;
  }
  __syncthreads();
  while (true) {
    if (tid == 0) {
      s_idx = atomicAdd(A.row_ctr, 1);
      S.cnt = 0;
      S.nsel = 0;
    }
    __syncthreads();
    if (s_idx >= A.nlist) break;
    const int r = A.rows[s_idx];
    const int q = A.quota[r];
    int *out = A.out_cols + A.cap_off[r];
    if (q <= 0) {
      if (tid == 0) A.out_cnt[r] = 0;
      __syncthreads();
      continue;
    }
    const int *lst;
    int cnt;
    if (A.levels == 1) {  // the CSR row is already a distinct list
      lst = A.l1.col + A.l1.rp[r];
      cnt = A.l1.rp[r + 1] - A.l1.rp[r];
    } else {
      expand_row(A, r, bm, list, S);
      __syncthreads();
      if (tid == 0 && S.cnt > A.list_cap) atomicOr(A.overflow, 1);
      lst = list;
      cnt = (int)min((int64_t)S.cnt, A.list_cap);
    }
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
          const unsigned long long c = composite(A.seed, A.pattern, r, lst[i]);
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
        const int c = lst[i];
        if (composite(A.seed, A.pattern, r, c) <= T) {
          const int pos = atomicAdd(&S.nsel, 1);
          if (m <= kSelCap) S.sel[pos] = c;
          else out[pos] = c;
        }
      }
    } else {
      for (int i = tid; i < cnt; i += kSB) {
        if (m <= kSelCap) S.sel[i] = lst[i];
        else out[i] = lst[i];
      }
    }
    __syncthreads();
    if (m <= kSelCap) {
      bitonic_sort_int(S.sel, m);
      for (int i = tid; i < m; i += kSB) out[i] = S.sel[i];
    } else if (A.levels > 1 || m < cnt) {
      // more than kSelCap chosen in arbitrary order: sort them in place
      // (odd-even transposition over global memory; rare, big quotas only)
      for (int ph = 0; ph < m; ph++) {
        for (int i = 2 * tid + (ph & 1); i + 1 < m; i += 2 * kSB) {
          const int x = out[i], y = out[i + 1];
          if (x > y) {
            out[i] = y;
            out[i + 1] = x;
          }
        }
        __syncthreads();
      }
    }
    if (tid == 0) A.out_cnt[r] = m;
    // clear exactly the bits that were set
    if (A.levels > 1)
      for (int i = tid; i < cnt; i += kSB) {
        const int c = list[i];
        bm[c >> 5] = 0u;
      }
    __syncthreads();
  }
}

// ---- pass 1: rejection sampling of large 2/3-hop rows --------------------
struct RejectArgs {
  int pattern;
  int nrows, ncols;
  Csr l1, l2, l3;
  int levels;
  Csr A, AT;                 // node -> edges, edge -> nodes
  const int *quota;
  const int64_t *cap_off;
  int *out_cols, *out_cnt;
  const int *rows;
  int nlist;
  int *row_ctr;
  int *defer_small, *defer_big, *ndefer;  // ndefer[0] small, [1] big
  uint64_t seed;
  int64_t reject_w;
  const int64_t *ps;         // 3-hop: exclusive scan over l2's incidences of
                             // |l3 row of the incidence's column| (nnz + 1)
  int mode3;                 // 0 auto, 1 paths, 2 uniform columns
  int mode3_shift;           // auto: uniform columns when W >= ncols * 2^mode3_shift
  int *stats;                // [0] rejection rows, [1] stalled, [3] uniform-mode rows
  Bloom bloom;               // member filters of the edges (3-hop patterns)
  long long *diag;           // debug builds: per-row {pattern, row, mode, n1, q, W,
  int *diag_n;               // rounds, s_memrealtime ticks} (HGX_REJ_DIAG_OUT)
  int diag_cap;
};

constexpr int kEvBits = 9;  // LDS hash of a node row's edges (<= kSB of them)
constexpr int kEvHash = 1 << kEvBits;

struct RejShared {
  int sel[kSelCap];
  int hash[kHash];
  int ev[kEvHash];  // PAT_NNE rejection rows: the row's edges E(v)
  int evid[kSB];    // and in E(v)'s (ascending) order
  int evsz[kSB];    // with their sizes
  int nev;          // |E(v)| when staged, else -1
  unsigned long long key[kSB];
  int flag[kSB];
  int a_id[kSB];
  long long a_off[kSB];
  long long wsl[kSB / 64];
  long long wml[kSB / 64];
  int ws[kSB / 64];
  int nsel;
  int idx;
};

__device__ __forceinline__ unsigned hslot(int c) {
  return ((unsigned)c * 2654435761u) >> (32 - kHashBits);
}
__device__ bool hash_has(const int *h, int c) {
  unsigned s = hslot(c);
  while (true) {
    const int k = h[s];
    if (k == c) return true;
    if (k < 0) return false;
    s = (s + 1) & (kHash - 1);
  }
}
__device__ void hash_put(int *h, int c) {
  unsigned s = hslot(c);
  while (true) {
    const int old = atomicCAS(&h[s], -1, c);
    if (old == -1 || old == c) return;
    s = (s + 1) & (kHash - 1);
  }
}

__device__ __forceinline__ unsigned evslot(int e) {
  return ((unsigned)e * 2654435761u) >> (32 - kEvBits);
}
__device__ bool ev_has(const int *h, int e) {
  unsigned s = evslot(e);
  while (true) {
    const int k = h[s];
    if (k == e) return true;
    if (k < 0) return false;
    s = (s + 1) & (kEvHash - 1);
  }
}

// With E(v) staged in LDS (S.ev, ids S.evid, sizes S.evsz; ascending):
// does some member u of edge c have an edge f of E(v) with f < lim? Each
// member costs its contiguous edge list (read kEvRead ids at a time, all
// loads before the LDS probes), members kEvWays at a time. The other walk
// -- every such f intersected with c from the smaller side, a binary search
// per probed node -- is cheaper when c is far larger than the row's edges:
// nne_meets picks by the probe counts. The same answer either way.
constexpr int kEvWays = 4;
constexpr int kEvRead = 8;
__device__ bool members_meet_ev(const RejectArgs &A, const RejShared &S, int c, int lim) {
  const int cb = A.AT.rp[c], ce = A.AT.rp[c + 1];
  for (int t = cb; t < ce; t += kEvWays) {
    int ub[kEvWays], ue[kEvWays];
#pragma unroll
    for (int k = 0; k < kEvWays; k++) {
      const int u = t + k < ce ? A.AT.col[t + k] : -1;
      ub[k] = u >= 0 ? A.A.rp[u] : 0;
      ue[k] = u >= 0 ? A.A.rp[u + 1] : 0;
    }
#pragma unroll
    for (int k = 0; k < kEvWays; k++) {
      for (int a0 = ub[k]; a0 < ue[k]; a0 += kEvRead) {
        int f[kEvRead];
#pragma unroll
        for (int j = 0; j < kEvRead; j++) f[j] = a0 + j < ue[k] ? A.A.col[a0 + j] : INT_MAX;
#pragma unroll
        for (int j = 0; j < kEvRead; j++)
          if (f[j] < lim && ev_has(S.ev, f[j])) return true;
      }
    }
  }
  return false;
}

// some e1 of E(v) with e1 < lim meets edge c (lim = INT_MAX: (v, c) in
// A A^T A); E(v) staged in LDS
__device__ bool nne_meets(const RejectArgs &A, const RejShared &S, int v, int c, int lim) {
  const int nc = A.AT.rp[c + 1] - A.AT.rp[c];
  long long probes = 0;
  for (int j = 0; j < S.nev && S.evid[j] < lim; j++) probes += min(S.evsz[j], nc);
  if (probes == 0) return false;
  if (2ll * nc <= 5ll * probes) return members_meet_ev(A, S, c, lim);
  for (int j = 0; j < S.nev && S.evid[j] < lim; j++)
    if (edges_min_common(A.A, A.AT, S.evid[j], c, A.bloom) != INT_MAX) return true;
  return false;
}

// path count of level-1 entity m of row r
__device__ __forceinline__ long long level1_weight(const RejectArgs &A, int m) {
  if (A.levels == 2) return A.l2.rp[m + 1] - A.l2.rp[m];
  return A.ps[A.l2.rp[m + 1]] - A.ps[A.l2.rp[m]];
}

__device__ __forceinline__ uint64_t umulhi64(uint64_t h, uint64_t n) {
  return __umul64hi(h, n);
}

// One candidate draw for row r (INT_MAX = rejected). mode: 0 2-hop paths,
// 1 3-hop paths, 2 3-hop uniform columns.
__device__ int draw_candidate(const RejectArgs &A, int r, int mode, bool small,
                              int n1, long long W, long long wmax,
                              const RejShared &S, uint64_t h) {
  const int b1 = A.l1.rp[r];
  const uint64_t h2 = hgx::mix64(h ^ 0x51ed27ull);
  const uint64_t h3 = hgx::mix64(h2 ^ 0xa5a5a5a5ull);
  if (mode == 2) {
    const int c = (int)hgx::bounded(h, (uint32_t)A.ncols);
    if (hash_has(S.hash, c)) return INT_MAX;
    const bool in = A.pattern == PAT_NNE ? (S.nev >= 0 ? nne_meets(A, S, r, c, INT_MAX)
                                                       : ne3_member(A.A, A.AT, r, c, A.bloom))
                                         : ne3_member(A.A, A.AT, c, r, A.bloom);
    return in ? c : INT_MAX;
  }
  // uniform path: level-1 entity m1 and the path offset w1 inside it
  int m1;
  long long w1;
  if (small) {
    const long long w = (long long)umulhi64(h, (uint64_t)W);
    const int j = upper_find(S.a_off, n1, w);
    m1 = S.a_id[j];
    w1 = w - S.a_off[j];
  } else {  // m1 uniform, accepted with weight / max weight
    m1 = A.l1.col[b1 + (int)hgx::bounded(h, (uint32_t)n1)];
    const long long wt = level1_weight(A, m1);
    if ((long long)umulhi64(h2, (uint64_t)wmax) >= wt) return INT_MAX;
    w1 = (long long)umulhi64(h3, (uint64_t)wt);
  }
  if (mode == 0) {
    const int c = A.l2.col[A.l2.rp[m1] + (int)w1];
    if (hash_has(S.hash, c)) return INT_MAX;
    const int f = first_common(A.l1.col + b1, A.l1.rp[r + 1] - b1,
                               A.l1.col + A.l1.rp[c], A.l1.rp[c + 1] - A.l1.rp[c]);
    return f == m1 ? c : INT_MAX;
  }
  // 3-hop: m2 = the l2 incidence t of m1 whose prefix interval holds w1
  const int tb = A.l2.rp[m1], te = A.l2.rp[m1 + 1];
  const long long target = A.ps[tb] + w1;
  int lo = tb, hi = te - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (A.ps[mid] <= target) lo = mid;
    else hi = mid - 1;
  }
  const int m2 = A.l2.col[lo];
  const int c = A.l3.col[A.l3.rp[m2] + (int)(target - A.ps[lo])];
  if (hash_has(S.hash, c)) return INT_MAX;
  // canonical (first) path to c, lexicographic in (m1, m2)
  if (A.pattern == PAT_NNE) {
    // r = v, m1 = e1 in E(v), m2 = u in e1, c = e: the first e1 of E(v)
    // meeting e, then the smallest common member (a walk over e's members
    // against E(v) in LDS measured slower here: an accepted path must rule
    // out every earlier e1, so it reads all of e's members, where this loop
    // stops at the first e1 meeting e -- usually an early, large one)
    for (int t = b1; t < A.l1.rp[r + 1]; t++) {
      const int e1 = A.l1.col[t];
      if (e1 > m1) break;
      const int u = edges_min_common(A.A, A.AT, e1, c, A.bloom);
      if (u != INT_MAX) return (e1 == m1 && u == m2) ? c : INT_MAX;
    }
    return INT_MAX;
  }
  // PAT_EEN: r = e, m1 = u in e, m2 = e2 in E(u), c = v: the first member u
  // of e with E(u) ∩ E(v) non-empty, then its smallest common edge
  const int *ev = A.A.col + A.A.rp[c];
  const int nev = A.A.rp[c + 1] - A.A.rp[c];
  for (int t = b1; t < A.l1.rp[r + 1]; t++) {
    const int u = A.l1.col[t];
    if (u > m1) break;
    const int f = first_common(A.A.col + A.A.rp[u], A.A.rp[u + 1] - A.A.rp[u], ev, nev);
    if (f != INT_MAX) return (u == m1 && f == m2) ? c : INT_MAX;
  }
  return INT_MAX;
}

__global__ __launch_bounds__(kSB) void reject_rows(RejectArgs A) {
  __shared__ RejShared S;
  const int tid = threadIdx.x;
  while (true) {
    if (tid == 0) S.idx = atomicAdd(A.row_ctr, 1);
    __syncthreads();
    const int i = S.idx;
    if (i >= A.nlist) break;
    const int r = A.rows[i];
    const int q = A.quota[r];
    if (q <= 0) {
      if (tid == 0) A.out_cnt[r] = 0;
      __syncthreads();
      continue;
    }
    if (q > kSelCap) {
      if (tid == 0) A.defer_big[atomicAdd(&A.ndefer[1], 1)] = r;
      __syncthreads();
      continue;
    }
    // path count W and max level-1 weight of the row
    const int b1 = A.l1.rp[r], e1 = A.l1.rp[r + 1], n1 = e1 - b1;
    long long w = 0, wm = 0;
    for (int t = b1 + tid; t < e1; t += kSB) {
      const long long x = level1_weight(A, A.l1.col[t]);
      w += x;
      wm = max(wm, x);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      w += __shfl_xor(w, off);
      wm = max(wm, (long long)__shfl_xor(wm, off));
    }
    if ((tid & 63) == 0) {
      S.wsl[tid >> 6] = w;
      S.wml[tid >> 6] = wm;
    }
    __syncthreads();
    long long W = 0, wmax = 0;
#pragma unroll
    for (int k = 0; k < kSB / 64; k++) {
      W += S.wsl[k];
      wmax = max(wmax, S.wml[k]);
    }
    __syncthreads();
    if (W <= A.reject_w) {
      if (tid == 0) A.defer_small[atomicAdd(&A.ndefer[0], 1)] = r;
      __syncthreads();
      continue;
    }
    int mode = 0;
    if (A.levels == 3)
      mode = (A.mode3 == 2 ||
              (A.mode3 == 0 && (A.mode3_shift >= 0 ? W >= ((long long)A.ncols << A.mode3_shift)
                                                   : (W << -A.mode3_shift) >= (long long)A.ncols)))
                 ? 2
                 : 1;
    const bool small = n1 <= kSB;
    if (mode != 2 && small) {  // exact path draws: prefix of weights in LDS
      long long x = 0;
      int id1 = -1;
      if (tid < n1) {
        id1 = A.l1.col[b1 + tid];
        x = level1_weight(A, id1);
      }
      long long tot;
      const long long o1 = block_scan_excl64(x, &tot, S.wsl);
      S.a_id[tid] = id1;
      S.a_off[tid] = o1;
    }
    for (int k = tid; k < kHash; k += kSB) S.hash[k] = -1;
    if (tid == 0) S.nsel = 0;
    // uniform columns of a node row: its edges into LDS for the membership
    // test (nne_meets)
    const bool stage_ev = mode == 2 && A.pattern == PAT_NNE && n1 <= kSB;
    for (int k = tid; k < kEvHash; k += kSB) S.ev[k] = -1;
    if (tid == 0) S.nev = stage_ev ? n1 : -1;
    __syncthreads();
    if (stage_ev && tid < n1) {
      const int e1 = A.l1.col[b1 + tid];
      S.evid[tid] = e1;
      S.evsz[tid] = A.AT.rp[e1 + 1] - A.AT.rp[e1];
      unsigned sl = evslot(e1);
      while (true) {
        const int old = atomicCAS(&S.ev[sl], -1, e1);
        if (old == -1 || old == e1) break;
        sl = (sl + 1) & (kEvHash - 1);
      }
    }
    __syncthreads();
    int stall = 0;
    bool done = false;
#ifdef HGX_DEBUG_KNOBS
    const unsigned long long t_row = __builtin_amdgcn_s_memrealtime();
    int rounds_used = 0;
#endif
    for (int round = 0; round < 4096; round++) {
#ifdef HGX_DEBUG_KNOBS
      rounds_used = round + 1;
#endif
      const uint64_t base = ((uint64_t)(uint32_t)r << 32) ^ ((uint64_t)round << 12);
      const uint64_t h = hgx::rand64(A.seed, 0x300 + A.pattern, base + tid);
      const int cand = draw_candidate(A, r, mode, small, n1, W, wmax, S, h);
      // repeats inside the round: keep the lowest thread (sort (col, tid))
      S.key[tid] = ((unsigned long long)(unsigned)cand << 32) | (unsigned)tid;
      __syncthreads();
      for (int size = 2; size <= kSB; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          if (tid < kSB / 2) {
            const int lo = 2 * tid - (tid & (stride - 1)), hi = lo + stride;
            const bool up = (lo & size) == 0;
            const unsigned long long x = S.key[lo], y = S.key[hi];
            if ((x > y) == up) {
              S.key[lo] = y;
              S.key[hi] = x;
            }
          }
          __syncthreads();
        }
      }
      {
        const unsigned long long k = S.key[tid];
        const int col = (int)(k >> 32);
        const bool fresh = col != INT_MAX &&
                           (tid == 0 || (int)(S.key[tid - 1] >> 32) != col);
        S.flag[(int)(k & 0xffffffffu)] = fresh ? 1 : 0;
      }
      __syncthreads();
      int total;
      const int rank = block_scan_excl(S.flag[tid], &total, S.ws);
      const int need = q - S.nsel;
      if (S.flag[tid] && rank < need) {
        S.sel[S.nsel + rank] = cand;
        hash_put(S.hash, cand);
      }
      __syncthreads();
      const int got = min(total, need);
      if (tid == 0) S.nsel += got;
      __syncthreads();
      if (S.nsel >= q) {
        done = true;
        break;
      }
      stall = got ? 0 : stall + 1;
      if (stall >= 32) break;
    }
#ifdef HGX_DEBUG_KNOBS
    if (A.diag && tid == 0) {
      const int k = atomicAdd(A.diag_n, 1);
      if (k < A.diag_cap) {
        long long *o = A.diag + 8ll * k;
        o[0] = A.pattern;
        o[1] = r;
        o[2] = done ? mode : -1 - mode;
        o[3] = n1;
        o[4] = q;
        o[5] = W;
        o[6] = rounds_used;
        o[7] = (long long)(__builtin_amdgcn_s_memrealtime() - t_row);
      }
    }
#endif
    if (!done) {  // the union looks smaller than q: expand it (pass 2)
      if (tid == 0) {
        A.defer_big[atomicAdd(&A.ndefer[1], 1)] = r;
        atomicAdd(&A.stats[1], 1);
      }
      __syncthreads();
      continue;
    }
    if (tid == 0) {
      atomicAdd(&A.stats[0], 1);
      if (mode == 2) atomicAdd(&A.stats[3], 1);
    }
    bitonic_sort_int(S.sel, q);
    int *out = A.out_cols + A.cap_off[r];
    for (int k = tid; k < q; k += kSB) out[k] = S.sel[k];
    if (tid == 0) A.out_cnt[r] = q;
    __syncthreads();
  }
}

// rows with a positive quota (order irrelevant: every draw is keyed by row)
__global__ void list_rows(const int *q, int n, int *rows, int *cnt) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += gridDim.x * blockDim.x) {
    if (q[i] > 0) rows[atomicAdd(cnt, 1)] = i;
  }
}

// |row of l3| summed over l2's incidences: val[t] = |l3 row l2.col[t]|
struct L3Len {
  const int *col2, *rp3;
  __host__ __device__ int64_t operator()(int t) const {
    const int c = col2[t];
    return (int64_t)(rp3[c + 1] - rp3[c]);
  }
};
__global__ void ps_finish(int64_t *p, int64_t n, L3Len g) {
  if (threadIdx.x == 0 && blockIdx.x == 0)
    p[n] = n ? p[n - 1] + g((int)(n - 1)) : 0;
}

// ---- record materialisation ----------------------------------------------
using hgx::REC_NN;
using hgx::REC_EE;
using hgx::REC_NE_NODE;
using hgx::REC_NE_EDGE;

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

// _sample_neighbors for the node-edge records of one kind block [b, e):
// nn_k from N(re-1), ne_k from E(ln-1), K draws with replacement each
// (hgx::draw_record_neighbors). The draws are keyed by (stream, block row,
// key): the row is id column `rowcol` of the record, the key its column
// (the other id: sampled columns are distinct within a row) or, for
// negatives (key_col 0, drawn with replacement), its rank in the row (its
// records start at b + off[row]). A record therefore draws the same
// neighbours whichever row range or rank emitted it, whatever its position,
// and the record store reloads it with them (hgx_store_load). An endpoint
// with no neighbours (possible for negatives of a graph with an isolated
// node or an empty edge) is an error, as np.random.choice on an empty row
// raises ValueError in the reference (hg2v_sample.py:49-51).
__global__ void draw_neighbors(int64_t b, int64_t e, int K, int R, int *idx,
                               const int64_t *off, int rowcol, int key_col,
                               const int *rp_n, const int *col_n,
                               const int *rp_e, const int *col_e,
                               uint64_t seed, uint64_t stream, int *err) {
  for (int64_t rec = b + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; rec < e;
       rec += (int64_t)gridDim.x * blockDim.x) {
    int *ri = idx + rec * R;
    const int v = ri[0] - 1, ed = ri[3] - 1;
    const int nb = rp_e[ed], nl = rp_e[ed + 1] - nb;
    const int eb = rp_n[v], el = rp_n[v + 1] - eb;
    if (nl == 0 || el == 0) {
      atomicOr(err, 1);
      continue;
    }
    const int row = ri[rowcol] - 1;
    const uint64_t key = key_col ? (uint64_t)(rowcol == 0 ? ed : v)
                                 : (uint64_t)(rec - b - off[row]);
    hgx::draw_record_neighbors(seed, stream, row, key, K, nb, nl, eb, el, col_e,
                               col_n, ri + 4);
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
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, out, n + 1, ctx->stream));
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

// pass 2 over `rows` (device list of n rows) with lists of list_cap columns
int expand_pass(hgx_ctx *ctx, const ExpandArgs &base, const int *rows, int n,
                int64_t list_cap) {
  if (n == 0) return HGX_OK;
  ExpandArgs a = base;
  const int nwords = (a.ncols + 31) / 32;
  const bool lds = a.levels > 1 && (size_t)nwords * 4 <= 48 * 1024;
  int nwg = 1024;
  if (a.levels > 1)
    while (nwg > 64 && (double)nwg * (list_cap * 4 + (lds ? 0 : nwords * 4)) > 4e9)
      nwg /= 2;
  nwg = std::min(nwg, std::max(n, 1));
  DevBuf list, bmap;
  if (a.levels > 1) {
    HGX_TRY(hgx_ensure(ctx, list, sizeof(int) * (size_t)nwg * list_cap + 16));
    if (!lds) {
      int rc = hgx_ensure(ctx, bmap, sizeof(unsigned) * (size_t)nwg * nwords);
      if (rc != HGX_OK) {
        hgx_release(list);
        return rc;
      }
    }
  }
  a.rows = rows;
  a.nlist = n;
  a.list_g = list.as<int>();
  a.bitmap_g = lds ? nullptr : bmap.as<unsigned>();
  a.list_cap = list_cap;
  a.lds_bitmap = lds;
  int rc = HGX_OK;
  if (hipMemsetAsync(a.row_ctr, 0, sizeof(int), ctx->stream) != hipSuccess)
    rc = hgx_fail(ctx, HGX_EHIP, "expand_rows queue reset failed");
  if (rc == HGX_OK) {
    hipLaunchKernelGGL(expand_rows, dim3(nwg), dim3(kSB), lds ? (size_t)nwords * 4 : 0,
                       ctx->stream, a);
    if (hipGetLastError() != hipSuccess)
      rc = hgx_fail(ctx, HGX_EHIP, "expand_rows launch failed");
  }
  if (hipStreamSynchronize(ctx->stream) != hipSuccess && rc == HGX_OK)
    rc = hgx_fail(ctx, HGX_EHIP, "expand_rows failed");
  hgx_release(list);
  hgx_release(bmap);
  return rc;
}

// filter words of edge e: 16 per 64-byte block, a power of two of blocks
// holding >= 16 bits per member
__global__ void bloom_words(const int *rp_e, int E, long long *words) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < E; e += gridDim.x * blockDim.x) {
    const long long want = (16ll * (rp_e[e + 1] - rp_e[e]) + 511) / 512;
    long long b = 1;
    while (b < want) b <<= 1;
    words[e] = 16 * b;
  }
}

// the 3 bits of every incidence (edge of incidence t by binary search)
__global__ void bloom_set(const int *rp_e, const int *col_e, int E, int64_t nnz,
                          const long long *off, unsigned *bits) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nnz;
       t += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = E - 1;
    while (lo < hi) {  // last edge e with rp_e[e] <= t
      const int mid = (lo + hi + 1) >> 1;
      if (rp_e[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    const long long o = off[lo];
    const unsigned bmask = (unsigned)((off[lo + 1] - o) / 16 - 1);
    const uint64_t h = bloom_hash(col_e[t]);
    unsigned *blk = bits + o + 16 * ((unsigned)(h >> 40) & bmask);
    const unsigned s0 = (unsigned)h & 511, s1 = (unsigned)(h >> 9) & 511,
                   s2 = (unsigned)(h >> 18) & 511;
    atomicOr(&blk[s0 >> 5], 1u << (s0 & 31));
    atomicOr(&blk[s1 >> 5], 1u << (s1 & 31));
    atomicOr(&blk[s2 >> 5], 1u << (s2 & 31));
  }
}

int ensure_bloom(hgx_ctx *ctx) {
  if (ctx->bloom_ok) return HGX_OK;
  const int E = ctx->E;
  HGX_TRY(hgx_ensure(ctx, ctx->bloom_off, sizeof(long long) * (E + 1)));
  long long *off = ctx->bloom_off.as<long long>();
  hipLaunchKernelGGL(bloom_words, dim3(grid_for(E, 256, 65536)), dim3(256), 0,
                     ctx->stream, ctx->rp_e.as<int>(), E, off);
  HGX_LAUNCH_CHECK(ctx);
  HGX_HIP(ctx, hipMemsetAsync(off + E, 0, sizeof(long long), ctx->stream));
  size_t tmp = 0;
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, off, off, E + 1, ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->s7, tmp + 256));
  HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(ctx->s7.p, tmp, off, off, E + 1, ctx->stream));
  long long words = 0;
  HGX_HIP(ctx, hipMemcpyAsync(&words, off + E, sizeof(long long), hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  HGX_TRY(hgx_ensure(ctx, ctx->bloom_bits, sizeof(unsigned) * (size_t)(words + 16)));
  HGX_HIP(ctx, hipMemsetAsync(ctx->bloom_bits.p, 0, sizeof(unsigned) * (size_t)(words + 16),
                              ctx->stream));
  if (ctx->nnz > 0) {
    hipLaunchKernelGGL(bloom_set, dim3(grid_for(ctx->nnz, 256, 65536)), dim3(256), 0,
                       ctx->stream, ctx->rp_e.as<int>(), ctx->col_e.as<int>(), E, ctx->nnz,
                       off, ctx->bloom_bits.as<unsigned>());
    HGX_LAUNCH_CHECK(ctx);
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->bloom_ok = true;
  return HGX_OK;
}

int run_pattern(hgx_ctx *ctx, int pattern, const int32_t *host_quota,
                int quota_all, uint64_t seed, PatOut &po) {
  const int N = ctx->N, E = ctx->E;
  const Csr A{ctx->rp_n.as<int>(), ctx->col_n.as<int>()};
  const Csr AT{ctx->rp_e.as<int>(), ctx->col_e.as<int>()};
  ExpandArgs a{};
  a.pattern = pattern;
  switch (pattern) {
    case PAT_A: a.nrows = N; a.ncols = E; a.l1 = A; a.levels = 1; break;
    case PAT_AT: a.nrows = E; a.ncols = N; a.l1 = AT; a.levels = 1; break;
    case PAT_NN: a.nrows = N; a.ncols = N; a.l1 = A; a.l2 = AT; a.levels = 2; break;
    case PAT_EE: a.nrows = E; a.ncols = E; a.l1 = AT; a.l2 = A; a.levels = 2; break;
    case PAT_NNE: a.nrows = N; a.ncols = E; a.l1 = A; a.l2 = AT; a.l3 = A; a.levels = 3; break;
    default: a.nrows = E; a.ncols = N; a.l1 = AT; a.l2 = A; a.l3 = AT; a.levels = 3; break;
  }
  // (before any work is queued: the build may grow the shared scratch)
  if (a.levels == 3 && ctx->tune.sample_reject_w > 0) HGX_TRY(ensure_bloom(ctx));
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
  // counters: [0] row queue, [1] listed rows, [2] deferred small, [3]
  // deferred big, [4] overflow, [5..8] rejection stats
  HGX_TRY(hgx_ensure(ctx, ctx->s0, 64));
  int *ctr = ctx->s0.as<int>();
  HGX_HIP(ctx, hipMemsetAsync(ctr, 0, 64, ctx->stream));
  // rows with a quota; two deferral lists
  DevBuf rows, dsmall, dbig;
  HGX_TRY(hgx_ensure(ctx, rows, sizeof(int) * (R + 1)));
  hipLaunchKernelGGL(list_rows, dim3(grid_for(R, 256)), dim3(256), 0,
                     ctx->stream, po.q.as<int>(), R, rows.as<int>(), ctr + 1);
  HGX_LAUNCH_CHECK(ctx);
  int nlist = 0;
  HGX_HIP(ctx, hipMemcpyAsync(&nlist, ctr + 1, sizeof(int), hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  a.quota = po.q.as<int>();
  a.cap_off = po.cap_off.as<int64_t>();
  a.out_cols = po.cols.as<int>();
  a.out_cnt = po.cnt.as<int>();
  a.row_ctr = ctr;
  a.seed = seed;
  a.overflow = ctr + 4;
  const int64_t reject_w = ctx->tune.sample_reject_w;
  const bool reject = a.levels > 1 && reject_w > 0;
  int st[4] = {0, 0, 0, 0};
  if (!reject) {
    HGX_TRY(expand_pass(ctx, a, rows.as<int>(), nlist,
                        a.levels == 1 ? 0 : (int64_t)a.ncols));
  } else {
    HGX_TRY(hgx_ensure(ctx, dsmall, sizeof(int) * (nlist + 1)));
    HGX_TRY(hgx_ensure(ctx, dbig, sizeof(int) * (nlist + 1)));
    DevBuf ps;
    if (a.levels == 3) {  // path counts through l2's incidences
      const int64_t nnz = ctx->nnz;
      HGX_TRY(hgx_ensure(ctx, ps, sizeof(int64_t) * (nnz + 1)));
      L3Len f{a.l2.col, a.l3.rp};
      hipcub::CountingInputIterator<int> ci(0);
      hipcub::TransformInputIterator<int64_t, L3Len, hipcub::CountingInputIterator<int>>
          it(ci, f);
      size_t tmp = 0;
      // the value at t == nnz is never used: scan nnz values, then the total
      HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, ps.as<int64_t>(),
                                                    nnz, ctx->stream));
      HGX_TRY(hgx_ensure(ctx, ctx->s7, tmp + 256));
      HGX_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(ctx->s7.p, tmp, it,
                                                    ps.as<int64_t>(), nnz,
                                                    ctx->stream));
      // ps[nnz] = ps[nnz-1] + val[nnz-1]
      hipLaunchKernelGGL(ps_finish, dim3(1), dim3(64), 0, ctx->stream,
                         ps.as<int64_t>(), nnz, f);
      HGX_LAUNCH_CHECK(ctx);
    }
    RejectArgs r{};
    r.pattern = pattern;
    r.nrows = a.nrows;
    r.ncols = a.ncols;
    r.l1 = a.l1;
    r.l2 = a.l2;
    r.l3 = a.l3;
    r.levels = a.levels;
    r.A = A;
    r.AT = AT;
    r.quota = a.quota;
    r.cap_off = a.cap_off;
    r.out_cols = a.out_cols;
    r.out_cnt = a.out_cnt;
    r.rows = rows.as<int>();
    r.nlist = nlist;
    r.row_ctr = ctr;
    r.defer_small = dsmall.as<int>();
    r.defer_big = dbig.as<int>();
    r.ndefer = ctr + 2;
    r.seed = seed;
    r.reject_w = reject_w;
    r.ps = ps.as<int64_t>();
    r.mode3 = ctx->tune.sample_mode3;
    r.mode3_shift = pattern == PAT_EEN ? ctx->tune.sample_mode3_shift_e
                                       : ctx->tune.sample_mode3_shift;
    r.stats = ctr + 5;
    if (a.levels == 3)
      r.bloom = Bloom{ctx->bloom_off.as<long long>(), ctx->bloom_bits.as<unsigned>()};
    DevBuf diag;
#ifdef HGX_DEBUG_KNOBS
    const char *diag_out = hgx_debug_env_str("HGX_REJ_DIAG_OUT");
    if (diag_out && nlist > 0) {
      HGX_TRY(hgx_ensure(ctx, diag, sizeof(long long) * 8 * (size_t)nlist + 64));
      HGX_HIP(ctx, hipMemsetAsync(diag.p, 0, 64, ctx->stream));
      r.diag_n = diag.as<int>();
      r.diag = reinterpret_cast<long long *>(diag.as<char>() + 64);
      r.diag_cap = nlist;
    }
#endif
    if (nlist > 0) {
      int dev = 0, ncu = 256;
      HGX_HIP(ctx, hipGetDevice(&dev));
      HGX_HIP(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      const int nwg = std::min(nlist, 4 * ncu);
      hipLaunchKernelGGL(reject_rows, dim3(nwg), dim3(kSB), 0, ctx->stream, r);
      HGX_LAUNCH_CHECK(ctx);
    }
#ifdef HGX_DEBUG_KNOBS
    if (r.diag) {
      int nd = 0;
      HGX_HIP(ctx, hipMemcpyAsync(&nd, diag.p, sizeof(int), hipMemcpyDeviceToHost,
                                  ctx->stream));
      HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
      nd = std::min(nd, nlist);
      std::vector<long long> h(8 * (size_t)nd);
      HGX_HIP(ctx, hipMemcpy(h.data(), r.diag, sizeof(long long) * h.size(),
                             hipMemcpyDeviceToHost));
      if (FILE *f = fopen(diag_out, "ab")) {
        fwrite(h.data(), sizeof(long long), h.size(), f);
        fclose(f);
      }
    }
#endif
    int nd[2] = {0, 0};
    HGX_HIP(ctx, hipMemcpyAsync(nd, ctr + 2, sizeof(nd), hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(st, ctr + 5, sizeof(st), hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    hgx_release(ps);
    hgx_release(diag);
    // deferred rows: small ones have at most reject_w distinct columns
    HGX_TRY(expand_pass(ctx, a, dsmall.as<int>(), nd[0],
                        std::min<int64_t>(a.ncols, std::max<int64_t>(2 * reject_w, 65536))));
    HGX_TRY(expand_pass(ctx, a, dbig.as<int>(), nd[1], (int64_t)a.ncols));
  }
  int ovf = 0;
  HGX_HIP(ctx, hipMemcpyAsync(&ovf, ctr + 4, sizeof(int), hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->sample_union_rows += st[0];
  ctx->sample_fallback_rows += st[1];
  ctx->sample_uniform_rows += st[3];
  HGX_CHECK(ctx, ovf == 0, HGX_EUNSUP,
            "a sampled row has more distinct columns than its expansion list");
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
  ctx->rec_in_order = false;
  ctx->store_carry = 0;  // no store batch tail survives a rewrite
  ctx->smp_family = -1;  // set by the sampler once its records are complete
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

// neighbour draws of one node-edge kind block: records [b, b + n), row of a
// record = id column rowcol (0: node rows, 3: edge rows), row r's records at
// b + off[r] (the block's exclusive record scan)
int neighbors(hgx_ctx *ctx, int64_t b, int64_t n, const DevBuf &off,
              int rowcol, uint64_t seed, uint64_t stream, int key_col) {
  if (n <= 0) return HGX_OK;
  const int64_t e = b + n;
  HGX_TRY(hgx_ensure(ctx, ctx->s1, 16));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s1.p, 0, sizeof(int), ctx->stream));
  hipLaunchKernelGGL(draw_neighbors, dim3(grid_for(e - b, 256)), dim3(256), 0,
                     ctx->stream, b, e, ctx->K, 4 + 2 * ctx->K,
                     ctx->rec_idx.as<int>(), off.as<int64_t>(), rowcol, key_col,
                     ctx->rp_n.as<int>(), ctx->col_n.as<int>(),
                     ctx->rp_e.as<int>(), ctx->col_e.as<int>(), seed, stream,
                     ctx->s1.as<int>());
  HGX_LAUNCH_CHECK(ctx);
  int err = 0;
  HGX_HIP(ctx, hipMemcpyAsync(&err, ctx->s1.p, sizeof(int), hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  HGX_CHECK(ctx, err == 0, HGX_EVALUE,
            "a cannot be empty unless no samples are taken (_sample_neighbors "
            "on a node without edges or an edge without nodes, "
            "hg2v_sample.py:49-51)");
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

// kind-block bounds of the record stream just emitted (hgx_records_blocks)
void set_blocks(hgx_ctx *ctx, std::initializer_list<int64_t> b) {
  int i = 0;
  for (int64_t v : b) ctx->rec_bounds[i++] = v;
  ctx->n_rec_blocks = i - 1;
}

void reset_stats(hgx_ctx *ctx) {
  ctx->sample_union_rows = ctx->sample_fallback_rows = 0;
  ctx->sample_uniform_rows = 0;
}

}  // namespace

// HOBE probability kernels live in hgx_hobe.hip
int hgx_hobe_prepare(hgx_ctx *ctx);
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
  reset_stats(ctx);
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
  HGX_TRY(neighbors(ctx, o_ne, ne_n.total, ne_n.rec_off, 0, seed, 0x200, 1));
  HGX_TRY(neighbors(ctx, o_en, ne_e.total, ne_e.rec_off, 3, seed, 0x201, 1));
  if (neg_node_quota) {
    HGX_TRY(neg_emit(ctx, REC_NN, gnn, ctx->N, o_neg, seed, 0x300));
    HGX_TRY(neg_emit(ctx, REC_EE, gee, ctx->E, o_gee, seed, 0x301));
    // the reference's "Node-Edge Negatives" block repeats edge-edge
    // sampling (hg2v_sample.py:215-221); kept for parity of counts
    HGX_TRY(neg_emit(ctx, REC_EE, gee, ctx->E, o_gee2, seed, 0x302));
    HGX_TRY(neg_emit(ctx, REC_NE_NODE, gne_n, ctx->E, o_gne, seed, 0x303));
    HGX_TRY(neg_emit(ctx, REC_NE_EDGE, gne_e, ctx->N, o_gen, seed, 0x304));
    HGX_TRY(neighbors(ctx, o_gne, gne_n.total, gne_n.off, 0, seed, 0x400, 0));
    HGX_TRY(neighbors(ctx, o_gen, gne_e.total, gne_e.off, 3, seed, 0x401, 0));
    set_blocks(ctx, {0, o_ee, o_ne, o_en, o_neg, o_gee, o_gee2, o_gne, o_gen, total});
  } else {
    set_blocks(ctx, {0, o_ee, o_ne, o_en, total});
  }
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->smp_family = 0;
  ctx->smp_seed = seed;
  if (n_records) *n_records = total;
  return HGX_OK;
}

extern "C" int hgx_sample_hobe_rows(hgx_ctx *ctx, uint64_t seed, int K,
                                    const int32_t *node_quota,
                                    const int32_t *edge_quota, int S,
                                    int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_CHECK(ctx, ctx->k > 0, HGX_ESTATE,
            "HOBE needs the algebraic-distance coords on device");
  HGX_CHECK(ctx, K >= 1 && K <= 16, HGX_EUNSUP, "num_neighbors %d outside [1,16]", K);
  HGX_CHECK(ctx, S >= 0, HGX_EINVAL, "num_samples must be >= 0 (hg2v_sample.py:647)");
  HGX_CHECK(ctx, (node_quota == nullptr) == (edge_quota == nullptr), HGX_EINVAL,
            "give both row quotas or neither");
  if (node_quota) {
    HGX_TRY(check_quota(ctx, node_quota, ctx->N, "node"));
    HGX_TRY(check_quota(ctx, edge_quota, ctx->E, "edge"));
  }
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  reset_stats(ctx);
  // AlgebraicDistanceSamples order (hg2v_sample.py:658-715)
  PatOut nn, ee, ne_n, ne_e;
  HGX_TRY(run_pattern(ctx, PAT_NN, node_quota, S, seed, nn));
  HGX_TRY(run_pattern(ctx, PAT_EE, edge_quota, S, seed, ee));
  HGX_TRY(run_pattern(ctx, PAT_NNE, node_quota, S, seed, ne_n));
  HGX_TRY(run_pattern(ctx, PAT_EEN, edge_quota, S, seed, ne_e));
  const int64_t o_ee = nn.total, o_ne = o_ee + ee.total;
  const int64_t o_en = o_ne + ne_n.total, total = o_en + ne_e.total;
  HGX_TRY(alloc_records(ctx, total, K));
  HGX_TRY(emit(ctx, REC_NN, nn, 0, 0.f));
  HGX_TRY(emit(ctx, REC_EE, ee, o_ee, 0.f));
  HGX_TRY(emit(ctx, REC_NE_NODE, ne_n, o_ne, 0.f));
  HGX_TRY(emit(ctx, REC_NE_EDGE, ne_e, o_en, 0.f));
  HGX_TRY(neighbors(ctx, o_ne, ne_n.total, ne_n.rec_off, 0, seed, 0x500, 1));
  HGX_TRY(neighbors(ctx, o_en, ne_e.total, ne_e.rec_off, 3, seed, 0x501, 1));
  HGX_TRY(hgx_hobe_prepare(ctx));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 0, 0, o_ee));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 1, o_ee, o_ne));
  // the node rows' and the edge rows' node-edge pairs as two launches (the
  // same per-pair work; their times apart in a kernel trace)
  HGX_TRY(hgx_hobe_fill_probs(ctx, 2, o_ne, o_en));
  HGX_TRY(hgx_hobe_fill_probs(ctx, 2, o_en, total));
  set_blocks(ctx, {0, o_ee, o_ne, o_en, total});
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->smp_family = 1;
  ctx->smp_seed = seed;
  if (n_records) *n_records = total;
  return HGX_OK;
}

extern "C" int hgx_sample_hobe(hgx_ctx *ctx, uint64_t seed, int K, int S,
                               int64_t *n_records) {
  return hgx_sample_hobe_rows(ctx, seed, K, nullptr, nullptr, S, n_records);
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
  reset_stats(ctx);
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
  HGX_TRY(neighbors(ctx, o_ne, ne_n.total, ne_n.rec_off, 0, seed, 0x600, 1));
  HGX_TRY(neighbors(ctx, o_en, ne_e.total, ne_e.rec_off, 3, seed, 0x601, 1));
  set_blocks(ctx, {0, o_ee, o_ne, o_en, total});
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

extern "C" int hgx_sample_uniform_rows(hgx_ctx *ctx, int64_t *rows) {
  if (!ctx) return HGX_EINVAL;
  if (rows) *rows = ctx->sample_uniform_rows;
  return HGX_OK;
}
