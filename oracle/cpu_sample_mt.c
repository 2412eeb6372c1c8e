/*
 * cpu_sample_mt.c -- multi-threaded CPU HOBE sampler: the timed CPU baseline
 * of AlgebraicDistanceSamples (hg2v_sample.py:632-717) for bench.py.
 *
 * TEST / BENCH INFRASTRUCTURE ONLY (like hgref.c): bench.py's cpu_baseline
 * legs time it; the product never links it. It is not a parity checker --
 * the reference's own sampler (numpy MT19937, one process plus a Pool) is
 * restated bit-exactly in hgref.c -- but the same algorithm organised the
 * way a CPU framework would run it: OpenMP over rows, per row the exact
 * 2-hop (nn: A A^T, ee: A^T A) or 3-hop (ne: A A^T A, A^T A A^T) pattern row
 * expanded with a per-thread stamp array, min(q, |row|) distinct columns
 * drawn uniformly (partial Fisher-Yates, splitmix64 keyed by seed / block /
 * row), the HOBE probabilities of every pair (_same_type_dist_calc
 * :527-543 and DiffTypeDistanceSample :588-629: max over shared targets of
 * min(w_i, w_j), w = (sqrt(k) - |a - b|) / sqrt(k)) by sorted-list
 * intersection with galloping, and K neighbours per side for node-edge
 * records (:49-51). Records are written in the reference's layout
 * (SamplesToModelInput, :751-797) and kind-block order (nn, ee, ne node
 * rows, ne edge rows). Exact expansion is feasible on the random 100k/50k
 * graph (C3); power-law hub rows (C4) would need the device's rejection
 * sampler, so the bench times this on C3.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static inline uint32_t bounded(uint64_t r, uint32_t n) {
  return (uint32_t)(((unsigned __int128)r * n) >> 64);
}

static inline float dist_weight(const float *a, const float *b, int k) {
  double s = 0.0;
  for (int i = 0; i < k; i++) {
    const float d = a[i] - b[i];
    s += (double)(d * d);
  }
  const float sk = (float)sqrt((double)k);
  return (sk - sqrtf((float)s)) / sk;
}

static inline int32_t seek(const int32_t *col, int32_t lo, int32_t hi, int32_t v) {
  int32_t step = 1, b = lo;
  while (b < hi && col[b] < v) { lo = b + 1; b += step; step <<= 1; }
  if (b > hi) b = hi;
  while (lo < b) {
    int32_t m = lo + (b - lo) / 2;
    if (col[m] < v) lo = m + 1; else b = m;
  }
  return lo;
}

/* max over t in row_i & row_j of min(w_it, w_jt) */
static float pair_prob(const int32_t *rp, const int32_t *col, int32_t i,
                       int32_t j, const float *src, const float *tgt, int k) {
  int32_t a = rp[i], ae = rp[i + 1], b = rp[j], be = rp[j + 1];
  const int gallop = (ae - a) * 16 < (be - b) || (be - b) * 16 < (ae - a);
  float p = 0.0f;
  while (a < ae && b < be) {
    if (col[a] < col[b]) a = gallop ? seek(col, a, ae, col[b]) : a + 1;
    else if (col[a] > col[b]) b = gallop ? seek(col, b, be, col[a]) : b + 1;
    else {
      const int32_t t = col[a];
      const float wi = dist_weight(src + (int64_t)i * k, tgt + (int64_t)t * k, k);
      const float wj = dist_weight(src + (int64_t)j * k, tgt + (int64_t)t * k, k);
      const float m = wj < wi ? wj : wi;
      if (m > p) p = m;
      a++; b++;
    }
  }
  return p;
}

typedef struct {
  const int32_t *rp1, *c1, *rp2, *c2, *rp3, *c3;
  int levels, ncols;
} pattern;

/* distinct columns of the pattern row r into list (stamp: ncols ints) */
static int64_t expand(const pattern *P, int32_t r, int32_t *stamp, int32_t gen,
                      int32_t *list) {
  int64_t m = 0;
  for (int32_t a = P->rp1[r]; a < P->rp1[r + 1]; a++) {
    const int32_t x = P->c1[a];
    for (int32_t b = P->rp2[x]; b < P->rp2[x + 1]; b++) {
      const int32_t y = P->c2[b];
      if (P->levels == 2) {
        if (stamp[y] != gen) { stamp[y] = gen; list[m++] = y; }
      } else {
        for (int32_t c = P->rp3[y]; c < P->rp3[y + 1]; c++) {
          const int32_t z = P->c3[c];
          if (stamp[z] != gen) { stamp[z] = gen; list[m++] = z; }
        }
      }
    }
  }
  return m;
}

static int cmp_i32(const void *a, const void *b) {
  const int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  return (x > y) - (x < y);
}

/* One block: rows r with quota q[r] of pattern P. Row r's records go to
 * slots [cap_off[r], cap_off[r] + cnt[r]) of the block's capacity layout. */
static void sample_block(int blk, const pattern *P, int32_t nrows,
                         const int32_t *q, const int64_t *cap_off,
                         int32_t *cnt, int32_t *idx, float *tgt, int R, int K,
                         const int32_t *rp_n, const int32_t *col_n,
                         const int32_t *rp_e, const int32_t *col_e,
                         const float *an, const float *ae, int k,
                         uint64_t seed, int64_t list_cap) {
#pragma omp parallel
  {
    int32_t *stamp = (int32_t *)calloc((size_t)P->ncols, sizeof(int32_t));
    int32_t *list = (int32_t *)malloc(sizeof(int32_t) * (size_t)list_cap);
    int32_t gen = 0;
#pragma omp for schedule(dynamic, 16)
    for (int32_t r = 0; r < nrows; r++) {
      if (q[r] <= 0) { cnt[r] = 0; continue; }
      gen++;
      const int64_t m = expand(P, r, stamp, gen, list);
      const int64_t take = q[r] < m ? q[r] : m;
      const uint64_t key = mix64(seed ^ mix64(((uint64_t)blk << 32) | (uint32_t)r));
      for (int64_t j = 0; j < take; j++) {  /* partial Fisher-Yates */
        const int64_t t = j + bounded(mix64(key + (uint64_t)j), (uint32_t)(m - j));
        const int32_t s = list[j]; list[j] = list[t]; list[t] = s;
      }
      qsort(list, (size_t)take, sizeof(int32_t), cmp_i32);
      for (int64_t j = 0; j < take; j++) {
        const int64_t rec = cap_off[r] + j;
        int32_t *ri = idx + rec * R;
        float *tt = tgt + rec * 3;
        memset(ri, 0, sizeof(int32_t) * R);
        tt[0] = tt[1] = tt[2] = 0.0f;
        const int32_t c = list[j];
        if (blk == 0) {        /* nn: node rows of A A^T */
          ri[0] = r + 1; ri[2] = c + 1;
          tt[0] = pair_prob(rp_n, col_n, r, c, an, ae, k);
        } else if (blk == 1) { /* ee: edge rows of A^T A */
          ri[1] = r + 1; ri[3] = c + 1;
          tt[1] = pair_prob(rp_e, col_e, r, c, ae, an, k);
        } else {               /* ne: (node v, edge e) */
          const int32_t v = blk == 2 ? r : c, e = blk == 2 ? c : r;
          ri[0] = v + 1; ri[3] = e + 1;
          float p = 0.0f;
          for (int32_t t = rp_n[v]; t < rp_n[v + 1]; t++) {
            const float pe = pair_prob(rp_e, col_e, e, col_n[t], ae, an, k);
            if (pe > p) p = pe;
          }
          tt[2] = p;
          const int32_t nb = rp_e[e], nl = rp_e[e + 1] - nb;
          const int32_t eb = rp_n[v], el = rp_n[v + 1] - eb;
          for (int s = 0; s < K; s++) {
            ri[4 + s] = col_e[nb + bounded(mix64(key ^ (0x100000ull + j * 64 + s)), nl)] + 1;
            ri[4 + K + s] = col_n[eb + bounded(mix64(key ^ (0x200000ull + j * 64 + s)), el)] + 1;
          }
        }
      }
      cnt[r] = (int32_t)take;
    }
    free(stamp);
    free(list);
  }
}

/* HOBE records of the rows with a quota (node_q[N], edge_q[E]); idx/tgt
 * have capacity 2 * (sum node_q + sum edge_q) records. Returns the record
 * count (records compacted to the front, kind blocks in order; bounds[5]
 * receives the block starts) or -1 on allocation failure. threads <= 0:
 * OpenMP's default. */
int64_t cpu_hobe_sample_mt(int32_t N, int32_t E, const int32_t *rp_n,
                           const int32_t *col_n, const int32_t *rp_e,
                           const int32_t *col_e, const float *alg_node,
                           const float *alg_edge, int k, const int32_t *node_q,
                           const int32_t *edge_q, int K, uint64_t seed,
                           int threads, int32_t *idx, float *tgt,
                           int64_t *bounds) {
  if (threads > 0) omp_set_num_threads(threads);
  const int R = 4 + 2 * K;
  pattern P[4] = {
      {rp_n, col_n, rp_e, col_e, NULL, NULL, 2, N},     /* nn   A A^T   */
      {rp_e, col_e, rp_n, col_n, NULL, NULL, 2, E},     /* ee   A^T A   */
      {rp_n, col_n, rp_e, col_e, rp_n, col_n, 3, E},    /* ne   A A^T A */
      {rp_e, col_e, rp_n, col_n, rp_e, col_e, 3, N}};   /* ne   A^T A A^T */
  const int32_t nrows[4] = {N, E, N, E};
  const int32_t *q[4] = {node_q, edge_q, node_q, edge_q};
  int64_t base = 0, out = 0;
  for (int b = 0; b < 4; b++) {
    const int32_t n = nrows[b];
    int64_t *cap_off = (int64_t *)malloc(sizeof(int64_t) * ((size_t)n + 1));
    int32_t *cnt = (int32_t *)malloc(sizeof(int32_t) * ((size_t)n + 1));
    if (!cap_off || !cnt) { free(cap_off); free(cnt); return -1; }
    cap_off[0] = base;
    for (int32_t r = 0; r < n; r++) cap_off[r + 1] = cap_off[r] + q[b][r];
    /* a row's pattern list never exceeds the column count */
    sample_block(b, &P[b], n, q[b], cap_off, cnt, idx, tgt, R, K, rp_n, col_n,
                 rp_e, col_e, alg_node, alg_edge, k, seed, P[b].ncols);
    bounds[b] = out;
    for (int32_t r = 0; r < n; r++) {  /* compact in row order */
      if (cnt[r] && cap_off[r] != out) {
        memmove(idx + out * R, idx + cap_off[r] * R, sizeof(int32_t) * R * cnt[r]);
        memmove(tgt + out * 3, tgt + cap_off[r] * 3, sizeof(float) * 3 * cnt[r]);
      }
      out += cnt[r];
    }
    base = out;  /* the next block's capacity starts after this block */
    free(cap_off);
    free(cnt);
  }
  bounds[4] = out;
  return out;
}
