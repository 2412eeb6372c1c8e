/*
 * hgref.c -- CPU restatement of the reference FOBE/HOBE hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity ORACLE: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline. The product
 * (hypergraphembedding_amd + libhgx.so) never links or calls it.
 *
 * Every function restates the algorithm of the reference file:line it cites
 * (JSybrandt/HypergraphEmbedding, read-only at /root/reference). Parity
 * pinning: the RNG, CSR/SpGEMM ordering, alg-dist, FOBE/HOBE samplers and
 * SamplesToModelInput are checked BIT-EXACT against golden vectors produced by
 * importing the reference's own modules (tests/golden/make_golden.py). The
 * trainer (hgref_train) restates Keras-2.x Adagrad semantics; keras/tensorflow
 * are absent from the image, so the trainer is "parity unpinned".
 *
 * Compile with -ffp-contract=off: the restatement must round exactly like
 * numpy (no fused multiply-adds).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* numpy legacy RandomState (MT19937) -- numpy/random/_mt19937.pyx,           */
/* distributions.c. Used by the reference via np.random.* (global state).    */
/* ------------------------------------------------------------------------- */
#define MT_N 624
#define MT_M 397
typedef struct {
  uint32_t mt[MT_N];
  int pos;
} hgref_rng;

hgref_rng *hgref_rng_create(uint32_t seed) {
  hgref_rng *s = (hgref_rng *)malloc(sizeof(hgref_rng));
  s->mt[0] = seed;
  for (int i = 1; i < MT_N; i++)
    s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
  s->pos = MT_N;
  return s;
}
void hgref_rng_destroy(hgref_rng *s) { free(s); }
void hgref_rng_copy(hgref_rng *dst, const hgref_rng *src) { *dst = *src; }
int hgref_rng_sizeof(void) { return (int)sizeof(hgref_rng); }

static void mt_twist(hgref_rng *s) {
  static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
  int i;
  uint32_t y;
  for (i = 0; i < MT_N - MT_M; i++) {
    y = (s->mt[i] & 0x80000000u) | (s->mt[i + 1] & 0x7fffffffu);
    s->mt[i] = s->mt[i + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
  }
  for (; i < MT_N - 1; i++) {
    y = (s->mt[i] & 0x80000000u) | (s->mt[i + 1] & 0x7fffffffu);
    s->mt[i] = s->mt[i + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
  }
  y = (s->mt[MT_N - 1] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
  s->mt[MT_N - 1] = s->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
  s->pos = 0;
}

uint32_t hgref_rng_next32(hgref_rng *s) {
  if (s->pos == MT_N) mt_twist(s);
  uint32_t y = s->mt[s->pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

static uint64_t next64(hgref_rng *s) {
  uint64_t hi = hgref_rng_next32(s);
  return (hi << 32) | hgref_rng_next32(s);
}

/* np.random.random(): ((a>>5)*2^26 + (b>>6)) / 2^53 */
double hgref_rng_double(hgref_rng *s) {
  int32_t a = (int32_t)(hgref_rng_next32(s) >> 5);
  int32_t b = (int32_t)(hgref_rng_next32(s) >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

void hgref_rng_random(hgref_rng *s, int64_t n, double *out) {
  for (int64_t i = 0; i < n; i++) out[i] = hgref_rng_double(s);
}

static uint64_t gen_mask(uint64_t max) {
  uint64_t m = max;
  m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16; m |= m >> 32;
  return m;
}

/* random_interval(max): used by legacy shuffle/permutation. */
static uint64_t rng_interval(hgref_rng *s, uint64_t max) {
  if (max == 0) return 0;
  uint64_t mask = gen_mask(max), v;
  if (max <= 0xffffffffull) {
    while ((v = (hgref_rng_next32(s) & mask)) > max) {}
  } else {
    while ((v = (next64(s) & mask)) > max) {}
  }
  return v;
}

/* legacy randint(0, n): random_bounded_uint64_fill(off=0, rng=n-1, masked). */
static int64_t rng_randint(hgref_rng *s, int64_t n) {
  uint64_t rng = (uint64_t)(n - 1);
  if (rng == 0) return 0;
  if (rng <= 0xffffffffull) {
    if (rng == 0xffffffffull) return (int64_t)hgref_rng_next32(s);
    uint32_t mask = (uint32_t)gen_mask(rng), v;
    while ((v = (hgref_rng_next32(s) & mask)) > rng) {}
    return (int64_t)v;
  }
  uint64_t mask = gen_mask(rng), v;
  while ((v = (next64(s) & mask)) > rng) {}
  return (int64_t)v;
}

int64_t hgref_rng_randint(hgref_rng *s, int64_t n) { return rng_randint(s, n); }

/* legacy permutation(n) = arange + shuffle: reversed Fisher-Yates, i=n-1..1 */
void hgref_rng_permutation(hgref_rng *s, int64_t n, int64_t *out) {
  for (int64_t i = 0; i < n; i++) out[i] = i;
  for (int64_t i = n - 1; i >= 1; i--) {
    int64_t j = (int64_t)rng_interval(s, (uint64_t)i);
    int64_t t = out[j]; out[j] = out[i]; out[i] = t;
  }
}

/* ------------------------------------------------------------------------- */
/* Sparse pattern products in scipy's SMMP column order.                     */
/* scipy csr_matmat emits each row's columns in REVERSE first-discovery order */
/* (linked list, head insertion). The reference samples from rows of these  */
/* products (hg2v_sample.py:154,167,659,679,698,703) via .nonzero()[1], so   */
/* the column order decides which element np.random.choice picks.           */
/* ------------------------------------------------------------------------- */
typedef struct {
  int64_t nrow;
  int64_t *p;  /* nrow+1 */
  int32_t *j;  /* p[nrow] */
} pat;

static void pat_free(pat *c) { free(c->p); free(c->j); c->p = NULL; c->j = NULL; }

static pat spgemm_pattern(int64_t nrow, const int64_t *Ap, const int32_t *Aj,
                          int64_t ncolB, const int64_t *Bp, const int32_t *Bj) {
  pat C;
  C.nrow = nrow;
  C.p = (int64_t *)malloc(sizeof(int64_t) * (nrow + 1));
  int64_t *next = (int64_t *)malloc(sizeof(int64_t) * (ncolB > 0 ? ncolB : 1));
  for (int64_t k = 0; k < ncolB; k++) next[k] = -1;
  int64_t cap = 1024, nnz = 0;
  C.j = (int32_t *)malloc(sizeof(int32_t) * cap);
  C.p[0] = 0;
  for (int64_t i = 0; i < nrow; i++) {
    int64_t head = -2, len = 0;
    for (int64_t jj = Ap[i]; jj < Ap[i + 1]; jj++) {
      int32_t j = Aj[jj];
      for (int64_t kk = Bp[j]; kk < Bp[j + 1]; kk++) {
        int32_t k = Bj[kk];
        if (next[k] == -1) { next[k] = head; head = k; len++; }
      }
    }
    if (nnz + len > cap) {
      while (nnz + len > cap) cap *= 2;
      C.j = (int32_t *)realloc(C.j, sizeof(int32_t) * cap);
    }
    for (int64_t t = 0; t < len; t++) {
      C.j[nnz++] = (int32_t)head;
      int64_t tmp = head; head = next[head]; next[tmp] = -1;
    }
    C.p[i + 1] = nnz;
  }
  free(next);
  return C;
}

static pat pat_view(int64_t nrow, const int32_t *rp32, const int32_t *col) {
  pat P;
  P.nrow = nrow;
  P.p = (int64_t *)malloc(sizeof(int64_t) * (nrow + 1));
  for (int64_t i = 0; i <= nrow; i++) P.p[i] = rp32[i];
  int64_t nnz = P.p[nrow];
  P.j = (int32_t *)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  memcpy(P.j, col, sizeof(int32_t) * nnz);
  return P;
}

/* Exposed for tests: row pointer + columns of A*B in SMMP order. Call with
 * cols=NULL to get nnz. */
int64_t hgref_spgemm(int64_t nrowA, const int32_t *Ap, const int32_t *Aj,
                     int64_t nrowB, int64_t ncolB, const int32_t *Bp,
                     const int32_t *Bj, int64_t *out_p, int32_t *out_j) {
  pat A = pat_view(nrowA, Ap, Aj), B = pat_view(nrowB, Bp, Bj);
  pat C = spgemm_pattern(nrowA, A.p, A.j, ncolB, B.p, B.j);
  int64_t nnz = C.p[nrowA];
  if (out_p) memcpy(out_p, C.p, sizeof(int64_t) * (nrowA + 1));
  if (out_j) memcpy(out_j, C.j, sizeof(int32_t) * nnz);
  pat_free(&A); pat_free(&B); pat_free(&C);
  return nnz;
}

/* ------------------------------------------------------------------------- */
/* Algebraic distance -- algebraic_distance.py:34-51 (_update_alg_dist),      */
/* 54-91 (node half then edge half using NEW node coords), 97-123 (joint     */
/* per-dim min-max rescale), 126-175 (driver). float64, same op order as the */
/* reference: b = (sum_e y_e*(1/|e|)) / (sum_e 1/|e|) accumulated in CSR     */
/* column order (sorted), then (a+b)/2, then (x-min)/(max-min).              */
/* Returns 0, or -1 for an isolated row (the reference raises                */
/* ZeroDivisionError at algebraic_distance.py:49).                            */
/* ------------------------------------------------------------------------- */
static int algdist_half(int64_t R, int k, const int32_t *rp, const int32_t *col,
                        const int32_t *rp_src, const double *self_in,
                        const double *src, double *out) {
  /* rows are independent and each row sums in CSR order, so the OpenMP
   * split changes nothing in the result (checker speed at C4 only) */
  int bad = 0;
#pragma omp parallel
  {
    double *acc = (double *)malloc(sizeof(double) * k);
#pragma omp for schedule(dynamic, 4096) reduction(|: bad)
    for (int64_t a = 0; a < R; a++) {
      if (rp[a + 1] == rp[a]) { bad = 1; continue; }
      for (int d = 0; d < k; d++) acc[d] = 0.0;
      double wsum = 0.0;
      for (int32_t t = rp[a]; t < rp[a + 1]; t++) {
        int32_t b = col[t];
        double w = 1.0 / (double)(rp_src[b + 1] - rp_src[b]);
        for (int d = 0; d < k; d++) acc[d] = acc[d] + src[(int64_t)b * k + d] * w;
        wsum = wsum + w;
      }
      for (int d = 0; d < k; d++) {
        double bd = acc[d] / wsum;
        out[a * k + d] = (self_in[a * k + d] + bd) / 2.0;
      }
    }
    free(acc);
  }
  return bad ? -1 : 0;
}

int hgref_algdist(int64_t N, int64_t E, int k, int iters, const int32_t *rp_n,
                  const int32_t *col_n, const int32_t *rp_e,
                  const int32_t *col_e, double *x, double *y) {
  double *xn = (double *)malloc(sizeof(double) * N * k);
  double *yn = (double *)malloc(sizeof(double) * E * k);
  double *mn = (double *)malloc(sizeof(double) * k);
  double *mx = (double *)malloc(sizeof(double) * k);
  int rc = 0;
  for (int it = 0; it < iters && rc == 0; it++) {
    rc = algdist_half(N, k, rp_n, col_n, rp_e, x, y, xn);
    if (rc) break;
    rc = algdist_half(E, k, rp_e, col_e, rp_n, y, xn, yn);
    if (rc) break;
    /* np.min(axis=0) of edges / nodes, then the min of the two (exact). */
    for (int d = 0; d < k; d++) { mn[d] = INFINITY; mx[d] = -INFINITY; }
    for (int64_t i = 0; i < N; i++)
      for (int d = 0; d < k; d++) {
        double v = xn[i * k + d];
        if (v < mn[d]) mn[d] = v;
        if (v > mx[d]) mx[d] = v;
      }
    for (int64_t i = 0; i < E; i++)
      for (int d = 0; d < k; d++) {
        double v = yn[i * k + d];
        if (v < mn[d]) mn[d] = v;
        if (v > mx[d]) mx[d] = v;
      }
    for (int64_t i = 0; i < N; i++)
      for (int d = 0; d < k; d++) {
        double v = xn[i * k + d] - mn[d];
        x[i * k + d] = v / (mx[d] - mn[d]);
      }
    for (int64_t i = 0; i < E; i++)
      for (int d = 0; d < k; d++) {
        double v = yn[i * k + d] - mn[d];
        y[i * k + d] = v / (mx[d] - mn[d]);
      }
  }
  free(xn); free(yn); free(mn); free(mx);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* Record layout = SamplesToModelInput(records, K, weighted=False)           */
/* (hg2v_sample.py:751-797): int32 [ln, le, rn, re, nn_0..K-1, ne_0..K-1],   */
/* each id +1 and 0 when absent/padded; float32 [nn_prob, ee_prob, ne_prob], */
/* unset -> 0. Records are emitted in the reference's generation order.      */
/* ------------------------------------------------------------------------- */
typedef struct {
  int K;
  int64_t n, cap;
  int32_t *idx;
  float *tgt;
} recbuf;

static int32_t *rec_slot(recbuf *rb) {
  if (rb->n >= rb->cap) return NULL;
  int R = 4 + 2 * rb->K;
  int32_t *r = rb->idx + rb->n * R;
  for (int i = 0; i < R; i++) r[i] = 0;
  float *t = rb->tgt + rb->n * 3;
  t[0] = t[1] = t[2] = 0.0f;
  return r;
}

/* _sample_adj_matrix (hg2v_sample.py:53-86), one row. Appends chosen column
 * ids to out (capacity >= max(q, rowlen)). Returns the count. */
static int64_t sample_row(hgref_rng *s, const int32_t *cols, int64_t len,
                          int64_t q, int negative, int64_t ncols, int32_t *out,
                          int64_t *perm_scratch) {
  if (negative) {
    for (int64_t t = 0; t < q; t++) out[t] = (int32_t)rng_randint(s, ncols);
    return q;
  }
  if (len == 0) return 0;
  int64_t m = q < len ? q : len;
  /* np.random.choice(cols, m, replace=False) = cols[permutation(len)[:m]] */
  hgref_rng_permutation(s, len, perm_scratch);
  for (int64_t t = 0; t < m; t++) out[t] = cols[perm_scratch[t]];
  return m;
}

/* _sample_neighbors (hg2v_sample.py:49-51): K draws with replacement. */
static void sample_neighbors(hgref_rng *s, const int32_t *cols, int64_t len,
                             int K, int32_t *out_plus1) {
  /* np.random.choice(cols, K, replace=True) = cols[randint(0, len, K)].
   * len==0 raises in numpy; rows reached here always have len>0. */
  for (int t = 0; t < K; t++)
    out_plus1[t] = cols[rng_randint(s, len)] + 1;
}

/* Pair list (row, col) for every row of pattern P with quota q[row]. */
typedef struct {
  int64_t n, cap;
  int32_t *a, *b;
} pairs;

static void pairs_push(pairs *P, int32_t a, int32_t b) {
  if (P->n == P->cap) {
    P->cap = P->cap ? P->cap * 2 : 4096;
    P->a = (int32_t *)realloc(P->a, sizeof(int32_t) * P->cap);
    P->b = (int32_t *)realloc(P->b, sizeof(int32_t) * P->cap);
  }
  P->a[P->n] = a; P->b[P->n] = b; P->n++;
}

static void sample_pattern(hgref_rng *s, const pat *P, int64_t ncols,
                           const int32_t *quota, int32_t quota_all, int negative,
                           pairs *out, int swap) {
  int64_t maxlen = 1;
  for (int64_t r = 0; r < P->nrow; r++) {
    int64_t l = P->p[r + 1] - P->p[r];
    int64_t q = quota ? quota[r] : quota_all;
    if (l > maxlen) maxlen = l;
    if (q > maxlen) maxlen = q;
  }
  int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * maxlen);
  int64_t *perm = (int64_t *)malloc(sizeof(int64_t) * maxlen);
  for (int64_t r = 0; r < P->nrow; r++) {
    int64_t q = quota ? quota[r] : quota_all;
    int64_t m = sample_row(s, P->j + P->p[r], P->p[r + 1] - P->p[r], q,
                           negative, ncols, buf, perm);
    for (int64_t t = 0; t < m; t++) {
      if (swap) pairs_push(out, buf[t], (int32_t)r);
      else pairs_push(out, (int32_t)r, buf[t]);
    }
  }
  free(buf); free(perm);
}

/* ------------------------------------------------------------------------- */
/* FOBE: BooleanSamples (hg2v_sample.py:125-242).                             */
/* Quotas are int(weight*num_samples) computed by the caller (:138-146).     */
/* ------------------------------------------------------------------------- */
int64_t hgref_fobe_sample(hgref_rng *s, int64_t N, int64_t E,
                          const int32_t *rp_n, const int32_t *col_n,
                          const int32_t *rp_e, const int32_t *col_e,
                          const int32_t *node_q, const int32_t *edge_q,
                          const int32_t *neg_node_q, const int32_t *neg_edge_q,
                          int K, int64_t cap, int32_t *idx, float *tgt) {
  recbuf rb = {K, 0, cap, idx, tgt};
  int R = 4 + 2 * K;
  pat A = pat_view(N, rp_n, col_n), AT = pat_view(E, rp_e, col_e);
  pat NN = spgemm_pattern(N, A.p, A.j, N, AT.p, AT.j);   /* :154 */
  pat EE = spgemm_pattern(E, AT.p, AT.j, E, A.p, A.j);   /* :167 */
  pairs P = {0, 0, NULL, NULL};
  int64_t overflow = 0;

  sample_pattern(s, &NN, N, node_q, 0, 0, &P, 0);        /* :157 */
  for (int64_t t = 0; t < P.n; t++) {
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    r[0] = P.a[t] + 1; r[2] = P.b[t] + 1; rb.tgt[rb.n * 3 + 0] = 1.0f; rb.n++;
  }
  P.n = 0;
  sample_pattern(s, &EE, E, edge_q, 0, 0, &P, 0);        /* :170 */
  for (int64_t t = 0; t < P.n; t++) {
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    r[1] = P.a[t] + 1; r[3] = P.b[t] + 1; rb.tgt[rb.n * 3 + 1] = 1.0f; rb.n++;
  }
  P.n = 0;
  sample_pattern(s, &A, E, node_q, 0, 0, &P, 0);         /* :178 */
  sample_pattern(s, &AT, N, edge_q, 0, 0, &P, 1);        /* :181 swapped */
  for (int64_t t = 0; t < P.n; t++) {                    /* :183-194 */
    int32_t v = P.a[t], e = P.b[t];
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    r[0] = v + 1; r[3] = e + 1;
    sample_neighbors(s, A.j + A.p[v], A.p[v + 1] - A.p[v], K, r + 4 + K);
    sample_neighbors(s, AT.j + AT.p[e], AT.p[e + 1] - AT.p[e], K, r + 4);
    rb.tgt[rb.n * 3 + 2] = 1.0f;
    rb.n++;
  }
  if (neg_node_q && neg_edge_q) {                        /* :198-240 */
    P.n = 0;
    sample_pattern(s, &NN, N, neg_node_q, 0, 1, &P, 0);
    for (int64_t t = 0; t < P.n; t++) {
      int32_t *r = rec_slot(&rb);
      if (!r) { overflow = 1; break; }
      r[0] = P.a[t] + 1; r[2] = P.b[t] + 1; rb.n++;
    }
    for (int rep = 0; rep < 2; rep++) {  /* edge-edge, and the :215-221 copy */
      P.n = 0;
      sample_pattern(s, &EE, E, neg_edge_q, 0, 1, &P, 0);
      for (int64_t t = 0; t < P.n; t++) {
        int32_t *r = rec_slot(&rb);
        if (!r) { overflow = 1; break; }
        r[1] = P.a[t] + 1; r[3] = P.b[t] + 1; rb.n++;
      }
    }
    P.n = 0;
    sample_pattern(s, &A, E, neg_node_q, 0, 1, &P, 0);
    sample_pattern(s, &AT, N, neg_edge_q, 0, 1, &P, 1);
    for (int64_t t = 0; t < P.n; t++) {
      int32_t v = P.a[t], e = P.b[t];
      int32_t *r = rec_slot(&rb);
      if (!r) { overflow = 1; break; }
      r[0] = v + 1; r[3] = e + 1;
      sample_neighbors(s, A.j + A.p[v], A.p[v + 1] - A.p[v], K, r + 4 + K);
      sample_neighbors(s, AT.j + AT.p[e], AT.p[e + 1] - AT.p[e], K, r + 4);
      rb.n++;
    }
  }
  (void)R;
  free(P.a); free(P.b);
  pat_free(&A); pat_free(&AT); pat_free(&NN); pat_free(&EE);
  return overflow ? -1 : rb.n;
}

/* ------------------------------------------------------------------------- */
/* HOBE probabilities.                                                        */
/* _same_type_dist_calc (hg2v_sample.py:527-543): for pair (i,j) over the    */
/* shared targets t: w = (sqrt(k) - ||a_i - a_t||_2)/sqrt(k) in float32,      */
/* prob = max_t min(w_it, w_jt), 0 when nothing is shared. numpy's norm of a */
/* float32 vector with k<32 is OpenBLAS sdot's tail loop: float products     */
/* accumulated in a double, then cast to float; sqrt in float32.             */
/* ------------------------------------------------------------------------- */
static float dist_weight(const float *a, const float *b, int k) {
  double acc = 0.0;
  for (int d = 0; d < k; d++) {
    float df = a[d] - b[d];
    float pr = df * df;
    acc += (double)pr;
  }
  float nrm = sqrtf((float)acc);
  float md = (float)sqrt((double)k);
  return (md - nrm) / md;
}

float hgref_dist_weight(const float *a, const float *b, int k) {
  return dist_weight(a, b, k);
}

/* first position in [lo, hi) of col with col[pos] >= v (galloping then
 * binary search) */
static int32_t seek(const int32_t *col, int32_t lo, int32_t hi, int32_t v) {
  int32_t step = 1, b = lo;
  while (b < hi && col[b] < v) { lo = b + 1; b += step; step <<= 1; }
  if (b > hi) b = hi;
  while (lo < b) {
    int32_t m = lo + (b - lo) / 2;
    if (col[m] < v) lo = m + 1; else b = m;
  }
  return lo;
}

/* sorted-list intersection of rows i and j of P; src/tgt coords. The
 * reference takes the max over the shared targets of min(w_it, w_jt)
 * (hg2v_sample.py:527-543); max and min are exact, so visiting the shared
 * targets by merge or by galloping from the shorter row gives the same
 * float. Galloping keeps the checker usable on power-law hub rows. */
static float same_type_prob(const int32_t *rp, const int32_t *col, int32_t i,
                            int32_t j, const float *src, const float *tgt,
                            int k) {
  int32_t a = rp[i], ae = rp[i + 1], b = rp[j], be = rp[j + 1];
  float prob = 0.0f;  /* prob = 0; prob = max(prob, min(w_ik, w_jk)) */
  const int gallop = (ae - a) * 16 < (be - b) || (be - b) * 16 < (ae - a);
  while (a < ae && b < be) {
    if (col[a] < col[b]) a = gallop ? seek(col, a, ae, col[b]) : a + 1;
    else if (col[a] > col[b]) b = gallop ? seek(col, b, be, col[a]) : b + 1;
    else {
      int32_t t = col[a];
      float wi = dist_weight(src + (int64_t)i * k, tgt + (int64_t)t * k, k);
      float wj = dist_weight(src + (int64_t)j * k, tgt + (int64_t)t * k, k);
      float m = wj < wi ? wj : wi;
      if (m > prob) prob = m;
      a++; b++;
    }
  }
  return prob;
}

/* kind 0: node-node over A (rp_n/col_n), 1: edge-edge over A^T,
 * 2: node-edge (DiffTypeDistanceSample, hg2v_sample.py:588-629):
 *    max over e' in E(v) of edge-edge prob(e, e'). */
void hgref_hobe_probs(int kind, int64_t n, const int32_t *pa, const int32_t *pb,
                      const int32_t *rp_n, const int32_t *col_n,
                      const int32_t *rp_e, const int32_t *col_e,
                      const float *alg_node, const float *alg_edge, int k,
                      float *out) {
  /* pairs are independent: OpenMP only for checker speed at C4 */
#pragma omp parallel for schedule(dynamic, 16) if (n > 64)
  for (int64_t t = 0; t < n; t++) {
    float p = 0.0f;
    if (kind == 0) {
      p = same_type_prob(rp_n, col_n, pa[t], pb[t], alg_node, alg_edge, k);
    } else if (kind == 1) {
      p = same_type_prob(rp_e, col_e, pa[t], pb[t], alg_edge, alg_node, k);
    } else {
      int32_t v = pa[t], e = pb[t];
      for (int32_t q = rp_n[v]; q < rp_n[v + 1]; q++) {
        float pe = same_type_prob(rp_e, col_e, e, col_n[q], alg_edge, alg_node, k);
        if (pe > p) p = pe;
      }
    }
    out[t] = p;
  }
}

/* ------------------------------------------------------------------------- */
/* HOBE: AlgebraicDistanceSamples (hg2v_sample.py:632-717),                   */
/* run_in_parallel=False semantics: pair draws in the parent; the ne         */
/* neighbour draws happen in the single forked Pool worker, i.e. they        */
/* continue from a COPY of the parent RNG state after the last pair draw,    */
/* in record order (:604-605); the parent state is not advanced by them.     */
/* ------------------------------------------------------------------------- */
int64_t hgref_hobe_sample(hgref_rng *s, int64_t N, int64_t E,
                          const int32_t *rp_n, const int32_t *col_n,
                          const int32_t *rp_e, const int32_t *col_e,
                          const float *alg_node, const float *alg_edge, int k,
                          int S, int K, int64_t cap, int32_t *idx, float *tgt) {
  recbuf rb = {K, 0, cap, idx, tgt};
  pat A = pat_view(N, rp_n, col_n), AT = pat_view(E, rp_e, col_e);
  pairs P = {0, 0, NULL, NULL};
  int64_t overflow = 0;
  float pr;

  pat NN = spgemm_pattern(N, A.p, A.j, N, AT.p, AT.j);           /* :659 */
  sample_pattern(s, &NN, N, NULL, S, 0, &P, 0);
  pat_free(&NN);
  for (int64_t t = 0; t < P.n; t++) {
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    hgref_hobe_probs(0, 1, P.a + t, P.b + t, rp_n, col_n, rp_e, col_e,
                     alg_node, alg_edge, k, &pr);
    r[0] = P.a[t] + 1; r[2] = P.b[t] + 1; rb.tgt[rb.n * 3 + 0] = pr; rb.n++;
  }
  P.n = 0;
  pat EE = spgemm_pattern(E, AT.p, AT.j, E, A.p, A.j);           /* :679 */
  sample_pattern(s, &EE, E, NULL, S, 0, &P, 0);
  pat_free(&EE);
  for (int64_t t = 0; t < P.n; t++) {
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    hgref_hobe_probs(1, 1, P.a + t, P.b + t, rp_n, col_n, rp_e, col_e,
                     alg_node, alg_edge, k, &pr);
    r[1] = P.a[t] + 1; r[3] = P.b[t] + 1; rb.tgt[rb.n * 3 + 1] = pr; rb.n++;
  }
  P.n = 0;
  pat NN2 = spgemm_pattern(N, A.p, A.j, N, AT.p, AT.j);
  pat NNE = spgemm_pattern(N, NN2.p, NN2.j, E, A.p, A.j);        /* :698 */
  pat_free(&NN2);
  sample_pattern(s, &NNE, E, NULL, S, 0, &P, 0);
  pat_free(&NNE);
  pat EE2 = spgemm_pattern(E, AT.p, AT.j, E, A.p, A.j);
  pat EEN = spgemm_pattern(E, EE2.p, EE2.j, N, AT.p, AT.j);      /* :703 */
  pat_free(&EE2);
  sample_pattern(s, &EEN, N, NULL, S, 0, &P, 1);
  pat_free(&EEN);
  hgref_rng w;  /* forked worker's copy */
  hgref_rng_copy(&w, s);
  for (int64_t t = 0; t < P.n; t++) {
    int32_t v = P.a[t], e = P.b[t];
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    r[0] = v + 1; r[3] = e + 1;
    sample_neighbors(&w, A.j + A.p[v], A.p[v + 1] - A.p[v], K, r + 4 + K);
    sample_neighbors(&w, AT.j + AT.p[e], AT.p[e + 1] - AT.p[e], K, r + 4);
    hgref_hobe_probs(2, 1, &v, &e, rp_n, col_n, rp_e, col_e, alg_node,
                     alg_edge, k, &pr);
    rb.tgt[rb.n * 3 + 2] = pr;
    rb.n++;
  }
  free(P.a); free(P.b);
  pat_free(&A); pat_free(&AT);
  return overflow ? -1 : rb.n;
}

/* ------------------------------------------------------------------------- */
/* Weighted-Jaccard samples (HG2V_ADJ_JAC / HG2V_NEIGH_JAC),                 */
/* WeightedJaccardSamples (hg2v_sample.py:395-510), run_in_parallel=False.   */
/* Features are per-incidence values on A's pattern: fn[] in node-major     */
/* (A) order (node2features, N x E), fe[] in edge-major (A^T) order          */
/* (edge2features, E x N), as UniformWeight / WeightByNeighborhood build.    */
/* ------------------------------------------------------------------------- */

/* SparseWeightedJaccard (hg2v_sample.py:250-273): over the sorted union of
 * both supports, num += min, den += max (the `x < y` branch), float32
 * sequential (0 + np.float32 -> float32); 0 if den == 0. */
static float swj(const int32_t *ac, const float *av, int64_t na,
                 const int32_t *bc, const float *bv, int64_t nb) {
  float num = 0.0f, den = 0.0f;
  int64_t i = 0, j = 0;
  while (i < na || j < nb) {
    float x, y;
    if (j >= nb || (i < na && ac[i] < bc[j])) { x = av[i++]; y = 0.0f; }
    else if (i >= na || bc[j] < ac[i]) { x = 0.0f; y = bv[j++]; }
    else { x = av[i++]; y = bv[j++]; }
    if (x < y) { num += x; den += y; }
    else { num += y; den += x; }
  }
  if (den == 0.0f) return 0.0f;
  return num / den;
}

/* GetAllCentroids / CentroidFromRows (hg2v_sample.py:276-326): row r =
 * (sum over t in row r of idx2targets, ascending, of targets2features row
 * t) / len(row r), float32 (scipy's ones @ sub-matrix adds rows in order),
 * stored as CSR with sorted columns, zeros dropped (.nonzero()). */
typedef struct {
  int64_t *p;
  int32_t *j;
  float *v;
} fcsr;

static fcsr centroids(int64_t R, const int32_t *rp, const int32_t *col,
                      int64_t ncols, const int32_t *frp, const int32_t *fcol,
                      const float *fval) {
  fcsr C;
  float *acc = (float *)calloc(ncols > 0 ? ncols : 1, sizeof(float));
  char *seen = (char *)calloc(ncols > 0 ? ncols : 1, 1);
  int32_t *touched = (int32_t *)malloc(sizeof(int32_t) * (ncols > 0 ? ncols : 1));
  int64_t cap = 1024, nnz = 0;
  C.p = (int64_t *)malloc(sizeof(int64_t) * (R + 1));
  C.j = (int32_t *)malloc(sizeof(int32_t) * cap);
  C.v = (float *)malloc(sizeof(float) * cap);
  C.p[0] = 0;
  for (int64_t r = 0; r < R; r++) {
    int64_t nt = 0;
    const int32_t len = rp[r + 1] - rp[r];
    for (int32_t q = rp[r]; q < rp[r + 1]; q++) {
      const int32_t t = col[q];
      for (int32_t z = frp[t]; z < frp[t + 1]; z++) {
        const int32_t c = fcol[z];
        if (!seen[c]) { seen[c] = 1; touched[nt++] = c; }
        acc[c] = acc[c] + fval[z];
      }
    }
    /* sorted column order */
    for (int64_t a = 1; a < nt; a++) {
      int32_t x = touched[a];
      int64_t b = a - 1;
      while (b >= 0 && touched[b] > x) { touched[b + 1] = touched[b]; b--; }
      touched[b + 1] = x;
    }
    if (nnz + nt > cap) {
      while (nnz + nt > cap) cap *= 2;
      C.j = (int32_t *)realloc(C.j, sizeof(int32_t) * cap);
      C.v = (float *)realloc(C.v, sizeof(float) * cap);
    }
    for (int64_t a = 0; a < nt; a++) {
      const int32_t c = touched[a];
      const float val = acc[c] / (float)len;
      if (val != 0.0f) { C.j[nnz] = c; C.v[nnz] = val; nnz++; }
      acc[c] = 0.0f;
      seen[c] = 0;
    }
    C.p[r + 1] = nnz;
  }
  free(acc); free(seen); free(touched);
  return C;
}

static void fcsr_free(fcsr *C) { free(C->p); free(C->j); free(C->v); }

/* Exposed for tests: centroid CSR of rows R of (rp, col) over the features
 * (frp, fcol, fval). Call with out_j == NULL for nnz (out_p filled). */
int64_t hgref_centroids(int64_t R, const int32_t *rp, const int32_t *col,
                        int64_t ncols, const int32_t *frp, const int32_t *fcol,
                        const float *fval, int64_t *out_p, int32_t *out_j,
                        float *out_v) {
  fcsr C = centroids(R, rp, col, ncols, frp, fcol, fval);
  const int64_t nnz = C.p[R];
  if (out_p) memcpy(out_p, C.p, sizeof(int64_t) * (R + 1));
  if (out_j) memcpy(out_j, C.j, sizeof(int32_t) * nnz);
  if (out_v) memcpy(out_v, C.v, sizeof(float) * nnz);
  fcsr_free(&C);
  return nnz;
}

/* kind 0 nn, 1 ee, 2 ne; cn = node2edge_centroid (N rows over nodes),
 * ce = edge2node_centroid (E rows over edges). */
static float jac_prob(int kind, int32_t a, int32_t b, const int32_t *rp_n,
                      const int32_t *col_n, const float *fn,
                      const int32_t *rp_e, const int32_t *col_e,
                      const float *fe, const fcsr *cn, const fcsr *ce) {
  if (kind == 0)  /* SameTypeJaccardSample over node2features */
    return swj(col_n + rp_n[a], fn + rp_n[a], rp_n[a + 1] - rp_n[a],
               col_n + rp_n[b], fn + rp_n[b], rp_n[b + 1] - rp_n[b]);
  if (kind == 1)
    return swj(col_e + rp_e[a], fe + rp_e[a], rp_e[a + 1] - rp_e[a],
               col_e + rp_e[b], fe + rp_e[b], rp_e[b + 1] - rp_e[b]);
  /* DiffTypeJaccardSample (:343-392): v = a, e = b */
  const float pn = swj(col_n + rp_n[a], fn + rp_n[a], rp_n[a + 1] - rp_n[a],
                       ce->j + ce->p[b], ce->v + ce->p[b], ce->p[b + 1] - ce->p[b]);
  const float pe = swj(col_e + rp_e[b], fe + rp_e[b], rp_e[b + 1] - rp_e[b],
                       cn->j + cn->p[a], cn->v + cn->p[a], cn->p[a + 1] - cn->p[a]);
  return pn * pe;
}

int64_t hgref_jaccard_sample(hgref_rng *s, int64_t N, int64_t E,
                             const int32_t *rp_n, const int32_t *col_n,
                             const int32_t *rp_e, const int32_t *col_e,
                             const float *fn, const float *fe,
                             const int32_t *node_q, const int32_t *edge_q,
                             int K, int64_t cap, int32_t *idx, float *tgt) {
  recbuf rb = {K, 0, cap, idx, tgt};
  pat A = pat_view(N, rp_n, col_n), AT = pat_view(E, rp_e, col_e);
  pairs P = {0, 0, NULL, NULL};
  int64_t overflow = 0;
  pat NN = spgemm_pattern(N, A.p, A.j, N, AT.p, AT.j);           /* :436 */
  sample_pattern(s, &NN, N, node_q, 0, 0, &P, 0);                /* :439 */
  for (int64_t t = 0; t < P.n; t++) {
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    r[0] = P.a[t] + 1; r[2] = P.b[t] + 1;
    rb.tgt[rb.n * 3 + 0] = jac_prob(0, P.a[t], P.b[t], rp_n, col_n, fn, rp_e,
                                    col_e, fe, NULL, NULL);
    rb.n++;
  }
  P.n = 0;
  pat EE = spgemm_pattern(E, AT.p, AT.j, E, A.p, A.j);           /* :461 */
  sample_pattern(s, &EE, E, edge_q, 0, 0, &P, 0);                /* :464 */
  for (int64_t t = 0; t < P.n; t++) {
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    r[1] = P.a[t] + 1; r[3] = P.b[t] + 1;
    rb.tgt[rb.n * 3 + 1] = jac_prob(1, P.a[t], P.b[t], rp_n, col_n, fn, rp_e,
                                    col_e, fe, NULL, NULL);
    rb.n++;
  }
  /* :481-491 centroids: node2edge_centroid over edge2features (nodes),
   * edge2node_centroid over node2features (edges) */
  fcsr cn = centroids(N, rp_n, col_n, N, rp_e, col_e, fe);
  fcsr ce = centroids(E, rp_e, col_e, E, rp_n, col_n, fn);
  P.n = 0;
  pat NNE = spgemm_pattern(N, NN.p, NN.j, E, A.p, A.j);          /* :493 */
  sample_pattern(s, &NNE, E, node_q, 0, 0, &P, 0);
  pat EEN = spgemm_pattern(E, EE.p, EE.j, N, AT.p, AT.j);        /* :498 */
  sample_pattern(s, &EEN, N, edge_q, 0, 0, &P, 1);
  hgref_rng w;  /* the single forked worker's copy of the parent stream */
  hgref_rng_copy(&w, s);
  for (int64_t t = 0; t < P.n; t++) {
    int32_t v = P.a[t], e = P.b[t];
    int32_t *r = rec_slot(&rb);
    if (!r) { overflow = 1; break; }
    r[0] = v + 1; r[3] = e + 1;
    sample_neighbors(&w, A.j + A.p[v], A.p[v + 1] - A.p[v], K, r + 4 + K);
    sample_neighbors(&w, AT.j + AT.p[e], AT.p[e + 1] - AT.p[e], K, r + 4);
    rb.tgt[rb.n * 3 + 2] = jac_prob(2, v, e, rp_n, col_n, fn, rp_e, col_e, fe,
                                    &cn, &ce);
    rb.n++;
  }
  free(P.a); free(P.b);
  fcsr_free(&cn); fcsr_free(&ce);
  pat_free(&A); pat_free(&AT); pat_free(&NN); pat_free(&EE);
  pat_free(&NNE); pat_free(&EEN);
  return overflow ? -1 : rb.n;
}

/* Exposed: Jaccard probabilities for pair lists (kind 0/1/2 as above). */
void hgref_jaccard_probs(int kind, int64_t n, const int32_t *pa,
                         const int32_t *pb, int64_t N, int64_t E,
                         const int32_t *rp_n, const int32_t *col_n,
                         const int32_t *rp_e, const int32_t *col_e,
                         const float *fn, const float *fe, float *out) {
  fcsr cn = {0, 0, 0}, ce = {0, 0, 0};
  if (kind == 2) {
    cn = centroids(N, rp_n, col_n, N, rp_e, col_e, fe);
    ce = centroids(E, rp_e, col_e, E, rp_n, col_n, fn);
  }
  for (int64_t t = 0; t < n; t++)
    out[t] = jac_prob(kind, pa[t], pb[t], rp_n, col_n, fn, rp_e, col_e, fe,
                      &cn, &ce);
  if (kind == 2) { fcsr_free(&cn); fcsr_free(&ce); }
}

/* ------------------------------------------------------------------------- */
/* Trainer: BooleanModel (hg2v_model.py:51-125, sigmoid heads + KLD) and      */
/* UnweightedFloatModel (:129-203, relu heads + MSE), fit loop of            */
/* embedding.py:269-305 -- Keras 2.x semantics restated (PARITY UNPINNED:    */
/* keras/tensorflow are absent):                                             */
/*   heads nn = act(N[ln].N[rn]), ee = act(E[le].E[re]),                      */
/*         ne = mean_k act(N[nn_k].N[ln]) * mean_k act(E[ne_k].E[re]);       */
/*   loss = sum over heads of batch-mean; KLD = yt'*log(yt'/yp') with         */
/*   clip(.,eps,1); MSE = (yp-yt)^2;                                          */
/*   Adagrad: a += g^2; p -= lr*g/(sqrt(a)+eps), duplicate rows summed.       */
/* perms: n_epochs x n permutation (Keras np.random.shuffle per epoch) or    */
/* NULL for in-order. EarlyStopping(monitor=loss, min_delta, patience=0).    */
/* ------------------------------------------------------------------------- */
static float act_f(int act, float z) {
  if (act == 0) return 1.0f / (1.0f + expf(-z));
  return z > 0.0f ? z : 0.0f;
}
static float act_d(int act, float z, float y) {
  if (act == 0) return y * (1.0f - y);
  return z > 0.0f ? 1.0f : 0.0f;
}
static float dot_f(const float *a, const float *b, int d) {
  float s = 0.0f;
  for (int i = 0; i < d; i++) s += a[i] * b[i];
  return s;
}

/* per-head loss value and dL/dyhat for ONE sample (not yet / batch) */
static void head_loss(int loss, float y, float yt, float *lv, float *g) {
  const float eps = 1e-7f;
  if (loss == 0) {
    float ytc = yt < eps ? eps : (yt > 1.0f ? 1.0f : yt);
    float ypc = y < eps ? eps : (y > 1.0f ? 1.0f : y);
    *lv = ytc * logf(ytc / ypc);
    *g = (y >= eps && y <= 1.0f) ? -ytc / ypc : 0.0f;
  } else {
    float df = y - yt;
    *lv = df * df;
    *g = 2.0f * df;
  }
}

/* Duplicate-row gradient sums: 0 (default) in float32 in emit order, as a
 * sequential TF CPU kernel would; 1 in float64, rounded to float32 once
 * before the Adagrad step (TF leaves the order of its fp32 segment sums
 * unspecified; the exact sum is the order-free member of that family, the
 * one the device's fixed-point sums approach). Test infrastructure: the
 * trainer parity tests report the distance between the two as the
 * ambiguity the reference semantics leave. */
/* per thread: the tests run both summation orders side by side from two
 * Python threads (ctypes calls run on the calling thread) */
static _Thread_local int g_dup_f64 = 0;
void hgref_train_set_dup_f64(int on) { g_dup_f64 = on; }

int hgref_train(int64_t n, int K, const int32_t *idx, const float *tgt, int d,
                int64_t n_node_rows, int64_t n_edge_rows, float *ntab,
                float *etab, float *nacc, float *eacc, int loss, int act,
                int batch, float lr, float eps, int max_epochs,
                const int64_t *perms, float min_delta, float *epoch_loss,
                int *epochs_run) {
  int R = 4 + 2 * K;
  float *gn = (float *)calloc((size_t)n_node_rows * d, sizeof(float));
  float *ge = (float *)calloc((size_t)n_edge_rows * d, sizeof(float));
  double *gnd = g_dup_f64 ? (double *)calloc((size_t)n_node_rows * d, sizeof(double)) : NULL;
  double *ged = g_dup_f64 ? (double *)calloc((size_t)n_edge_rows * d, sizeof(double)) : NULL;
  char *tn = (char *)calloc((size_t)n_node_rows, 1);
  char *te = (char *)calloc((size_t)n_edge_rows, 1);
  int64_t *touched_n = (int64_t *)malloc(sizeof(int64_t) * (size_t)batch * R + 8);
  int64_t *touched_e = (int64_t *)malloc(sizeof(int64_t) * (size_t)batch * R + 8);
  float *a_k = (float *)malloc(sizeof(float) * (K + 1));
  float *b_k = (float *)malloc(sizeof(float) * (K + 1));
  float *sa = (float *)malloc(sizeof(float) * (K + 1));
  float *sb = (float *)malloc(sizeof(float) * (K + 1));
  double best = INFINITY;
  int ep;
  for (ep = 0; ep < max_epochs; ep++) {
    const int64_t *perm = perms ? perms + (int64_t)ep * n : NULL;
    double loss_sum = 0.0;
    for (int64_t b0 = 0; b0 < n; b0 += batch) {
      int64_t b1 = b0 + batch < n ? b0 + batch : n;
      float inv_b = 1.0f / (float)(b1 - b0);
      int64_t ntn = 0, nte = 0;
      double bl = 0.0;
      for (int64_t q = b0; q < b1; q++) {
        int64_t rec = perm ? perm[q] : q;
        const int32_t *r = idx + rec * R;
        const float *yt = tgt + rec * 3;
        int32_t ln = r[0], le = r[1], rn = r[2], re = r[3];
        const int32_t *nnk = r + 4, *nek = r + 4 + K;
        const float *Nl = ntab + (int64_t)ln * d, *Nr = ntab + (int64_t)rn * d;
        const float *El = etab + (int64_t)le * d, *Er = etab + (int64_t)re * d;
        float z1 = dot_f(Nl, Nr, d), y1 = act_f(act, z1);
        float z2 = dot_f(El, Er, d), y2 = act_f(act, z2);
        float P = 0.0f, Q = 0.0f;
        for (int t = 0; t < K; t++) {
          a_k[t] = dot_f(ntab + (int64_t)nnk[t] * d, Nl, d);
          sa[t] = act_f(act, a_k[t]);
          P += sa[t];
          b_k[t] = dot_f(etab + (int64_t)nek[t] * d, Er, d);
          sb[t] = act_f(act, b_k[t]);
          Q += sb[t];
        }
        P = P / (float)K;
        Q = Q / (float)K;
        float y3 = P * Q;
        float l1, l2, l3, g1, g2, g3;
        head_loss(loss, y1, yt[0], &l1, &g1);
        head_loss(loss, y2, yt[1], &l2, &g2);
        head_loss(loss, y3, yt[2], &l3, &g3);
        bl += (double)l1 + (double)l2 + (double)l3;
        g1 *= inv_b; g2 *= inv_b; g3 *= inv_b;
        float dz1 = g1 * act_d(act, z1, y1);
        float dz2 = g2 * act_d(act, z2, y2);
        float dP = g3 * Q / (float)K, dQ = g3 * P / (float)K;
#define TOUCH_N(row) do { if (!tn[row]) { tn[row] = 1; touched_n[ntn++] = row; } } while (0)
#define TOUCH_E(row) do { if (!te[row]) { te[row] = 1; touched_e[nte++] = row; } } while (0)
#define ACC(g, gd, row, i, v)                                             \
  do {                                                                    \
    float v_ = (v);                                                       \
    if (gd) gd[(int64_t)(row) * d + (i)] += (double)v_;                   \
    else g[(int64_t)(row) * d + (i)] += v_;                               \
  } while (0)
        TOUCH_N(ln); TOUCH_N(rn);
        for (int i = 0; i < d; i++) {
          ACC(gn, gnd, ln, i, dz1 * Nr[i]);
          ACC(gn, gnd, rn, i, dz1 * Nl[i]);
        }
        TOUCH_E(le); TOUCH_E(re);
        for (int i = 0; i < d; i++) {
          ACC(ge, ged, le, i, dz2 * Er[i]);
          ACC(ge, ged, re, i, dz2 * El[i]);
        }
        for (int t = 0; t < K; t++) {
          float da = dP * act_d(act, a_k[t], sa[t]);
          const float *Nk = ntab + (int64_t)nnk[t] * d;
          TOUCH_N(nnk[t]);
          for (int i = 0; i < d; i++) {
            ACC(gn, gnd, nnk[t], i, da * Nl[i]);
            ACC(gn, gnd, ln, i, da * Nk[i]);
          }
          float db = dQ * act_d(act, b_k[t], sb[t]);
          const float *Ek = etab + (int64_t)nek[t] * d;
          TOUCH_E(nek[t]);
          for (int i = 0; i < d; i++) {
            ACC(ge, ged, nek[t], i, db * Er[i]);
            ACC(ge, ged, re, i, db * Ek[i]);
          }
        }
#undef ACC
      }
      /* Adagrad over touched rows (untouched rows have g == 0: no-op). */
      for (int64_t u = 0; u < ntn; u++) {
        int64_t row = touched_n[u];
        float *p = ntab + row * d, *a = nacc + row * d, *g = gn + row * d;
        double *gd = gnd ? gnd + row * d : NULL;
        for (int i = 0; i < d; i++) {
          float gi = gd ? (float)gd[i] : g[i];
          float na = a[i] + gi * gi;
          a[i] = na;
          p[i] = p[i] - (lr * gi) / (sqrtf(na) + eps);
          g[i] = 0.0f;
          if (gd) gd[i] = 0.0;
        }
        tn[row] = 0;
      }
      for (int64_t u = 0; u < nte; u++) {
        int64_t row = touched_e[u];
        float *p = etab + row * d, *a = eacc + row * d, *g = ge + row * d;
        double *gd = ged ? ged + row * d : NULL;
        for (int i = 0; i < d; i++) {
          float gi = gd ? (float)gd[i] : g[i];
          float na = a[i] + gi * gi;
          a[i] = na;
          p[i] = p[i] - (lr * gi) / (sqrtf(na) + eps);
          g[i] = 0.0f;
          if (gd) gd[i] = 0.0;
        }
        te[row] = 0;
      }
      loss_sum += bl;  /* = batch_mean * batch_size summed (BaseLogger) */
    }
    double cur = loss_sum / (double)n;
    if (epoch_loss) epoch_loss[ep] = (float)cur;
    if (cur < best - (double)min_delta) {
      best = cur;
    } else {
      ep++;
      break;
    }
  }
  if (epochs_run) *epochs_run = ep;
  free(gn); free(ge); free(gnd); free(ged); free(tn); free(te);
  free(touched_n); free(touched_e);
  free(a_k); free(b_k); free(sa); free(sb);
  return 0;
}

/* ------------------------------------------------------------------------- */
/* hg2v_weighting.py distance and span weights (34-64, 67-103, 170-192,      */
/* 207-293) with the dict helpers ZeroOneScaleValues / OneMinusValues /       */
/* AlphaScaleValues (301-333).                                               */
/* `norm` = np.linalg.norm = sqrt(x.dot(x)): numpy's FLOAT_dot / DOUBLE_dot   */
/* call OpenBLAS sdot / ddot. The fixtures come from numpy's OpenBLAS 0.3.29  */
/* SkylakeX kernels, restated here (probed on 3,000 random vectors):          */
/* sdot: k & ~31 elements in 4 x 8 float FMA accumulators (64-blocks in       */
/* 4 x 16, folded l + l+8), ((a0+a1)+a2)+a3, lanes l + l+4, (h0+h1)+(h2+h3),  */
/* the rest added in double as float products; float sqrt of the float.      */
/* ddot: k & ~15 in 4 x 4 double FMA accumulators (32-blocks 4 x 8, folded    */
/* l + l+4), same sum, (s0+s2)+(s1+s3), the rest by double FMA; sqrt.          */
/* norm 1 = ord inf (max |d|).                                                 */
/* ------------------------------------------------------------------------- */
float hgref_norm32(const float *a, const float *b, int k, int norm) {
  if (norm == 1) {
    float m = 0.0f;
    for (int i = 0; i < k; i++) {
      float d = fabsf(a[i] - b[i]);
      if (d > m) m = d;
    }
    return m;
  }
  int n1 = k & ~31, n64 = n1 & ~63, i = 0;
  float tot = 0.0f;
  if (n1) {
    float acc[32] = {0}, s[8], h[4];
    if (n64) {
      float a5[64] = {0};
      for (; i < n64; i += 64)
        for (int t = 0; t < 64; t++) {
          float d = a[i + t] - b[i + t];
          a5[t] = fmaf(d, d, a5[t]);
        }
      for (int j = 0; j < 4; j++)
        for (int l = 0; l < 8; l++) acc[j * 8 + l] = a5[j * 16 + l] + a5[j * 16 + l + 8];
    }
    for (; i < n1; i += 32)
      for (int t = 0; t < 32; t++) {
        float d = a[i + t] - b[i + t];
        acc[t] = fmaf(d, d, acc[t]);
      }
    for (int l = 0; l < 8; l++) s[l] = ((acc[l] + acc[8 + l]) + acc[16 + l]) + acc[24 + l];
    for (int l = 0; l < 4; l++) h[l] = s[l] + s[l + 4];
    tot = (h[0] + h[1]) + (h[2] + h[3]);
  }
  double dot = tot;
  for (; i < k; i++) {
    float d = a[i] - b[i];
    float p = d * d;
    dot += (double)p;
  }
  return sqrtf((float)dot);
}

double hgref_norm64(const float *a, const float *b, int k, int norm) {
  if (norm == 1) {
    double m = 0.0;
    for (int i = 0; i < k; i++) {
      double d = fabs((double)a[i] - (double)b[i]);
      if (d > m) m = d;
    }
    return m;
  }
  int n1 = k & ~15, n32 = n1 & ~31, i = 0;
  double dot = 0.0;
  if (n1) {
    double acc[16] = {0}, s[4];
    if (n32) {
      double a5[32] = {0};
      for (; i < n32; i += 32)
        for (int t = 0; t < 32; t++) {
          double d = (double)a[i + t] - (double)b[i + t];
          a5[t] = fma(d, d, a5[t]);
        }
      for (int j = 0; j < 4; j++)
        for (int l = 0; l < 4; l++) acc[j * 4 + l] = a5[j * 8 + l] + a5[j * 8 + l + 4];
    }
    for (; i < n1; i += 16)
      for (int t = 0; t < 16; t++) {
        double d = (double)a[i + t] - (double)b[i + t];
        acc[t] = fma(d, d, acc[t]);
      }
    for (int l = 0; l < 4; l++) s[l] = ((acc[l] + acc[4 + l]) + acc[8 + l]) + acc[12 + l];
    dot = (s[0] + s[2]) + (s[1] + s[3]);
  }
  for (; i < k; i++) {
    double d = (double)a[i] - (double)b[i];
    dot = fma(d, d, dot);
  }
  return sqrt(dot);
}

/* ZeroOneScaleValues -> OneMinusValues -> AlphaScaleValues on np.float32
 * values (hg2v_weighting.py:94-95): float32 arithmetic, alpha and 1 - alpha
 * weak Python scalars cast to float32 (numpy 2, NEP 50) */
static void scale_f32(int64_t n, float *v, float mn, float mx, double alpha) {
  float delta = mx - mn, a32 = (float)alpha, b32 = (float)(1.0 - alpha);
  for (int64_t t = 0; t < n; t++) {
    float o = delta == 0.0f ? 0.0f : 1.0f - (v[t] - mn) / delta;
    float p = b32 * o;
    v[t] = a32 + p;
  }
}

/* WeightByDistance (hg2v_weighting.py:67-103): per incidence (v, e) of A
 * (out_n, A's CSR order) and A^T (out_e), norm(node_vec - edge_vec) with
 * float32 vectors X[N x k], Y[E x k], then the scaling over all incidences.
 * Zeros are kept here (the reference's lil_matrix drops them). */
void hgref_weight_distance(int64_t N, int64_t E, const int32_t *rp_n,
                           const int32_t *col_n, const int32_t *rp_e,
                           const int32_t *col_e, const float *X, const float *Y,
                           int k, int norm, double alpha, float *out_n,
                           float *out_e) {
  float mn = INFINITY, mx = 0.0f;
  for (int64_t v = 0; v < N; v++)
    for (int32_t t = rp_n[v]; t < rp_n[v + 1]; t++) {
      float w = hgref_norm32(X + v * k, Y + (int64_t)col_n[t] * k, k, norm);
      out_n[t] = w;
      if (w < mn) mn = w;
      if (w > mx) mx = w;
    }
  for (int64_t e = 0; e < E; e++)
    for (int32_t t = rp_e[e]; t < rp_e[e + 1]; t++)
      out_e[t] = hgref_norm32(X + (int64_t)col_e[t] * k, Y + e * k, k, norm);
  int64_t nnz = rp_n[N];
  if (nnz == 0) return;
  scale_f32(nnz, out_n, mn, mx, alpha);
  scale_f32(nnz, out_e, mn, mx, alpha);
}

static int cmp_i32(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  return (x > y) - (x < y);
}

/* WeightBySameTypeDistance, one half (hg2v_weighting.py:37-52 on
 * node2edge * node2edge.T, :55-62): the pattern of P Q (P = rp/col over R
 * rows, Q = rq/cq), diagonal included, as CSR with ascending columns;
 * value = norm of the difference of the rows' vectors tab[R x k], scaled
 * over all entries. float32 throughout: np.array(emb.values) of protobuf's
 * upb repeated-float container (protobuf 7) is a float32 array. Returns
 * nnz; with col_out == NULL only counts (rowptr still filled). */
int64_t hgref_weight_same_type(int64_t R, const int32_t *rp, const int32_t *col,
                               const int32_t *rq, const int32_t *cq,
                               const float *tab, int k, int norm, double alpha,
                               int64_t *rowptr, int32_t *col_out,
                               float *val_out) {
  int64_t nnz = 0, cap = 16;
  int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * cap);
  float mn = INFINITY, mx = 0.0f;
  for (int64_t r = 0; r < R; r++) {
    int64_t m = 0;
    for (int32_t t = rp[r]; t < rp[r + 1]; t++) {
      int32_t e = col[t];
      for (int32_t j = rq[e]; j < rq[e + 1]; j++) {
        if (m == cap) {
          cap *= 2;
          buf = (int32_t *)realloc(buf, sizeof(int32_t) * cap);
        }
        buf[m++] = cq[j];
      }
    }
    qsort(buf, (size_t)m, sizeof(int32_t), cmp_i32);
    if (rowptr) rowptr[r] = nnz;
    for (int64_t i = 0; i < m; i++) {
      if (i > 0 && buf[i] == buf[i - 1]) continue;
      if (col_out) {
        float v = hgref_norm32(tab + r * k, tab + (int64_t)buf[i] * k, k, norm);
        col_out[nnz] = buf[i];
        val_out[nnz] = v;
        if (v < mn) mn = v;
        if (v > mx) mx = v;
      }
      nnz++;
    }
  }
  if (rowptr) rowptr[R] = nnz;
  free(buf);
  if (col_out && nnz) scale_f32(nnz, val_out, mn, mx, alpha);
  return nnz;
}

/* ComputeSpans (hg2v_weighting.py:214-233, 236-293): per row r of P, over
 * its neighbours c and dimensions, diff = other[c] - mine[r] (np.subtract
 * of two float32 containers: float32); span = max(0, max diff) -
 * min(0, min diff) */
static void spans_of(int64_t R, const int32_t *rp, const int32_t *col,
                     const float *mine, const float *other, int k, float *span) {
  for (int64_t r = 0; r < R; r++) {
    float lo = 0.0f, hi = 0.0f;
    for (int32_t t = rp[r]; t < rp[r + 1]; t++)
      for (int d = 0; d < k; d++) {
        float df = other[(int64_t)col[t] * k + d] - mine[r * k + d];
        if (df > hi) hi = df;
        if (df < lo) lo = df;
      }
    span[r] = (hi - lo) + 0.0f;
  }
}

/* WeightByAlgebraicSpan (hg2v_weighting.py:170-192) given the spans'
 * embedding: spans of nodes (over their edges) and edges (over their
 * nodes), each side zero-one / one-minus / alpha scaled (np.float32
 * values) and kept float32 (DictToSparseRow); node_major[t] = the value of
 * incidence t's edge (A multiply), edge_major[t] = its node's (A^T). */
void hgref_weight_span(int64_t N, int64_t E, const int32_t *rp_n,
                       const int32_t *col_n, const int32_t *rp_e,
                       const int32_t *col_e, const float *X, const float *Y,
                       int k, double alpha, float *sn, float *se,
                       float *node_major, float *edge_major) {
  spans_of(N, rp_n, col_n, X, Y, k, sn);
  spans_of(E, rp_e, col_e, Y, X, k, se);
  float *wn = (float *)malloc(sizeof(float) * (N + 1));
  float *we = (float *)malloc(sizeof(float) * (E + 1));
  for (int side = 0; side < 2; side++) {
    int64_t R = side ? E : N;
    const float *s = side ? se : sn;
    float *w = side ? we : wn;
    float mn = INFINITY, mx = 0.0f;
    for (int64_t r = 0; r < R; r++) {
      if (s[r] < mn) mn = s[r];
      if (s[r] > mx) mx = s[r];
      w[r] = s[r];
    }
    if (R) scale_f32(R, w, mn, mx, alpha);
  }
  for (int32_t t = 0; t < rp_n[N]; t++) node_major[t] = we[col_n[t]];
  for (int32_t t = 0; t < rp_e[E]; t++) edge_major[t] = wn[col_e[t]];
  free(wn);
  free(we);
}
