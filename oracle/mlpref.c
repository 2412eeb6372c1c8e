/*
 * CPU restatement of the Keras MLPs behind the embedding combiners and the
 * link-prediction classifier. TEST INFRASTRUCTURE ONLY (the checker of
 * libhgx's hgx_mlp_*, and bench.py's CPU baseline for them); never the
 * product path.
 *
 * Models (Keras 2.x semantics, restated from the reference's model code):
 *   kind 0  evaluation_util.py:489-505  (_TrainNodeEdgeEmbeddingClassifier)
 *           x = [node_emb | edge_emb] -> Dense(d, relu) -> Dense(1, sigmoid)
 *   kind 1  combine_embeddings_util.py:95-130 (with_auto_encoder=False)
 *           per side Dropout(0.5) -> Dense(h, relu) -> Dense(d, sigmoid);
 *           Concatenate -> Dense(d, relu) -> Dense(1, sigmoid)
 *   kind 2  the same + per side joint -> Dense(h, relu) -> Dense(in, relu)
 *           reproducing the undropped input; loss weights [4, 1, 1]
 *           (combine_embeddings_util.py:110-145)
 * Training: loss = sum_o w_o * mean_batch(mean_cols((y - t)^2)) (Keras
 * mean_squared_error), gradients of the whole batch, then Adagrad on every
 * kernel and bias (a += g^2; p -= lr g / (sqrt(a) + eps), accumulators from
 * zero), batches in the given permutation order, EarlyStopping(monitor=loss,
 * min_delta, patience=0) on the batch-size-weighted epoch mean.
 * Dropout: Keras draws its mask from TF's RNG, which cannot be reproduced;
 * both this restatement and the device use the counter-based mask below
 * (keep = bit of rand64(seed, stream, p * ceil(in4/64) + col/64)), so GPU
 * parity is checked with identical masks. PARITY UNPINNED against the
 * reference itself: keras/tensorflow are absent here, and no reference test
 * pins trained values.
 *
 * Arithmetic: every dot product is a sequential fmaf chain over the
 * reduction index (the v_mfma_f32 products are exact f32 fma steps), so
 * device and restatement differ only by the device's 4-way split of each
 * reduction. Built with -ffp-contract=off; OpenMP parallelises over output
 * rows (each element is computed by one thread, order fixed), so the result
 * does not depend on the thread count.
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
static inline uint64_t rand64(uint64_t seed, uint64_t stream, uint64_t ctr) {
  return mix64(mix64(seed ^ mix64(stream + 0x632be59bd9b4e019ull)) + ctr);
}

enum { SIGMOID = 0, RELU = 1 };
/* Cephes expf as explicit fma steps: the device computes the same bits */
static inline float hexp(float x) {
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
static inline float act_f(int a, float z) {
  return a == SIGMOID ? 1.0f / (1.0f + hexp(-z)) : (z > 0.f ? z : 0.f);
}
static inline float act_d(int a, float y) {
  return a == SIGMOID ? y * (1.0f - y) : (y > 0.f ? 1.0f : 0.0f);
}

typedef struct {
  int K, N, act;
  int seg, off; /* device position of input k: k < seg ? k : off + k - seg */
  float *W, *b, *aW, *ab, *gW, *gb;
} Layer;

typedef struct {
  int kind, in, out, hid, nl;
  Layer L[10];
  int pre_n, pre_e, joint_n, joint_e, post_n, post_e, rec_n, rec_e, hidden, label;
} Net;

static void add_layer(Net *n, int K, int N, int act) {
  Layer *l = &n->L[n->nl++];
  l->seg = K;
  l->off = 0;
  l->K = K;
  l->N = N;
  l->act = act;
  l->W = calloc((size_t)K * N, sizeof(float));
  l->aW = calloc((size_t)K * N, sizeof(float));
  l->gW = calloc((size_t)K * N, sizeof(float));
  l->b = calloc(N, sizeof(float));
  l->ab = calloc(N, sizeof(float));
  l->gb = calloc(N, sizeof(float));
}

static void net_init(Net *n, int kind, int in, int out) {
  memset(n, 0, sizeof(*n));
  n->kind = kind;
  n->in = in;
  n->out = out;
  n->pre_n = n->pre_e = n->joint_n = n->joint_e = n->post_n = n->post_e = -1;
  n->rec_n = n->rec_e = n->hidden = n->label = -1;
  if (kind == 0) {
    n->hid = in;
    n->pre_n = n->nl;
    add_layer(n, 2 * in, in, RELU);
    n->L[n->pre_n].seg = in;            /* [node | edge], each 4-aligned */
    n->L[n->pre_n].off = (in + 3) / 4 * 4;
    n->label = n->nl;
    add_layer(n, in, 1, SIGMOID);
    return;
  }
  const int h = (in + out) / 2;
  n->hid = h;
  n->pre_n = n->nl; add_layer(n, in, h, RELU);
  n->pre_e = n->nl; add_layer(n, in, h, RELU);
  n->joint_n = n->nl; add_layer(n, h, out, SIGMOID);
  n->joint_e = n->nl; add_layer(n, h, out, SIGMOID);
  if (kind == 2) {
    n->post_n = n->nl; add_layer(n, out, h, RELU);
    n->post_e = n->nl; add_layer(n, out, h, RELU);
    n->rec_n = n->nl; add_layer(n, h, in, RELU);
    n->rec_e = n->nl; add_layer(n, h, in, RELU);
  }
  n->hidden = n->nl; add_layer(n, 2 * out, out, RELU);
  n->L[n->hidden].seg = out;            /* [J_node | J_edge], each 64-aligned */
  n->L[n->hidden].off = (out + 63) / 64 * 64;
  n->label = n->nl; add_layer(n, out, 1, SIGMOID);
}

static void net_free(Net *n) {
  for (int q = 0; q < n->nl; q++) {
    Layer *l = &n->L[q];
    free(l->W); free(l->aW); free(l->gW); free(l->b); free(l->ab); free(l->gb);
  }
}

static void weights_io(Net *n, float *flat, int set) {
  int64_t off = 0;
  for (int q = 0; q < n->nl; q++) {
    Layer *l = &n->L[q];
    const size_t nw = (size_t)l->K * l->N;
    if (set) {
      memcpy(l->W, flat + off, nw * sizeof(float));
      memcpy(l->b, flat + off + nw, l->N * sizeof(float));
      memset(l->aW, 0, nw * sizeof(float));
      memset(l->ab, 0, l->N * sizeof(float));
    } else {
      memcpy(flat + off, l->W, nw * sizeof(float));
      memcpy(flat + off + nw, l->b, l->N * sizeof(float));
    }
    off += nw + l->N;
  }
}

/* Reduction order of the device (hgx_mlp.hip): a dot product over positions
 * p is split into 4 partial fmaf chains by wave w = (p % 64) / 16 (each in
 * increasing p: the v_mfma_f32_32x32x2_f32 steps of that wave), combined as
 * ((w0 + w1) + w2) + w3. Zero padding of the device layout adds exact
 * no-ops, so only the positions matter. */
#define WAVE(p) (((p)&63) >> 4)
static int g_grad_only = 0;

/* Y[m][n] = act(sum_k X[m][k] W[k][n] + b[n]); n innermost (vectorises) */
static void fwd(const Layer *l, int M, const float *X, int ldx, float *Y, int ldy) {
#pragma omp parallel
  {
    float *acc = malloc(sizeof(float) * 4 * l->N);
#pragma omp for schedule(static)
    for (int m = 0; m < M; m++) {
      for (int q = 0; q < 4 * l->N; q++) acc[q] = 0.f;
      for (int k = 0; k < l->K; k++) {
        const int pos = k < l->seg ? k : l->off + (k - l->seg);
        float *a = acc + WAVE(pos) * l->N;
        const float xv = X[(size_t)m * ldx + k];
        const float *w = l->W + (size_t)k * l->N;
        for (int n = 0; n < l->N; n++) a[n] = fmaf(xv, w[n], a[n]);
      }
      float *z = Y + (size_t)m * ldy;
      for (int n = 0; n < l->N; n++) {
        const float v = ((acc[n] + acc[l->N + n]) + acc[2 * l->N + n]) + acc[3 * l->N + n];
        z[n] = act_f(l->act, v + l->b[n]);
      }
    }
    free(acc);
  }
}

/* the N = 1 label layer's dot product: 64 lane chains (k = lane + 64 j),
 * then the device's butterfly (xor 1, xor 2, half-row mirror, row mirror,
 * xor 16, xor 32) */
static float head_dot(const float *h, const float *w, int K) {
  float x[64], y[64];
  for (int l = 0; l < 64; l++) {
    float s = 0.f;
    for (int k = l; k < K; k += 64) s = fmaf(h[k], w[k], s);
    x[l] = s;
  }
  for (int step = 0; step < 6; step++) {
    for (int l = 0; l < 64; l++) {
      int p;
      switch (step) {
        case 0: p = l ^ 1; break;
        case 1: p = l ^ 2; break;
        case 2: p = (l & ~7) | (7 - (l & 7)); break;
        case 3: p = (l & ~15) | (15 - (l & 15)); break;
        case 4: p = l ^ 16; break;
        default: p = l ^ 32; break;
      }
      y[l] = x[l] + x[p];
    }
    memcpy(x, y, sizeof(x));
  }
  return x[0];
}

static void head_fwd(const Layer *l, int M, const float *H, int ldh, float *y) {
  for (int m = 0; m < M; m++)
    y[m] = act_f(l->act, head_dot(H + (size_t)m * ldh, l->W, l->K) + l->b[0]);
}

/* dX[m][k] = (sum over the terms' n of dZ_t[m][n] W_t[row0_t + k][n]) *
 * act'(Y[m][k]): one device accumulator per wave runs over term 0's
 * positions, then term 1's */
typedef struct {
  const float *dZ;
  const Layer *l;
  int row0;
} Term;
static void bwd_terms(int M, const Term *t, int nt, int K, const float *Y, int ldy,
                      int act, float *dX, int ldd) {
  float *Wt[2];
  for (int q = 0; q < nt; q++) {
    const Layer *l = t[q].l;
    Wt[q] = malloc(sizeof(float) * (size_t)l->N * K);
    for (int k = 0; k < K; k++)
      for (int n = 0; n < l->N; n++)
        Wt[q][(size_t)n * K + k] = l->W[(size_t)(t[q].row0 + k) * l->N + n];
  }
#pragma omp parallel
  {
    float *acc = malloc(sizeof(float) * 4 * K);
#pragma omp for schedule(static)
    for (int m = 0; m < M; m++) {
      for (int q = 0; q < 4 * K; q++) acc[q] = 0.f;
      for (int q = 0; q < nt; q++) {
        const int N = t[q].l->N;
        for (int n = 0; n < N; n++) {
          float *a = acc + WAVE(n) * K;
          const float dv = t[q].dZ[(size_t)m * N + n];
          const float *w = Wt[q] + (size_t)n * K;
          for (int k = 0; k < K; k++) a[k] = fmaf(dv, w[k], a[k]);
        }
      }
      for (int k = 0; k < K; k++) {
        const float v = ((acc[k] + acc[K + k]) + acc[2 * K + k]) + acc[3 * K + k];
        dX[(size_t)m * ldd + k] = v * act_d(act, Y[(size_t)m * ldy + k]);
      }
    }
    free(acc);
  }
  for (int q = 0; q < nt; q++) free(Wt[q]);
}

/* weight gradient (reduction over batch rows in the device's order), the
 * bias gradient (8 row groups m = g, g+8, ..., then g = 0..7), Adagrad */
static void wgrad_update(Layer *l, int M, const float *X, int ldx, const float *dZ,
                         float lr, float eps) {
#pragma omp parallel
  {
    float *acc = malloc(sizeof(float) * 4 * l->N);
#pragma omp for schedule(static)
    for (int k = 0; k < l->K; k++) {
      for (int q = 0; q < 4 * l->N; q++) acc[q] = 0.f;
      for (int m = 0; m < M; m++) {
        float *a = acc + WAVE(m) * l->N;
        const float xv = X[(size_t)m * ldx + k];
        const float *dz = dZ + (size_t)m * l->N;
        for (int n = 0; n < l->N; n++) a[n] = fmaf(xv, dz[n], a[n]);
      }
      float *g = l->gW + (size_t)k * l->N;
      for (int n = 0; n < l->N; n++)
        g[n] = ((acc[n] + acc[l->N + n]) + acc[2 * l->N + n]) + acc[3 * l->N + n];
    }
    free(acc);
  }
  for (int n = 0; n < l->N; n++) {
    float s[8] = {0};
    for (int m = 0; m < M; m++) s[m & 7] += dZ[(size_t)m * l->N + n];
    float g = 0.f;
    for (int q = 0; q < 8; q++) g += s[q];
    l->gb[n] = g;
  }
  const size_t nw = (size_t)l->K * l->N;
  if (g_grad_only) { /* debug twin of the device's HGX_MLP_GRAD_AT */
    memcpy(l->W, l->gW, nw * sizeof(float));
    memcpy(l->b, l->gb, l->N * sizeof(float));
    return;
  }
#pragma omp parallel for schedule(static)
  for (size_t q = 0; q < nw; q++) {
    const float g = l->gW[q];
    l->aW[q] = l->aW[q] + g * g;
    l->W[q] = l->W[q] - (lr * g) / (sqrtf(l->aW[q]) + eps);
  }
  for (int n = 0; n < l->N; n++) {
    const float g = l->gb[n];
    l->ab[n] = l->ab[n] + g * g;
    l->b[n] = l->b[n] - (lr * g) / (sqrtf(l->ab[n]) + eps);
  }
}

typedef struct {
  int64_t nrows, erows;
  const float *nt, *et;
} Tabs;

/* input rows of a batch; kind 0: [node | edge]; else the side's row,
 * dropped when `stream` != 0 (mask keyed by the epoch position p0 + m) */
static void gather(const Net *n, const Tabs *t, int side, int M, const int32_t *nr,
                   const int32_t *er, int64_t p0, uint64_t seed, uint32_t stream,
                   int drop, float *X) {
  const int in = n->in;
  if (n->kind == 0) {
    for (int m = 0; m < M; m++) {
      memcpy(X + (size_t)m * 2 * in, t->nt + (size_t)nr[m] * in, in * sizeof(float));
      memcpy(X + (size_t)m * 2 * in + in, t->et + (size_t)er[m] * in, in * sizeof(float));
    }
    return;
  }
  const int w64 = (((in + 3) / 4 * 4) + 63) / 64;
  for (int m = 0; m < M; m++) {
    const float *src = side == 0 ? t->nt + (size_t)nr[m] * in : t->et + (size_t)er[m] * in;
    for (int k = 0; k < in; k++) {
      float v = src[k];
      if (drop) {
        const uint64_t r = rand64(seed, stream + (uint32_t)side,
                                  (uint64_t)(p0 + m) * (uint64_t)w64 + (k >> 6));
        v = ((r >> (k & 63)) & 1) ? v * 2.0f : 0.0f;
      }
      X[(size_t)m * in + k] = v;
    }
  }
}

typedef struct {
  float *Xn, *Xe, *Tn, *Te, *Hn, *He, *J, *Hm, *Pn, *Pe, *Rn, *Re, *y;
  float *dHn, *dHe, *dHm, *dz4, *dPn, *dPe, *dRn, *dRe;
} Bufs;

static float *fz(size_t n) { return calloc(n ? n : 1, sizeof(float)); }

static void bufs_alloc(Bufs *b, const Net *n, int B) {
  const int in = n->in, h = n->hid, d = n->out;
  const int xin = n->kind == 0 ? 2 * in : in;
  b->Xn = fz((size_t)B * xin); b->Xe = fz((size_t)B * in);
  b->Tn = fz((size_t)B * in); b->Te = fz((size_t)B * in);
  b->Hn = fz((size_t)B * h); b->He = fz((size_t)B * h);
  b->J = fz((size_t)B * 2 * d); b->Hm = fz((size_t)B * d);
  b->Pn = fz((size_t)B * h); b->Pe = fz((size_t)B * h);
  b->Rn = fz((size_t)B * in); b->Re = fz((size_t)B * in);
  b->y = fz(B);
  b->dHn = fz((size_t)B * h); b->dHe = fz((size_t)B * h);
  b->dHm = fz((size_t)B * d);
  b->dz4 = fz(B); b->dPn = fz((size_t)B * h); b->dPe = fz((size_t)B * h);
  b->dRn = fz((size_t)B * in); b->dRe = fz((size_t)B * in);
}
static void bufs_free(Bufs *b) {
  float **p = (float **)b;
  for (size_t q = 0; q < sizeof(Bufs) / sizeof(float *); q++) free(p[q]);
}

/* forward of M rows; train = dropout on (combiners) */
static void forward(Net *n, const Tabs *t, Bufs *b, int M, const int32_t *nr,
                    const int32_t *er, int64_t p0, uint64_t seed, uint32_t stream,
                    int train) {
  const int d = n->out;
  if (n->kind == 0) {
    gather(n, t, 0, M, nr, er, p0, seed, stream, 0, b->Xn);
    fwd(&n->L[n->pre_n], M, b->Xn, 2 * n->in, b->Hn, n->hid);
    head_fwd(&n->L[n->label], M, b->Hn, n->hid, b->y);
    return;
  }
  gather(n, t, 0, M, nr, er, p0, seed, stream, train, b->Xn);
  gather(n, t, 1, M, nr, er, p0, seed, stream, train, b->Xe);
  fwd(&n->L[n->pre_n], M, b->Xn, n->in, b->Hn, n->hid);
  fwd(&n->L[n->pre_e], M, b->Xe, n->in, b->He, n->hid);
  fwd(&n->L[n->joint_n], M, b->Hn, n->hid, b->J, 2 * d);
  fwd(&n->L[n->joint_e], M, b->He, n->hid, b->J + d, 2 * d);
  fwd(&n->L[n->hidden], M, b->J, 2 * d, b->Hm, d);
  head_fwd(&n->L[n->label], M, b->Hm, d, b->y);
  if (n->kind == 2 && train) {
    fwd(&n->L[n->post_n], M, b->J, 2 * d, b->Pn, n->hid);
    fwd(&n->L[n->post_e], M, b->J + d, 2 * d, b->Pe, n->hid);
    fwd(&n->L[n->rec_n], M, b->Pn, n->hid, b->Rn, n->in);
    fwd(&n->L[n->rec_e], M, b->Pe, n->hid, b->Re, n->in);
  }
}

/* one training batch; returns its loss */
static double train_batch(Net *n, const Tabs *t, Bufs *b, int M, const int32_t *nr,
                          const int32_t *er, const float *lab, int64_t p0, uint64_t seed,
                          uint32_t stream, float lr, float eps) {
  const int d = n->out, h = n->hid, in = n->in;
  forward(n, t, b, M, nr, er, p0, seed, stream, 1);
  const float lw = n->kind == 2 ? 4.0f : 1.0f;
  double loss = 0.0, se = 0.0;
  for (int m = 0; m < M; m++) {
    const float diff = b->y[m] - lab[m];
    se += (double)diff * diff;
    b->dz4[m] = lw * 2.0f * diff / (float)M * act_d(SIGMOID, b->y[m]);
  }
  loss += lw * se / M;
  /* the label layer's input delta (fused into the device's head kernel) */
  const Layer *lab_l = &n->L[n->label];
  float *Hin = n->kind == 0 ? b->Hn : b->Hm, *dHin = n->kind == 0 ? b->dHn : b->dHm;
  const int hin = n->kind == 0 ? h : d;
  for (int m = 0; m < M; m++)
    for (int k = 0; k < hin; k++)
      dHin[(size_t)m * hin + k] =
          b->dz4[m] * lab_l->W[k] * act_d(RELU, Hin[(size_t)m * hin + k]);
  if (n->kind == 0) {
    wgrad_update(&n->L[n->pre_n], M, b->Xn, 2 * in, b->dHn, lr, eps);
    wgrad_update(&n->L[n->label], M, b->Hn, h, b->dz4, lr, eps);
    return loss;
  }
  float *dJn = malloc(sizeof(float) * (size_t)M * d), *dJe = malloc(sizeof(float) * (size_t)M * d);
  if (n->kind == 2) {
    float *R[2] = {b->Rn, b->Re}, *dR[2] = {b->dRn, b->dRe}, *X[2] = {b->Tn, b->Te};
    float *P[2] = {b->Pn, b->Pe}, *dP[2] = {b->dPn, b->dPe};
    const int rl[2] = {n->rec_n, n->rec_e};
    gather(n, t, 0, M, nr, er, p0, seed, stream, 0, b->Tn);
    gather(n, t, 1, M, nr, er, p0, seed, stream, 0, b->Te);
    for (int s = 0; s < 2; s++) {
      double sr = 0.0;
      for (int m = 0; m < M; m++)
        for (int k = 0; k < in; k++) {
          const size_t q = (size_t)m * in + k;
          const float diff = R[s][q] - X[s][q];
          sr += (double)diff * diff;
          dR[s][q] = 1.0f * 2.0f * diff / ((float)in * (float)M) * act_d(RELU, R[s][q]);
        }
      loss += sr / ((double)in * M);
      Term tr = {dR[s], &n->L[rl[s]], 0};
      bwd_terms(M, &tr, 1, h, P[s], h, RELU, dP[s], h);
    }
  }
  /* joint layers: from the merged hidden layer (+ the post layers) */
  for (int s = 0; s < 2; s++) {
    Term tj[2] = {{b->dHm, &n->L[n->hidden], s * d},
                  {s ? b->dPe : b->dPn, &n->L[s ? n->post_e : n->post_n], 0}};
    bwd_terms(M, tj, n->kind == 2 ? 2 : 1, d, b->J + s * d, 2 * d, SIGMOID,
              s ? dJe : dJn, d);
  }
  Term tn = {dJn, &n->L[n->joint_n], 0}, te = {dJe, &n->L[n->joint_e], 0};
  bwd_terms(M, &tn, 1, h, b->Hn, h, RELU, b->dHn, h);
  bwd_terms(M, &te, 1, h, b->He, h, RELU, b->dHe, h);
  /* every gradient was taken with the pre-update weights; now update */
  wgrad_update(&n->L[n->pre_n], M, b->Xn, in, b->dHn, lr, eps);
  wgrad_update(&n->L[n->pre_e], M, b->Xe, in, b->dHe, lr, eps);
  wgrad_update(&n->L[n->joint_n], M, b->Hn, h, dJn, lr, eps);
  wgrad_update(&n->L[n->joint_e], M, b->He, h, dJe, lr, eps);
  if (n->kind == 2) {
    wgrad_update(&n->L[n->post_n], M, b->J, 2 * d, b->dPn, lr, eps);
    wgrad_update(&n->L[n->post_e], M, b->J + d, 2 * d, b->dPe, lr, eps);
    wgrad_update(&n->L[n->rec_n], M, b->Pn, h, b->dRn, lr, eps);
    wgrad_update(&n->L[n->rec_e], M, b->Pe, h, b->dRe, lr, eps);
  }
  wgrad_update(&n->L[n->hidden], M, b->J, 2 * d, b->dHm, lr, eps);
  wgrad_update(&n->L[n->label], M, b->Hm, d, b->dz4, lr, eps);
  free(dJn);
  free(dJe);
  return loss;
}

/* OpenMP threads of the following calls (bench.py's CPU baseline; the
   results do not depend on it) */
void mlpref_set_threads(int threads) {
  if (threads > 0) omp_set_num_threads(threads);
}

int mlpref_num_weights(int kind, int in, int out, int64_t *nw) {
  Net n;
  net_init(&n, kind, in, out);
  int64_t s = 0;
  for (int q = 0; q < n.nl; q++) s += (int64_t)n.L[q].K * n.L[q].N + n.L[q].N;
  net_free(&n);
  *nw = s;
  return 0;
}

/* max_batches > 0 stops after that many batches (CPU-baseline timing) */
int mlpref_fit(int kind, int in, int out, float *weights, int64_t node_rows,
               const float *ntab, int64_t edge_rows, const float *etab, int64_t n,
               const int32_t *nrow, const int32_t *erow, const float *label, int batch,
               int max_epochs, float lr, float eps, float min_delta, uint64_t seed,
               const int64_t *perms, int64_t max_batches, float *epoch_loss,
               int *epochs_run) {
  Net net;
  net_init(&net, kind, in, out);
  weights_io(&net, weights, 1);
  Tabs t = {node_rows, edge_rows, ntab, etab};
  Bufs b;
  bufs_alloc(&b, &net, batch);
  int32_t *bn = malloc(sizeof(int32_t) * batch), *be = malloc(sizeof(int32_t) * batch);
  float *bl = malloc(sizeof(float) * batch);
  double best = INFINITY;
  int ran = 0;
  int64_t done = 0;
  const char *ga = getenv("HGX_MLP_GRAD_AT");
  const int64_t grad_at = ga ? atoll(ga) : -1;
  for (int ep = 0; ep < max_epochs; ep++) {
    const int64_t *perm = perms + (int64_t)ep * n;
    const uint32_t stream = 0x44000000u + 4u * (uint32_t)ep;
    double tot = 0.0;
    int64_t seen = 0;
    for (int64_t p0 = 0; p0 < n; p0 += batch) {
      const int M = (int)(n - p0 < batch ? n - p0 : batch);
      for (int m = 0; m < M; m++) {
        const int64_t s = perm[p0 + m];
        bn[m] = nrow[s];
        be[m] = erow[s];
        bl[m] = label[s];
      }
      g_grad_only = grad_at >= 0 && done >= grad_at;
      tot += train_batch(&net, &t, &b, M, bn, be, bl, p0, seed, stream, lr, eps) * M;
      seen += M;
      ++done;
      if (max_batches > 0 && done >= max_batches) break;
    }
    const double eloss = tot / (double)seen;
    if (epoch_loss) epoch_loss[ep] = (float)eloss;
    ran = ep + 1;
    if (max_batches > 0 && done >= max_batches) break;
    if (eloss + (double)min_delta < best) best = eloss;
    else break;
  }
  if (epochs_run) *epochs_run = ran;
  weights_io(&net, weights, 0);
  free(bn); free(be); free(bl);
  bufs_free(&b);
  net_free(&net);
  return 0;
}

/* output 0: label per pair; 1 / 2: joint node / edge rows (n x out) */
int mlpref_predict(int kind, int in, int out, const float *weights, int64_t node_rows,
                   const float *ntab, int64_t edge_rows, const float *etab, int output,
                   int64_t n, const int32_t *nrow, const int32_t *erow, float *res) {
  Net net;
  net_init(&net, kind, in, out);
  weights_io(&net, (float *)weights, 1);
  Tabs t = {node_rows, edge_rows, ntab, etab};
  const int B = 256;
  Bufs b;
  bufs_alloc(&b, &net, B);
  int32_t *zero = calloc(B, sizeof(int32_t));
  for (int64_t p0 = 0; p0 < n; p0 += B) {
    const int M = (int)(n - p0 < B ? n - p0 : B);
    const int32_t *nr = nrow ? nrow + p0 : zero, *er = erow ? erow + p0 : zero;
    forward(&net, &t, &b, M, nr, er, p0, 0, 0, 0);
    for (int m = 0; m < M; m++) {
      if (output == 0) res[p0 + m] = b.y[m];
      else
        memcpy(res + (p0 + m) * out, b.J + (size_t)m * 2 * out + (output == 2 ? out : 0),
               out * sizeof(float));
    }
  }
  free(zero);
  bufs_free(&b);
  net_free(&net);
  return 0;
}
