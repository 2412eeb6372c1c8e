/*
 * Multi-threaded CPU trainer: the CPU BASELINE of bench.py (timing only).
 * Test/bench infrastructure, never the product path.
 *
 * Same Keras-2.x semantics as hgref_train (hgref.c: hg2v_model.py:51-203,
 * embedding.py:269-305) with the work of one batch spread over OpenMP
 * threads the way a CPU framework does it:
 *   forward and backward per record in parallel, each record writing its
 *   gradient rows to per-slot buffers (no atomics); the batch's unique rows
 *   found by a counting sort; then per unique row, in parallel, the sum of
 *   its slots (in slot order) and the Adagrad update.
 * Batches stay sequential (the reference's semantics), so the result equals
 * hgref_train up to float summation order of duplicate rows.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline float act_f(int act, float z) {
  if (act == 0) return 1.0f / (1.0f + expf(-z));
  return z > 0.0f ? z : 0.0f;
}
static inline float act_d(int act, float z, float y) {
  if (act == 0) return y * (1.0f - y);
  return z > 0.0f ? 1.0f : 0.0f;
}
static inline float dot_f(const float *a, const float *b, int d) {
  float s = 0.0f;
  for (int i = 0; i < d; i++) s += a[i] * b[i];
  return s;
}
static inline void head_loss(int loss, float y, float yt, float *lv, float *g) {
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

int cpu_train_mt(int64_t n, int K, const int32_t *idx, const float *tgt, int d,
                 int64_t n_node_rows, int64_t n_edge_rows, float *ntab,
                 float *etab, float *nacc, float *eacc, int loss, int act,
                 int batch, float lr, float eps, int epochs, int threads,
                 double *loss_out) {
  if (threads > 0) omp_set_num_threads(threads);
  const int R = 4 + 2 * K;
  const int64_t SB = (int64_t)batch * R;
  /* per-slot gradient rows of one batch (no atomics), then per unique row */
  float *gs = (float *)malloc(sizeof(float) * SB * d);
  int32_t *un = (int32_t *)calloc((size_t)n_node_rows, sizeof(int32_t));
  int32_t *ue = (int32_t *)calloc((size_t)n_edge_rows, sizeof(int32_t));
  int64_t *urow = (int64_t *)malloc(sizeof(int64_t) * (SB + 1));
  int32_t *ucnt = (int32_t *)malloc(sizeof(int32_t) * (SB + 2));
  int32_t *uoff = (int32_t *)malloc(sizeof(int32_t) * (SB + 2));
  int32_t *slots = (int32_t *)malloc(sizeof(int32_t) * (SB + 1));
  int32_t *slot_u = (int32_t *)malloc(sizeof(int32_t) * (SB + 1));
  double total = 0.0;
  for (int ep = 0; ep < epochs; ep++) {
    for (int64_t b0 = 0; b0 < n; b0 += batch) {
      const int64_t b1 = b0 + batch < n ? b0 + batch : n;
      const float inv_b = 1.0f / (float)(b1 - b0);
      double bl = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : bl)
      for (int64_t q = b0; q < b1; q++) {
        const int32_t *r = idx + q * R;
        const float *yt = tgt + q * 3;
        const int32_t ln = r[0], le = r[1], rn = r[2], re = r[3];
        const int32_t *nnk = r + 4, *nek = r + 4 + K;
        const float *Nl = ntab + (int64_t)ln * d, *Nr = ntab + (int64_t)rn * d;
        const float *El = etab + (int64_t)le * d, *Er = etab + (int64_t)re * d;
        float a_k[16], b_k[16], sa[16], sb[16];
        const float z1 = dot_f(Nl, Nr, d), y1 = act_f(act, z1);
        const float z2 = dot_f(El, Er, d), y2 = act_f(act, z2);
        float P = 0.0f, Q = 0.0f;
        for (int t = 0; t < K; t++) {
          a_k[t] = dot_f(ntab + (int64_t)nnk[t] * d, Nl, d);
          sa[t] = act_f(act, a_k[t]);
          P += sa[t];
          b_k[t] = dot_f(etab + (int64_t)nek[t] * d, Er, d);
          sb[t] = act_f(act, b_k[t]);
          Q += sb[t];
        }
        P /= (float)K;
        Q /= (float)K;
        float l1, l2, l3, g1, g2, g3;
        head_loss(loss, y1, yt[0], &l1, &g1);
        head_loss(loss, y2, yt[1], &l2, &g2);
        head_loss(loss, P * Q, yt[2], &l3, &g3);
        bl += (double)l1 + (double)l2 + (double)l3;
        g1 *= inv_b; g2 *= inv_b; g3 *= inv_b;
        const float dz1 = g1 * act_d(act, z1, y1), dz2 = g2 * act_d(act, z2, y2);
        const float dP = g3 * Q / (float)K, dQ = g3 * P / (float)K;
        float *g = gs + (q - b0) * R * d;  /* slots in record-layout order */
        float *gln = g, *gle = g + d, *grn = g + 2 * d, *gre = g + 3 * d;
        for (int i = 0; i < d; i++) {
          gln[i] = dz1 * Nr[i];
          grn[i] = dz1 * Nl[i];
          gle[i] = dz2 * Er[i];
          gre[i] = dz2 * El[i];
        }
        for (int t = 0; t < K; t++) {
          const float da = dP * act_d(act, a_k[t], sa[t]);
          const float db = dQ * act_d(act, b_k[t], sb[t]);
          const float *Nk = ntab + (int64_t)nnk[t] * d, *Ek = etab + (int64_t)nek[t] * d;
          float *gk = g + (4 + t) * d, *hk = g + (4 + K + t) * d;
          for (int i = 0; i < d; i++) {
            gk[i] = da * Nl[i];
            gln[i] += da * Nk[i];
            hk[i] = db * Er[i];
            gre[i] += db * Ek[i];
          }
        }
      }
      /* unique rows of the batch and their slots (counting sort) */
      const int64_t ns = (b1 - b0) * R;
      int64_t nu = 0;
      for (int64_t t = 0; t < ns; t++) {
        const int s = (int)(t % R);
        const int edge = s == 1 || s == 3 || s >= 4 + K;
        const int32_t row = idx[b0 * R + t];
        int32_t *m = edge ? ue : un;
        if (!m[row]) {
          m[row] = (int32_t)++nu;
          urow[nu - 1] = edge ? -(int64_t)row - 1 : row;
          ucnt[nu - 1] = 0;
        }
        slot_u[t] = m[row] - 1;
        ucnt[m[row] - 1]++;
      }
      uoff[0] = 0;
      for (int64_t u = 0; u < nu; u++) uoff[u + 1] = uoff[u] + ucnt[u];
      for (int64_t u = 0; u < nu; u++) ucnt[u] = uoff[u];
      for (int64_t t = 0; t < ns; t++) slots[ucnt[slot_u[t]]++] = (int32_t)t;
#pragma omp parallel for schedule(static)
      for (int64_t u = 0; u < nu; u++) {
        const int e = urow[u] < 0;
        const int64_t row = e ? -urow[u] - 1 : urow[u];
        float *p = (e ? etab : ntab) + row * d, *a = (e ? eacc : nacc) + row * d;
        float gsum[1024];
        for (int i = 0; i < d; i++) gsum[i] = 0.0f;
        for (int32_t j = uoff[u]; j < uoff[u + 1]; j++) {
          const float *gj = gs + (int64_t)slots[j] * d;
          for (int i = 0; i < d; i++) gsum[i] += gj[i];
        }
        for (int i = 0; i < d; i++) {
          const float na = a[i] + gsum[i] * gsum[i];
          a[i] = na;
          p[i] = p[i] - (lr * gsum[i]) / (sqrtf(na) + eps);
        }
        (e ? ue : un)[row] = 0;
      }
      total += bl;
    }
  }
  if (loss_out) *loss_out = total / (double)n / (double)(epochs > 0 ? epochs : 1);
  free(gs); free(un); free(ue); free(urow); free(ucnt); free(uoff); free(slots);
  free(slot_u);
  return 0;
}
