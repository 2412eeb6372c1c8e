// Host-side synthetic incidence generation and CSR transpose for the
// large configurations of SURVEY.md §8(d) (C4/C5: power-law 10M x 5M,
// ~2e8 incidences), where numpy sorting of 2e8 keys takes minutes.
// Bench / test data plumbing, not a reference entry point; no device code.
//
// Power-law graph: node v has 1 + Poisson(mean - 1) distinct edges, each
// drawn with probability proportional to rank^-exponent (Vose alias table);
// duplicates within a node are redrawn. Edges no node picked are dropped and
// the rest renumbered in order, so every row of both orientations is
// non-empty. Work is split into a fixed number of node chunks with their own
// counter-based streams: the result depends only on the seed.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#include "hgx.h"
#include "hgx_internal.h"

namespace {

constexpr int kChunks = 64;

struct Stream {
  uint64_t s;
  explicit Stream(uint64_t seed, uint64_t id)
      : s(hgx::mix64(seed ^ hgx::mix64(id + 0x9e3779b97f4a7c15ull))) {}
  uint64_t next() { return hgx::mix64(s += 0x9e3779b97f4a7c15ull); }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

int poisson(Stream &r, double lam) {
  // Knuth's product method (lam ~ 19 here: ~20 draws per sample)
  const double L = std::exp(-lam);
  int k = 0;
  double p = 1.0;
  do {
    k++;
    p *= r.uniform();
  } while (p > L);
  return k - 1;
}

struct Alias {
  std::vector<double> prob;
  std::vector<int32_t> alias;
  explicit Alias(int32_t n, double exponent) : prob(n), alias(n) {
    std::vector<double> w(n);
    double sum = 0.0;
    for (int32_t i = 0; i < n; i++) sum += (w[i] = std::pow((double)(i + 1), -exponent));
    std::vector<int32_t> small, large;
    small.reserve(n);
    large.reserve(n);
    for (int32_t i = 0; i < n; i++) {
      w[i] = w[i] * n / sum;
      (w[i] < 1.0 ? small : large).push_back(i);
    }
    while (!small.empty() && !large.empty()) {
      const int32_t s = small.back(), l = large.back();
      small.pop_back();
      prob[s] = w[s];
      alias[s] = l;
      w[l] = (w[l] + w[s]) - 1.0;
      if (w[l] < 1.0) {
        large.pop_back();
        small.push_back(l);
      }
    }
    for (int32_t i : large) prob[i] = 1.0, alias[i] = i;
    for (int32_t i : small) prob[i] = 1.0, alias[i] = i;
  }
  int32_t draw(Stream &r) const {
    const uint64_t x = r.next();
    const int32_t i = (int32_t)((x >> 32) * (uint64_t)prob.size() >> 32);
    const double u = (double)(x & 0xffffffffu) * (1.0 / 4294967296.0);
    return u < prob[i] ? i : alias[i];
  }
};

template <class F>
void parallel_chunks(int n, F fn) {
  const int nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++)
    th.emplace_back([&, t] {
      for (int c = t; c < n; c += nt) fn(c);
    });
  for (auto &x : th) x.join();
}

}  // namespace

extern "C" int hgx_synth_powerlaw(int32_t N, int32_t E, double mean_degree,
                                  double exponent, uint64_t seed,
                                  int32_t *rowptr_n, int32_t *col_n,
                                  int64_t *nnz, int32_t *E_out) {
  if (N < 1 || E < 1 || !(mean_degree >= 1.0) || !rowptr_n || !nnz)
    return HGX_EINVAL;
  // degrees (a pure function of the seed: the two calls agree)
  std::vector<int64_t> chunk_nnz(kChunks + 1, 0);
  const int32_t per = (N + kChunks - 1) / kChunks;
  parallel_chunks(kChunks, [&](int c) {
    Stream r(seed, 2 * (uint64_t)c);
    const int32_t v0 = std::min(N, c * per), v1 = std::min(N, v0 + per);
    int64_t s = 0;
    for (int32_t v = v0; v < v1; v++) {
      const int d = std::min<int64_t>(1 + poisson(r, mean_degree - 1.0), E);
      rowptr_n[v + 1] = d;
      s += d;
    }
    chunk_nnz[c + 1] = s;
  });
  rowptr_n[0] = 0;
  int64_t total = 0;
  for (int c = 0; c < kChunks; c++) total += chunk_nnz[c + 1];
  if (total >= INT32_MAX) return HGX_EUNSUP;
  for (int32_t v = 0; v < N; v++) rowptr_n[v + 1] += rowptr_n[v];
  *nnz = total;
  if (!col_n) return HGX_OK;
  if (!E_out) return HGX_EINVAL;
  const Alias table(E, exponent);
  std::vector<uint8_t> used(E, 0);
  parallel_chunks(kChunks, [&](int c) {
    Stream r(seed, 2 * (uint64_t)c + 1);
    const int32_t v0 = std::min(N, c * per), v1 = std::min(N, v0 + per);
    for (int32_t v = v0; v < v1; v++) {
      int32_t *p = col_n + rowptr_n[v];
      const int d = rowptr_n[v + 1] - rowptr_n[v];
      for (int i = 0; i < d; i++) p[i] = table.draw(r);
      for (;;) {  // distinct edges per node: redraw duplicates
        std::sort(p, p + d);
        bool dup = false;
        for (int i = 1; i < d; i++)
          if (p[i] == p[i - 1]) {
            p[i] = table.draw(r);
            dup = true;
          }
        if (!dup) break;
      }
    }
  });
  for (int64_t i = 0; i < total; i++) used[col_n[i]] = 1;
  std::vector<int32_t> remap(E);
  int32_t k = 0;
  for (int32_t e = 0; e < E; e++) remap[e] = used[e] ? k++ : -1;
  *E_out = k;
  if (k != E)
    parallel_chunks(kChunks, [&](int c) {
      const int64_t i0 = total * c / kChunks, i1 = total * (c + 1) / kChunks;
      for (int64_t i = i0; i < i1; i++) col_n[i] = remap[col_n[i]];
    });
  return HGX_OK;
}

extern "C" int hgx_csr_transpose(int32_t nrow, int32_t ncol,
                                 const int32_t *rowptr, const int32_t *col,
                                 int32_t *rowptr_t, int32_t *col_t) {
  if (nrow < 0 || ncol < 0 || !rowptr || !rowptr_t) return HGX_EINVAL;
  const int64_t nnz = rowptr[nrow];
  std::fill(rowptr_t, rowptr_t + ncol + 1, 0);
  for (int64_t i = 0; i < nnz; i++) {
    if (col[i] < 0 || col[i] >= ncol) return HGX_EINVAL;
    rowptr_t[col[i] + 1]++;
  }
  for (int32_t c = 0; c < ncol; c++) rowptr_t[c + 1] += rowptr_t[c];
  std::vector<int32_t> fill(rowptr_t, rowptr_t + ncol);
  // rows visited in order: each transposed row comes out sorted
  for (int32_t r = 0; r < nrow; r++)
    for (int32_t t = rowptr[r]; t < rowptr[r + 1]; t++) col_t[fill[col[t]]++] = r;
  return HGX_OK;
}
