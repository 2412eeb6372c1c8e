// Host-side (CPU) link-prediction helpers with Python `random` semantics:
// the sample loops of SampleMissingConnections and RemoveRandomConnections
// (evaluation_util.py:84-158) run natively while drawing exactly the numbers
// CPython's `random` module would, so the caller can hand over
// random.getstate(), get the same picks as the reference's Python loop, and
// put the advanced state back with random.setstate().
//
// CPython's generator (Modules/_randommodule.c, Lib/random.py), restated:
//   MT19937 (624 words + position), genrand_uint32 with the usual tempering;
//   getrandbits(k <= 32) = genrand >> (32 - k);
//   _randbelow(n) = rejection on getrandbits(n.bit_length());
//   random() = ((a >> 5) * 2^26 + (b >> 6)) / 2^53;
//   shuffle(x): for i = len-1 .. 1: j = _randbelow(i + 1); swap(x[i], x[j]).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <unordered_set>
#include <vector>

#include "hgx.h"

namespace {

thread_local char g_err[256];
int fail(int code, const char *msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

struct PyMT {
  uint32_t mt[624];
  int pos;
  void load(const uint32_t *s) {
    memcpy(mt, s, sizeof(mt));
    pos = (int)s[624];
  }
  void store(uint32_t *s) const {
    memcpy(s, mt, sizeof(mt));
    s[624] = (uint32_t)pos;
  }
  uint32_t next() {
    if (pos >= 624) {
      static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
      int kk = 0;
      uint32_t y;
      for (; kk < 624 - 397; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; kk++) {
        y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
      pos = 0;
    }
    uint32_t y = mt[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // _randbelow(n), 1 <= n < 2^32
  uint32_t below(uint64_t n) {
    int k = 0;
    while ((n >> k) != 0) k++;  // n.bit_length()
    uint32_t r = next() >> (32 - k);
    while (r >= n) r = next() >> (32 - k);
    return r;
  }
  double random() {
    const uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
};

}  // namespace

extern "C" {

const char *hgx_lp_last_error(void) { return g_err; }

int hgx_pyrandom_sample_missing(uint32_t *state, int32_t n_nodes, int32_t n_edges,
                                const int64_t *rowptr, const int32_t *col,
                                int64_t num_samples, int32_t *node_pos,
                                int32_t *edge_pos, int64_t *n_out) {
  if (!state || !rowptr || !n_out || (num_samples > 0 && (!node_pos || !edge_pos)))
    return fail(HGX_EINVAL, "null argument");
  if (n_nodes <= 0 || n_edges <= 0)
    return fail(HGX_EINVAL, "hypergraph needs nodes and edges");
  if ((double)num_samples >= (double)n_nodes * (double)n_edges || num_samples < 0)
    return fail(HGX_EINVAL, "num_samples < num_nodes * num_edges");
  PyMT g;
  g.load(state);
  std::unordered_set<uint64_t> seen;
  seen.reserve((size_t)num_samples * 2 + 16);
  int64_t got = 0, tries = 10 * num_samples;
  while (got < num_samples && tries) {
    tries--;
    const uint32_t p = g.below((uint64_t)n_nodes);  // random.choice(nodes)
    const uint32_t q = g.below((uint64_t)n_edges);  // random.choice(edges)
    // `edge_idx not in hypergraph.node[node_idx].edges`: sorted positions
    const int32_t *b = col + rowptr[p], *e = col + rowptr[p + 1];
    const int32_t *it = std::lower_bound(b, e, (int32_t)q);
    if (it != e && *it == (int32_t)q) continue;
    if (seen.insert(((uint64_t)p << 32) | q).second) {
      node_pos[got] = (int32_t)p;
      edge_pos[got] = (int32_t)q;
      got++;
    }
  }
  g.store(state);
  *n_out = got;
  return HGX_OK;
}

int hgx_pyrandom_remove_connections(uint32_t *state, int64_t n_pairs,
                                    const int32_t *pair_node,
                                    const int32_t *pair_edge, int32_t *node_deg,
                                    int32_t *edge_size, double probability,
                                    int64_t *removed, int64_t *n_removed) {
  if (!state || !n_removed || (n_pairs > 0 && (!pair_node || !pair_edge || !node_deg ||
                                               !edge_size || !removed)))
    return fail(HGX_EINVAL, "null argument");
  if (!(probability >= 0.0 && probability <= 1.0))
    return fail(HGX_EINVAL, "0 <= probability <= 1");
  PyMT g;
  g.load(state);
  std::vector<int64_t> order((size_t)n_pairs);
  for (int64_t i = 0; i < n_pairs; i++) order[i] = i;
  for (int64_t i = n_pairs - 1; i >= 1; i--) {  // random.shuffle(node_edges)
    if ((uint64_t)i + 1 > 0xffffffffull) return fail(HGX_EUNSUP, "more than 2^32 pairs");
    const int64_t j = g.below((uint64_t)i + 1);
    std::swap(order[i], order[j]);
  }
  int64_t nr = 0;
  for (int64_t t = 0; t < n_pairs; t++) {
    const int64_t i = order[t];
    const int32_t p = pair_node[i], q = pair_edge[i];
    if (node_deg[p] == 1) continue;   // the node's last connection
    if (edge_size[q] == 1) continue;  // the edge's last connection
    if (g.random() < probability && probability > 0) {
      node_deg[p]--;
      edge_size[q]--;
      removed[nr++] = i;
    }
  }
  g.store(state);
  *n_removed = nr;
  return HGX_OK;
}

}  // extern "C"
