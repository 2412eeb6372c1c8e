// Native hypergraph.proto wire-format reader and HypergraphEmbedding writer
// (SURVEY.md §8f rank 1). Host code only.
//
// Reader: a serialized `Hypergraph` (hypergraph.proto:6-23) goes straight to
// the compressed incidence that Incidence.from_hypergraph builds from the
// parsed message. That is CompressRange (hypergraph_util.py:223-244:
// sorted keys -> 0..n-1) over the union of every node's `edges` list
// (Relabel, hypergraph_util.py:208-212), with duplicates dropped, plus the
// float weights (default 1). Map semantics follow protobuf: a repeated key
// keeps its last entry; `edges` may be packed or not; unknown fields are
// skipped. Python protobuf needs minutes for the 2e8-incidence C4 graph and
// refuses messages over 2 GiB. This needs one pass and a sort.
//
// Writer: a `HypergraphEmbedding` (hypergraph.proto:26-35) from the device
// tables, keyed by the original ids, entries in ascending key order.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "hgx.h"

namespace {

thread_local std::string g_host_err;

int host_fail(int code, const std::string &msg) {
  g_host_err = msg;
  return code;
}

struct Reader {
  const uint8_t *p, *end;
  bool ok = true;
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64 && p < end; s += 7) {
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  uint32_t fixed32() {
    if (end - p < 4) {
      ok = false;
      return 0;
    }
    uint32_t v;
    memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  // returns the sub-range of a length-delimited field
  Reader sub() {
    const uint64_t n = varint();
    Reader r{p, p};
    if (!ok || n > (uint64_t)(end - p)) {
      ok = false;
      return r;
    }
    r.end = p + n;
    p += n;
    return r;
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1:
        if (end - p < 8) ok = false;
        else p += 8;
        break;
      case 2: sub(); break;
      case 5: fixed32(); break;
      default: ok = false;
    }
  }
};

constexpr int kChunksP = 64;

template <class F>
void run_chunks(int n, F fn) {
  const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++)
    th.emplace_back([&, t] {
      for (int c = t; c < n; c += nt) fn(c);
    });
  for (auto &x : th) x.join();
}

struct NodeRec {
  int32_t key;
  float weight;
  int64_t off;  // into the edge-id pool
  int32_t cnt;
};

}  // namespace

struct hgx_hg {
  int32_t N = 0, E = 0;
  int64_t nnz = 0;
  std::vector<int32_t> rp_n, col_n;
  std::vector<int64_t> node_ids, edge_ids;
  std::vector<float> node_w, edge_w;
};

extern "C" const char *hgx_host_last_error(void) { return g_host_err.c_str(); }

extern "C" int hgx_proto_parse_hypergraph(const uint8_t *buf, int64_t len,
                                          hgx_hg **out, int32_t *N, int32_t *E,
                                          int64_t *nnz) {
  if (!out || (len > 0 && !buf) || len < 0)
    return host_fail(HGX_EINVAL, "null buffer or handle");
  *out = nullptr;
  std::vector<NodeRec> nodes;
  std::vector<int32_t> pool;
  std::vector<std::pair<int32_t, float>> edges;  // (key, weight)
  Reader r{buf, buf + len};
  while (r.ok && r.p < r.end) {
    const uint64_t tag = r.varint();
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if ((field == 1 || field == 2) && wt == 2) {
      Reader e = r.sub();
      int32_t key = 0;
      float weight = 1.0f;
      const int64_t off = (int64_t)pool.size();
      while (e.ok && e.p < e.end) {
        const uint64_t t = e.varint();
        const int f = (int)(t >> 3), w = (int)(t & 7);
        if (f == 1 && w == 0) {
          key = (int32_t)e.varint();
        } else if (f == 2 && w == 2) {  // NodeData / EdgeData
          Reader v = e.sub();  // a repeated value field merges into the first
          while (v.ok && v.p < v.end) {
            const uint64_t tv = v.varint();
            const int fv = (int)(tv >> 3), wv = (int)(tv & 7);
            if (fv == 1 && wv == 0) {
              const int32_t x = (int32_t)v.varint();
              if (field == 1) pool.push_back(x);
            } else if (fv == 1 && wv == 2) {  // packed
              Reader pk = v.sub();
              while (pk.ok && pk.p < pk.end) {
                const int32_t x = (int32_t)pk.varint();
                if (field == 1) pool.push_back(x);
              }
              if (!pk.ok) v.ok = false;
            } else if (fv == 3 && wv == 5) {
              const uint32_t bits = v.fixed32();
              memcpy(&weight, &bits, 4);
            } else {
              v.skip(wv);
            }
          }
          if (!v.ok) e.ok = false;
        } else {
          e.skip(w);
        }
      }
      if (!e.ok) r.ok = false;
      if (field == 1)
        nodes.push_back({key, weight, off, (int32_t)((int64_t)pool.size() - off)});
      else
        edges.push_back({key, weight});
    } else {
      r.skip(wt);
    }
  }
  if (!r.ok) return host_fail(HGX_EINVAL, "malformed Hypergraph message");

  // last entry per key wins (protobuf map semantics); order by key. Files
  // written in key order (the common case) skip the sort.
  auto keep_last = [](auto &v, auto key_of) {
    bool sorted = true;
    for (size_t i = 1; i < v.size() && sorted; i++)
      sorted = key_of(v[i - 1]) < key_of(v[i]);
    if (sorted) return;
    std::vector<size_t> idx(v.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
      return key_of(v[a]) < key_of(v[b]);
    });
    std::vector<typename std::decay<decltype(v)>::type::value_type> outv;
    outv.reserve(idx.size());
    for (size_t i = 0; i < idx.size(); i++) {
      if (i + 1 < idx.size() && key_of(v[idx[i]]) == key_of(v[idx[i + 1]])) continue;
      outv.push_back(v[idx[i]]);
    }
    v.swap(outv);
  };
  keep_last(nodes, [](const NodeRec &n) { return n.key; });
  keep_last(edges, [](const std::pair<int32_t, float> &e) { return e.first; });

  auto *h = new hgx_hg();
  h->N = (int32_t)nodes.size();
  h->E = (int32_t)edges.size();
  h->node_ids.resize(h->N);
  h->node_w.resize(h->N);
  h->edge_ids.resize(h->E);
  h->edge_w.resize(h->E);
  std::vector<int32_t> ekeys(h->E);
  for (int32_t i = 0; i < h->E; i++) {
    ekeys[i] = edges[i].first;
    h->edge_ids[i] = edges[i].first;
    h->edge_w[i] = edges[i].second;
  }
  // edge key -> compressed index: a direct table when the keys are dense
  // enough, else binary search over the sorted keys
  const int64_t kmin = h->E ? ekeys.front() : 0, kmax = h->E ? ekeys.back() : -1;
  const bool dense = h->E && kmax - kmin < 8ll * h->E + 1024;
  std::vector<int32_t> table;
  if (dense) {
    table.assign((size_t)(kmax - kmin + 1), -1);
    for (int32_t i = 0; i < h->E; i++) table[(size_t)(ekeys[i] - kmin)] = i;
  }
  auto lookup = [&](int32_t key) -> int32_t {
    if (dense) return (key < kmin || key > kmax) ? -1 : table[(size_t)(key - kmin)];
    auto it = std::lower_bound(ekeys.begin(), ekeys.end(), key);
    return (it == ekeys.end() || *it != key) ? -1 : (int32_t)(it - ekeys.begin());
  };
  // per node: map, sort, dedupe in place in the pool (node chunks on
  // threads), then one prefix and a copy
  std::vector<int32_t> cnt((size_t)h->N);
  std::vector<int64_t> bad(kChunksP, -1);
  const int32_t per = (h->N + kChunksP - 1) / kChunksP;
  run_chunks(kChunksP, [&](int c) {
    const int32_t v0 = std::min(h->N, c * per), v1 = std::min(h->N, v0 + per);
    for (int32_t i = v0; i < v1; i++) {
      const NodeRec &n = nodes[i];
      int32_t *row = pool.data() + n.off;
      for (int32_t t = 0; t < n.cnt; t++) {
        const int32_t x = lookup(row[t]);
        if (x < 0) {
          bad[c] = ((int64_t)n.key << 32) | (uint32_t)row[t];
          return;
        }
        row[t] = x;
      }
      std::sort(row, row + n.cnt);
      cnt[i] = (int32_t)(std::unique(row, row + n.cnt) - row);
    }
  });
  for (int64_t x : bad)
    if (x != -1) {
      delete h;
      return host_fail(HGX_EINVAL, "node " + std::to_string((int32_t)(x >> 32)) +
                                       " lists edge " + std::to_string((int32_t)x) +
                                       " missing from hypergraph.edge");
    }
  h->rp_n.assign((size_t)h->N + 1, 0);
  int64_t run = 0;
  for (int32_t i = 0; i < h->N; i++) {
    h->node_ids[i] = nodes[i].key;
    h->node_w[i] = nodes[i].weight;
    run += cnt[i];
    if (run >= INT32_MAX) {
      delete h;
      return host_fail(HGX_EUNSUP, "incidence count exceeds int32 CSR range");
    }
    h->rp_n[i + 1] = (int32_t)run;
  }
  h->col_n.resize((size_t)run);
  run_chunks(kChunksP, [&](int c) {
    const int32_t v0 = std::min(h->N, c * per), v1 = std::min(h->N, v0 + per);
    for (int32_t i = v0; i < v1; i++)
      std::copy(pool.data() + nodes[i].off, pool.data() + nodes[i].off + cnt[i],
                h->col_n.data() + h->rp_n[i]);
  });
  h->nnz = (int64_t)h->col_n.size();
  *out = h;
  if (N) *N = h->N;
  if (E) *E = h->E;
  if (nnz) *nnz = h->nnz;
  return HGX_OK;
}

extern "C" int hgx_proto_hypergraph_fill(const hgx_hg *h, int32_t *rowptr_n,
                                         int32_t *col_n, int64_t *node_ids,
                                         int64_t *edge_ids, float *node_weight,
                                         float *edge_weight) {
  if (!h) return host_fail(HGX_EINVAL, "null hypergraph handle");
  if (rowptr_n) std::copy(h->rp_n.begin(), h->rp_n.end(), rowptr_n);
  if (col_n) std::copy(h->col_n.begin(), h->col_n.end(), col_n);
  if (node_ids) std::copy(h->node_ids.begin(), h->node_ids.end(), node_ids);
  if (edge_ids) std::copy(h->edge_ids.begin(), h->edge_ids.end(), edge_ids);
  if (node_weight) std::copy(h->node_w.begin(), h->node_w.end(), node_weight);
  if (edge_weight) std::copy(h->edge_w.begin(), h->edge_w.end(), edge_weight);
  return HGX_OK;
}

extern "C" void hgx_proto_hypergraph_free(hgx_hg *h) { delete h; }

namespace {

size_t varint_len(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}
uint8_t *put_varint(uint8_t *p, uint64_t v) {
  while (v >= 0x80) {
    *p++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *p++ = (uint8_t)v;
  return p;
}
// int32 keys are varint-encoded as sign-extended 64-bit
uint64_t key_bits(int64_t k) { return (uint64_t)(int64_t)(int32_t)k; }

// one map<int32, Embedding> entry: key (field 1), value (field 2) =
// Embedding{ repeated float values = 1 } unpacked (proto2 default)
size_t entry_body_len(int64_t key, int d) {
  const size_t emb = (size_t)d * 5;  // tag 0x0d + fixed32 per value
  return 1 + varint_len(key_bits(key)) + 1 + varint_len(emb) + emb;
}

uint8_t *put_entry(uint8_t *p, int field, int64_t key, const float *v, int d) {
  const size_t body = entry_body_len(key, d);
  p = put_varint(p, (uint64_t)(field << 3 | 2));
  p = put_varint(p, body);
  *p++ = 0x08;  // key, varint
  p = put_varint(p, key_bits(key));
  *p++ = 0x12;  // value, length-delimited
  p = put_varint(p, (size_t)d * 5);
  for (int i = 0; i < d; i++) {
    *p++ = 0x0d;
    memcpy(p, v + i, 4);
    p += 4;
  }
  return p;
}

}  // namespace

extern "C" int hgx_proto_write_embedding(
    int64_t n_nodes, const int64_t *node_ids, const float *node_tab,
    int64_t n_edges, const int64_t *edge_ids, const float *edge_tab, int d,
    const char *method_name, uint8_t *out, int64_t cap, int64_t *len) {
  if (!len || d < 0 || n_nodes < 0 || n_edges < 0)
    return host_fail(HGX_EINVAL, "bad embedding arguments");
  if ((n_nodes && (!node_ids || !node_tab)) || (n_edges && (!edge_ids || !edge_tab)))
    return host_fail(HGX_EINVAL, "null id or table buffer");
  // ids in ascending order (deterministic serialisation)
  auto order = [](int64_t n, const int64_t *ids) {
    std::vector<int64_t> o(n);
    for (int64_t i = 0; i < n; i++) o[i] = i;
    std::sort(o.begin(), o.end(), [&](int64_t a, int64_t b) { return ids[a] < ids[b]; });
    return o;
  };
  const std::vector<int64_t> on = order(n_nodes, node_ids), oe = order(n_edges, edge_ids);
  size_t total = 0;
  for (int64_t i = 0; i < n_nodes; i++) {
    const size_t b = entry_body_len(node_ids[i], d);
    total += 1 + varint_len(b) + b;
  }
  for (int64_t i = 0; i < n_edges; i++) {
    const size_t b = entry_body_len(edge_ids[i], d);
    total += 1 + varint_len(b) + b;
  }
  total += 1 + varint_len(key_bits(d));
  const size_t mlen = method_name ? strlen(method_name) : 0;
  if (method_name) total += 1 + varint_len(mlen) + mlen;
  *len = (int64_t)total;
  if (!out) return HGX_OK;
  if (cap < (int64_t)total) return host_fail(HGX_EINVAL, "output buffer too small");
  uint8_t *p = out;
  for (int64_t j : on) p = put_entry(p, 1, node_ids[j], node_tab + (size_t)j * d, d);
  for (int64_t j : oe) p = put_entry(p, 2, edge_ids[j], edge_tab + (size_t)j * d, d);
  *p++ = 0x18;  // dim
  p = put_varint(p, key_bits(d));
  if (method_name) {
    *p++ = 0x22;  // method_name
    p = put_varint(p, mlen);
    memcpy(p, method_name, mlen);
    p += mlen;
  }
  return (size_t)(p - out) == total ? HGX_OK
                                    : host_fail(HGX_EINVAL, "internal size mismatch");
}

// Hypergraph writer (bench / test data): node map entries {key, NodeData{
// edges}} then edge map entries {key, EdgeData{nodes}}, repeated int32
// unpacked (proto2's default, what Python protobuf writes), keys ascending
// in the given id order, weights left at their default.
namespace {
size_t list_len(const int32_t *ids, const int64_t *map, int64_t n) {
  size_t b = 0;
  for (int64_t i = 0; i < n; i++) b += 1 + varint_len(key_bits(map[ids[i]]));
  return b;
}
uint8_t *put_list_entry(uint8_t *p, int field, int64_t key, const int32_t *ids,
                        const int64_t *map, int64_t n) {
  const size_t inner = list_len(ids, map, n);
  const size_t body = 1 + varint_len(key_bits(key)) + 1 + varint_len(inner) + inner;
  p = put_varint(p, (uint64_t)(field << 3 | 2));
  p = put_varint(p, body);
  *p++ = 0x08;
  p = put_varint(p, key_bits(key));
  *p++ = 0x12;
  p = put_varint(p, inner);
  for (int64_t i = 0; i < n; i++) {
    *p++ = 0x08;
    p = put_varint(p, key_bits(map[ids[i]]));
  }
  return p;
}
size_t list_entry_len(int64_t key, const int32_t *ids, const int64_t *map, int64_t n) {
  const size_t inner = list_len(ids, map, n);
  const size_t body = 1 + varint_len(key_bits(key)) + 1 + varint_len(inner) + inner;
  return 1 + varint_len(body) + body;
}
}  // namespace

extern "C" int hgx_proto_write_hypergraph(
    int32_t N, int32_t E, const int32_t *rp_n, const int32_t *col_n,
    const int32_t *rp_e, const int32_t *col_e, const int64_t *node_ids,
    const int64_t *edge_ids, uint8_t *out, int64_t cap, int64_t *len) {
  if (!len || N < 0 || E < 0 || !rp_n || !col_n || !rp_e || !col_e || !node_ids ||
      !edge_ids)
    return host_fail(HGX_EINVAL, "bad hypergraph arguments");
  size_t total = 0;
  for (int32_t v = 0; v < N; v++)
    total += list_entry_len(node_ids[v], col_n + rp_n[v], edge_ids, rp_n[v + 1] - rp_n[v]);
  for (int32_t e = 0; e < E; e++)
    total += list_entry_len(edge_ids[e], col_e + rp_e[e], node_ids, rp_e[e + 1] - rp_e[e]);
  *len = (int64_t)total;
  if (!out) return HGX_OK;
  if (cap < (int64_t)total) return host_fail(HGX_EINVAL, "output buffer too small");
  uint8_t *p = out;
  for (int32_t v = 0; v < N; v++)
    p = put_list_entry(p, 1, node_ids[v], col_n + rp_n[v], edge_ids, rp_n[v + 1] - rp_n[v]);
  for (int32_t e = 0; e < E; e++)
    p = put_list_entry(p, 2, edge_ids[e], col_e + rp_e[e], node_ids, rp_e[e + 1] - rp_e[e]);
  return (size_t)(p - out) == total ? HGX_OK
                                    : host_fail(HGX_EINVAL, "internal size mismatch");
}

// HypergraphEmbedding reader (hypergraph.proto:26-35): the merged message of
// one serialized buffer -- a single message, or shards concatenated (the
// wire format merges them: map entries union, last key wins, last dim /
// method_name wins). Pass 1 walks the top-level fields (length prefixes
// only); pass 2 decodes the map entries on threads. `values` may be packed
// or unpacked; every entry must carry the same number of values.
namespace {
struct EmbEntry {
  int32_t key;
  int32_t field;  // 1 node, 2 edge
  const uint8_t *p, *end;
};
}  // namespace

struct hgx_emb {
  int64_t width = 0;
  int32_t dim = 0;
  std::string method;
  std::vector<int64_t> node_ids, edge_ids;
  std::vector<float> node_tab, edge_tab;
};

extern "C" int hgx_proto_parse_embedding(const uint8_t *buf, int64_t len,
                                         hgx_emb **out, int64_t *n_nodes,
                                         int64_t *n_edges, int64_t *width,
                                         int32_t *dim) {
  if (!out || (len > 0 && !buf) || len < 0)
    return host_fail(HGX_EINVAL, "null buffer or handle");
  *out = nullptr;
  auto *h = new hgx_emb();
  std::vector<EmbEntry> ents;
  Reader r{buf, buf + len};
  while (r.ok && r.p < r.end) {
    const uint64_t tag = r.varint();
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if ((field == 1 || field == 2) && wt == 2) {
      Reader e = r.sub();
      ents.push_back({0, field, e.p, e.end});
    } else if (field == 3 && wt == 0) {
      h->dim = (int32_t)r.varint();
    } else if (field == 4 && wt == 2) {
      Reader s = r.sub();
      h->method.assign((const char *)s.p, (size_t)(s.end - s.p));
    } else {
      r.skip(wt);
    }
  }
  if (!r.ok) {
    delete h;
    return host_fail(HGX_EINVAL, "malformed HypergraphEmbedding message");
  }
  // pass 2: key and value range of every entry, in parallel
  const int64_t n = (int64_t)ents.size();
  std::vector<int64_t> cnt((size_t)n, -1);
  std::vector<const uint8_t *> vbeg((size_t)n), vend((size_t)n);
  const int64_t per = (n + kChunksP - 1) / kChunksP;
  std::vector<int> badc(kChunksP, 0);
  run_chunks(kChunksP, [&](int c) {
    const int64_t i0 = std::min(n, c * per), i1 = std::min(n, i0 + per);
    for (int64_t i = i0; i < i1; i++) {
      Reader e{ents[i].p, ents[i].end};
      int64_t m = 0;
      const uint8_t *vb = nullptr, *ve = nullptr;
      bool ok = true;
      while (e.ok && e.p < e.end && ok) {
        const uint64_t t = e.varint();
        const int f = (int)(t >> 3), w = (int)(t & 7);
        if (f == 1 && w == 0) {
          ents[i].key = (int32_t)e.varint();
        } else if (f == 2 && w == 2) {  // Embedding{ repeated float values = 1 }
          Reader v = e.sub();
          if (vb) ok = false;  // a split value field: not written by anyone
          vb = v.p;
          ve = v.end;
          while (v.ok && v.p < v.end) {
            const uint64_t tv = v.varint();
            const int fv = (int)(tv >> 3), wv = (int)(tv & 7);
            if (fv == 1 && wv == 5) {
              v.fixed32();
              m++;
            } else if (fv == 1 && wv == 2) {
              Reader q = v.sub();
              if ((q.end - q.p) % 4) ok = false;
              m += (q.end - q.p) / 4;
            } else {
              v.skip(wv);
            }
          }
          if (!v.ok) ok = false;
        } else {
          e.skip(w);
        }
      }
      if (!e.ok || !ok) {
        badc[c] = 1;
        return;
      }
      cnt[i] = m;
      vbeg[i] = vb;
      vend[i] = ve;
    }
  });
  for (int b : badc)
    if (b) {
      delete h;
      return host_fail(HGX_EINVAL, "malformed HypergraphEmbedding entry");
    }
  h->width = n ? cnt[0] : (int64_t)h->dim;
  for (int64_t i = 0; i < n; i++)
    if (cnt[i] != h->width) {
      delete h;
      return host_fail(HGX_EINVAL, "embedding entries of different lengths (" +
                                       std::to_string(cnt[i]) + " vs " +
                                       std::to_string(h->width) + ")");
    }
  // last entry per key wins; ascending keys
  std::vector<int64_t> order((size_t)n);
  for (int64_t i = 0; i < n; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    if (ents[a].field != ents[b].field) return ents[a].field < ents[b].field;
    return ents[a].key < ents[b].key;
  });
  std::vector<int64_t> keep;
  keep.reserve((size_t)n);
  for (int64_t t = 0; t < n; t++) {
    const int64_t i = order[t];
    if (t + 1 < n && ents[order[t + 1]].field == ents[i].field &&
        ents[order[t + 1]].key == ents[i].key)
      continue;
    keep.push_back(i);
  }
  int64_t nn = 0;
  while (nn < (int64_t)keep.size() && ents[keep[nn]].field == 1) nn++;
  const int64_t ne = (int64_t)keep.size() - nn, W = h->width;
  h->node_ids.resize((size_t)nn);
  h->edge_ids.resize((size_t)ne);
  h->node_tab.resize((size_t)(nn * W));
  h->edge_tab.resize((size_t)(ne * W));
  const int64_t nk = (int64_t)keep.size(), perk = (nk + kChunksP - 1) / kChunksP;
  run_chunks(kChunksP, [&](int c) {
    const int64_t t0 = std::min(nk, c * perk), t1 = std::min(nk, t0 + perk);
    for (int64_t t = t0; t < t1; t++) {
      const int64_t i = keep[t];
      const bool isn = t < nn;
      const int64_t row = isn ? t : t - nn;
      (isn ? h->node_ids : h->edge_ids)[row] = ents[i].key;
      float *dst = (isn ? h->node_tab.data() : h->edge_tab.data()) + row * W;
      Reader v{vbeg[i], vend[i]};
      int64_t m = 0;
      while (v.p < v.end && m < W) {
        const uint64_t tv = v.varint();
        const int fv = (int)(tv >> 3), wv = (int)(tv & 7);
        if (fv == 1 && wv == 5) {
          const uint32_t bits = v.fixed32();
          memcpy(dst + m++, &bits, 4);
        } else if (fv == 1 && wv == 2) {
          Reader q = v.sub();
          const int64_t k = (q.end - q.p) / 4;
          memcpy(dst + m, q.p, (size_t)k * 4);
          m += k;
        } else {
          v.skip(wv);
        }
      }
    }
  });
  *out = h;
  if (n_nodes) *n_nodes = nn;
  if (n_edges) *n_edges = ne;
  if (width) *width = W;
  if (dim) *dim = h->dim;
  return HGX_OK;
}

extern "C" int hgx_proto_embedding_fill(const hgx_emb *h, int64_t *node_ids,
                                        float *node_tab, int64_t *edge_ids,
                                        float *edge_tab, char *method_name,
                                        int64_t cap) {
  if (!h) return host_fail(HGX_EINVAL, "null embedding handle");
  if (node_ids) std::copy(h->node_ids.begin(), h->node_ids.end(), node_ids);
  if (edge_ids) std::copy(h->edge_ids.begin(), h->edge_ids.end(), edge_ids);
  if (node_tab) std::copy(h->node_tab.begin(), h->node_tab.end(), node_tab);
  if (edge_tab) std::copy(h->edge_tab.begin(), h->edge_tab.end(), edge_tab);
  if (method_name) {
    if (cap < (int64_t)h->method.size() + 1)
      return host_fail(HGX_EINVAL, "method_name buffer too small");
    memcpy(method_name, h->method.c_str(), h->method.size() + 1);
  }
  return HGX_OK;
}

extern "C" int64_t hgx_proto_embedding_method_len(const hgx_emb *h) {
  return h ? (int64_t)h->method.size() : -1;
}

extern "C" void hgx_proto_embedding_free(hgx_emb *h) { delete h; }
