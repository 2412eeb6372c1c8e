// Compact record store: record streams larger than HBM trained with Keras'
// global shuffle. See include/hgx.h (hgx_store_*).
//
// The reference materialises every SimilarityRecord once and calls
// model.fit(..., shuffle=True): every epoch is a fresh uniform permutation
// of the WHOLE stream cut into batches of 256 (embedding.py:277-302). At
// the 10M/5M config the stream is 5.9e9 records, 404 GB in the trainer's
// 68-byte layout (SamplesToModelInput, hg2v_sample.py:751-797). Here every
// record is sampled once and kept as 12 bytes:
//   w0 = kind block << 28 | row      (the row it was sampled from)
//   w1 = column (negatives: rank of the record in its row)
//   w2 = target bits (negatives: 0)
// -- everything else of the record is a function of these (the neighbour
// lists are keyed draws, hgx::draw_record_neighbors; a negative's column
// is the keyed draw of emit_negatives), so hgx_store_load rebuilds the
// sampler's records bit for bit. Packing verifies exactly that.
//
// Epoch order: record r's key is a bijective 64-bit mix of its identity
// (w0, w1) and the epoch seed, so keys are distinct and the order "sorted
// by key" is a pseudo-random permutation of the stream that does not
// depend on where a record sits in the store (one rank or eight ranks
// filling it, any append order: the same epoch). hgx_store_plan cuts the
// key space into chunks of at most `budget` records by a 2^14-bin
// histogram; hgx_store_load selects a chunk's records, sorts them by key
// and writes them as trainer records in that order, so consecutive loads
// walk the epoch's global order. Batches follow the global order too: a
// load keeps the (n mod batch) records of its tail for the next load, so
// every batch but the epoch's last holds exactly `batch` records, as
// Keras cuts them.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <type_traits>
#include <vector>

#include "hgx_internal.h"

namespace {

using hgx::REC_EE;
using hgx::REC_NE_EDGE;
using hgx::REC_NE_NODE;
using hgx::REC_NN;

constexpr int kMaxBlocks = 9;
constexpr int kRowBits = 28;
constexpr uint32_t kRowMask = (1u << kRowBits) - 1;
constexpr int kBinBits = 14;
constexpr int kBins = 1 << kBinBits;  // == HGX_STORE_BINS
static_assert(kBins == HGX_STORE_BINS, "bin count");

// What a stored record's block index means (the sampler's kind blocks)
struct BlockTab {
  int nb;
  int kind[kMaxBlocks];
  // id columns of the row and of the column, the target column, whether
  // row / column index nodes (all from `kind`, precomputed on the host)
  int rpos[kMaxBlocks], cpos[kMaxBlocks], tpos[kMaxBlocks];
  int rnode[kMaxBlocks], cnode[kMaxBlocks];
  int neg[kMaxBlocks];
  int ncols[kMaxBlocks];            // negatives: columns of the draw
  uint32_t col_stream[kMaxBlocks];  // negatives: emit_negatives stream
  uint32_t nbr_stream[kMaxBlocks];  // node-edge blocks: draw_neighbors stream
  int64_t bound[kMaxBlocks + 1];    // hgx_store_append: record block bounds
};

// the samplers' block layouts (hgx_sample.hip: hgx_sample_fobe,
// hgx_sample_hobe_rows; streams as they pass them)
void block_table(const hgx_ctx *ctx, int family, BlockTab &t) {
  memset(&t, 0, sizeof(t));
  auto set = [&](int b, int kind, int neg, int ncols, uint32_t cs, uint32_t ns) {
    static const int rp[4] = {0, 1, 0, 3}, cp[4] = {2, 3, 3, 0}, tp[4] = {0, 1, 2, 2};
    static const int rn[4] = {1, 0, 1, 0}, cn[4] = {1, 0, 0, 1};
    t.kind[b] = kind;
    t.rpos[b] = rp[kind];
    t.cpos[b] = cp[kind];
    t.tpos[b] = tp[kind];
    t.rnode[b] = rn[kind];
    t.cnode[b] = cn[kind];
    t.neg[b] = neg;
    t.ncols[b] = ncols;
    t.col_stream[b] = cs;
    t.nbr_stream[b] = ns;
  };
  if (family == 0) {  // BooleanSamples (hg2v_sample.py:156-240)
    t.nb = 9;
    set(0, REC_NN, 0, 0, 0, 0);
    set(1, REC_EE, 0, 0, 0, 0);
    set(2, REC_NE_NODE, 0, 0, 0, 0x200);
    set(3, REC_NE_EDGE, 0, 0, 0, 0x201);
    set(4, REC_NN, 1, ctx->N, 0x300, 0);
    set(5, REC_EE, 1, ctx->E, 0x301, 0);
    set(6, REC_EE, 1, ctx->E, 0x302, 0);
    set(7, REC_NE_NODE, 1, ctx->E, 0x303, 0x400);
    set(8, REC_NE_EDGE, 1, ctx->N, 0x304, 0x401);
  } else {  // AlgebraicDistanceSamples (hg2v_sample.py:658-715)
    t.nb = 4;
    set(0, REC_NN, 0, 0, 0, 0);
    set(1, REC_EE, 0, 0, 0, 0);
    set(2, REC_NE_NODE, 0, 0, 0, 0x500);
    set(3, REC_NE_EDGE, 0, 0, 0, 0x501);
  }
}

struct Csr4 {
  const int *rp_n, *col_n, *rp_e, *col_e;
  int N, E;
};

// The trainer record of stored entry (w0, w1, w2): ids (+1 shifted, 0 =
// absent) at id positions [0, 4 + 2K), targets [0, 3). CHECK = false:
// written to ri / tg; CHECK = true: compared with the record at ri / tg
// (hgx_store_append's lossless check): diff gets 4 (ids), 8 (targets), 16
// (neighbours) for a difference. Returns false for an entry naming rows
// outside the graph or a node-edge endpoint without neighbours (the
// sampler refuses those): nothing is then read from the incidence.
template <bool CHECK, typename IdPtr = std::conditional_t<CHECK, const int *, int *>,
          typename TgPtr = std::conditional_t<CHECK, const float *, float *>>
__device__ __forceinline__ bool expand_one(uint32_t w0, uint32_t w1, uint32_t w2,
                                           const BlockTab &t, int K, uint64_t seed,
                                           const Csr4 &g, IdPtr ri, TgPtr tg,
                                           int &diff) {
  const int b = (int)(w0 >> kRowBits);
  if (b >= t.nb) return false;
  const int row = (int)(w0 & kRowMask);
  const int neg = t.neg[b], rpos = t.rpos[b], cpos = t.cpos[b], tpos = t.tpos[b];
  const int rnode = t.rnode[b], cnode = t.cnode[b];
  const int col = neg ? (int)hgx::bounded(  // emit_negatives' keyed column
                            hgx::rand64(seed, t.col_stream[b],
                                        ((uint64_t)row << 32) | w1),
                            (uint32_t)t.ncols[b])
                      : (int)w1;
  if (row >= (rnode ? g.N : g.E) || col < 0 || col >= (cnode ? g.N : g.E))
    return false;
  const int R = 4 + 2 * K;
  const bool ne = t.kind[b] >= REC_NE_NODE;
  for (int s = 0; s < 4; s++) {
    const int want = s == rpos ? row + 1 : s == cpos ? col + 1 : 0;
    if constexpr (CHECK) {
      if (ri[s] != want) diff |= 4;
    } else {
      ri[s] = want;
    }
  }
  const float p = __uint_as_float(w2);
  for (int s = 0; s < 3; s++) {
    const float want = s == tpos ? p : 0.f;
    if constexpr (CHECK) {
      if (__float_as_uint(tg[s]) != __float_as_uint(want)) diff |= 8;
    } else {
      tg[s] = want;
    }
  }
  if (!ne) {
    for (int s = 4; s < R; s++) {
      if constexpr (CHECK) {
        if (ri[s] != 0) diff |= 16;
      } else {
        ri[s] = 0;
      }
    }
    return true;
  }
  const int v = rnode ? row : col;
  const int e = rnode ? col : row;
  const int nb = g.rp_e[e], nl = g.rp_e[e + 1] - nb;
  const int eb = g.rp_n[v], el = g.rp_n[v + 1] - eb;
  if (nl <= 0 || el <= 0) return false;
  // hgx::draw_record_neighbors, one neighbour at a time
  const uint64_t rk =
      hgx::rand64_key(seed, ((uint64_t)t.nbr_stream[b] << 32) | (uint32_t)row);
  const uint64_t key = neg ? (uint64_t)w1 : (uint64_t)col;
  for (int k = 0; k < K; k++) {
    const uint64_t h = hgx::mix64(rk + key * 64 + k);
    const uint64_t h2 = hgx::mix64(rk + key * 64 + 32 + k);
    const int a = g.col_e[nb + hgx::bounded(h, (uint32_t)nl)] + 1;
    const int c = g.col_n[eb + hgx::bounded(h2, (uint32_t)el)] + 1;
    if constexpr (CHECK) {
      if (ri[4 + k] != a || ri[4 + K + k] != c) diff |= 16;
    } else {
      ri[4 + k] = a;
      ri[4 + K + k] = c;
    }
  }
  return true;
}

// Pack records [0, n) of the sampler's stream (kind blocks t.bound) into
// out[3 * i], checking that each reloads bit for bit. err bits: 1 a record
// does not reload as sampled (4 ids, 8 targets, 16 neighbours differ, 32
// rows outside the graph; 64 << block: the blocks concerned), 2 a row id
// past 2^28.
__global__ void store_pack(const int *idx, const float *tgt, int64_t n, int K,
                           BlockTab t, Csr4 g, uint64_t seed, uint32_t *out,
                           int *err) {
  const int R = 4 + 2 * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int b = 0;
    for (int q = 1; q < t.nb; q++) b += i >= t.bound[q] ? 1 : 0;
    const int *ri = idx + i * R;
    const int rpos = t.rpos[b], cpos = t.cpos[b];
    const int row = ri[rpos] - 1, col = ri[cpos] - 1;
    const float p = tgt[i * 3 + t.tpos[b]];
    int bad = row < 0 || (uint32_t)row > kRowMask ? 2 : 0;
    uint32_t w1 = (uint32_t)col;
    if (t.neg[b] && !bad) {
      // rank in the row: a block's records are grouped by row, rows
      // ascending (galloping back to the row's first record, then bisection)
      const int64_t b0 = t.bound[b];
      int64_t good = i, step = 1, lo = b0 - 1;
      while (good - step >= b0) {
        if (idx[(good - step) * R + rpos] - 1 != row) {
          lo = good - step;
          break;
        }
        good -= step;
        step <<= 1;
      }
      while (good - lo > 1) {
        const int64_t mid = lo + (good - lo) / 2;
        if (idx[mid * R + rpos] - 1 == row) good = mid;
        else lo = mid;
      }
      w1 = (uint32_t)(i - good);
    }
    const uint32_t w0 = ((uint32_t)b << kRowBits) | ((uint32_t)row & kRowMask);
    const uint32_t w2 = __float_as_uint(p);
    if (!bad) {
      int diff = 0;
      const bool ok = expand_one<true>(w0, w1, w2, t, K, seed, g, ri, tgt + i * 3, diff);
      if (!ok) diff |= 32;
      if (diff) {
        bad = 1 | diff | (64 << b);
        // the first mismatching record, for the error message
        if (atomicCAS(err + 1, 0, 1) == 0) {
          err[2] = (int)i;
          err[3] = b;
          err[4] = row;
          err[5] = col;
        }
      }
    }
    uint32_t *o = out + 3 * i;
    o[0] = w0;
    o[1] = w1;
    o[2] = w2;
    if (bad) atomicOr(err, bad);
  }
}

// epoch key of a stored record: bijective in its identity (w0, w1)
__device__ __forceinline__ uint64_t epoch_key(uint32_t w0, uint32_t w1, uint64_t k1,
                                              uint64_t k2) {
  const uint64_t id = ((uint64_t)w0 << 32) | w1;
  return hgx::mix64(hgx::mix64(id ^ k1) ^ k2);
}

__global__ void store_hist(const uint32_t *st, int64_t n, uint64_t k1, uint64_t k2,
                           unsigned *hist) {
  __shared__ unsigned h[kBins];
  for (int i = threadIdx.x; i < kBins; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = epoch_key(st[3 * i], st[3 * i + 1], k1, k2);
    atomicAdd(&h[key >> (64 - kBinBits)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kBins; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// Records whose key lies in bins [lo, hi): copied to sel (their keys to
// keys, their positions in sel to vals). Tiles of 256 x kSelItems entries
// (item j of thread t at tile + j * 256 + t, coalesced), one atomic per
// tile for the tile's base: a per-wave atomic on the one counter serialised
// the selection (223 ms for 2^28 of 1.2e9 entries vs 2.6 ms for the
// histogram pass over the same store). Where a record lands in sel depends
// on the tiles' atomic order; the load's order does not: the keys are
// distinct and sorted.
constexpr int kSelItems = 8;
__global__ __launch_bounds__(256) void store_select(
    const uint32_t *st, int64_t n, uint64_t k1, uint64_t k2, uint32_t lo, uint32_t hi,
    uint32_t *sel, unsigned long long *keys, int *vals, unsigned long long *count) {
  __shared__ unsigned wave_off[4];
  __shared__ unsigned long long tile_base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1;
  const int64_t tile = 256 * kSelItems;
  for (int64_t t0 = blockIdx.x * tile; t0 < n; t0 += (int64_t)gridDim.x * tile) {
    uint32_t w0[kSelItems], w1[kSelItems], w2[kSelItems];
    uint64_t key[kSelItems];
    unsigned long long mask[kSelItems];
    unsigned wtot = 0;
#pragma unroll
    for (int j = 0; j < kSelItems; j++) {
      const int64_t i = t0 + j * 256 + threadIdx.x;
      bool take = false;
      w0[j] = w1[j] = w2[j] = 0;
      key[j] = 0;
      if (i < n) {
        w0[j] = st[3 * i];
        w1[j] = st[3 * i + 1];
        w2[j] = st[3 * i + 2];
        key[j] = epoch_key(w0[j], w1[j], k1, k2);
        const uint32_t bin = (uint32_t)(key[j] >> (64 - kBinBits));
        take = bin >= lo && bin < hi;
      }
      mask[j] = __ballot(take);
      wtot += (unsigned)__popcll(mask[j]);
    }
    if (lane == 0) wave_off[wave] = wtot;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned run = 0;
      for (int w = 0; w < 4; w++) {
        const unsigned c = wave_off[w];
        wave_off[w] = run;
        run += c;
      }
      tile_base = run ? atomicAdd(count, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    int64_t base = (int64_t)tile_base + wave_off[wave];
#pragma unroll
    for (int j = 0; j < kSelItems; j++) {
      if ((mask[j] >> lane) & 1ull) {
        const int64_t pos = base + __popcll(mask[j] & below);
        uint32_t *o = sel + 3 * pos;
        o[0] = w0[j];
        o[1] = w1[j];
        o[2] = w2[j];
        keys[pos] = key[j];
        vals[pos] = (int)pos;
      }
      base += __popcll(mask[j]);
    }
    __syncthreads();  // wave_off / tile_base reused by the next tile
  }
}

// trainer records [off, off + m) from the selected entries in key order
__global__ void store_expand(const uint32_t *sel, const int *order, int64_t m,
                             int64_t off, BlockTab t, int K, uint64_t seed, Csr4 g,
                             int *idx, float *tgt, int *err) {
  const int R = 4 + 2 * K;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t *c = sel + 3 * (int64_t)order[i];
    int diff = 0;
    if (!expand_one<false>(c[0], c[1], c[2], t, K, seed, g, idx + (off + i) * R,
                           tgt + (off + i) * 3, diff))
      atomicOr(err, 1);
  }
}

int grid_for(int64_t work, int per_block, int cap = 8192) {
  int64_t gr = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(gr, cap));
}

Csr4 csr_of(const hgx_ctx *ctx) {
  return Csr4{ctx->rp_n.as<int>(), ctx->col_n.as<int>(), ctx->rp_e.as<int>(),
              ctx->col_e.as<int>(), ctx->N, ctx->E};
}

// the store's capacity grown to `cap` records, keeping its contents
int store_grow(hgx_ctx *ctx, int64_t cap) {
  if (cap <= ctx->cap_store && ctx->store.p) return HGX_OK;
  DevBuf nb;
  HGX_TRY(hgx_ensure(ctx, nb, sizeof(uint32_t) * 3 * (size_t)std::max<int64_t>(cap, 1)));
  if (ctx->n_store > 0)
    HGX_HIP(ctx, hipMemcpyAsync(nb.p, ctx->store.p, sizeof(uint32_t) * 3 * ctx->n_store,
                                hipMemcpyDeviceToDevice, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  hgx_release(ctx->store);
  ctx->store = nb;
  ctx->cap_store = cap;
  return HGX_OK;
}

void epoch_keys(uint64_t epoch_seed, uint64_t &k1, uint64_t &k2) {
  k1 = hgx::mix64(epoch_seed ^ 0x53544f52454b3130ull);
  k2 = hgx::mix64(epoch_seed ^ 0x53544f52454b3230ull);
}

}  // namespace

extern "C" int hgx_store_reset(hgx_ctx *ctx, int64_t capacity) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, capacity >= 0, HGX_EINVAL, "negative store capacity");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  ctx->n_store = 0;
  ctx->store_family = -1;
  ctx->store_K = 0;
  ctx->store_seed = 0;
  ctx->store_carry = 0;
  ctx->st_hist_ok = false;
  if (capacity > ctx->cap_store) {
    hgx_release(ctx->store);  // nothing to keep
    ctx->cap_store = 0;
    HGX_TRY(store_grow(ctx, capacity));
  }
  return HGX_OK;
}

// Frees the store, its load scratch and the record buffers the last load
// filled (at C4: the ~71 GB store, ~19 GB of st_* scratch and a ~36 GB
// chunk), so the device's HBM is back for the next embedding or the
// combiner. The context stays usable: the next reset / append / write grows
// the store again.
extern "C" int hgx_store_release(hgx_ctx *ctx) {
  if (!ctx) return HGX_EINVAL;
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  for (DevBuf *b : {&ctx->store, &ctx->st_sel, &ctx->st_keys, &ctx->st_vals, &ctx->st_tmp,
                    &ctx->st_hist, &ctx->rec_idx, &ctx->rec_tgt})
    hgx_release(*b);
  ctx->cap_store = 0;
  ctx->n_store = 0;
  ctx->store_family = -1;
  ctx->store_K = 0;
  ctx->store_seed = 0;
  ctx->store_carry = 0;
  ctx->st_hist_ok = false;
  ctx->n_rec = 0;
  ctx->smp_family = -1;
  ctx->rec_in_order = false;
  ctx->rec_bounds[0] = ctx->rec_bounds[1] = 0;
  ctx->n_rec_blocks = 1;
  return HGX_OK;
}

// the store's sampler family / K / seed: set by the first records, equal
// for every later one
static int store_adopt(hgx_ctx *ctx, int family, int K, uint64_t seed) {
  if (ctx->n_store == 0) {
    ctx->store_family = family;
    ctx->store_K = K;
    ctx->store_seed = seed;
    BlockTab t;
    block_table(ctx, family, t);
    ctx->store_blocks = t.nb;
    return HGX_OK;
  }
  HGX_CHECK(ctx, ctx->store_family == family && ctx->store_K == K &&
                     ctx->store_seed == seed,
            HGX_EINVAL,
            "records of sampler family %d / K %d / seed %llu do not join a store "
            "of family %d / K %d / seed %llu",
            family, K, (unsigned long long)seed, ctx->store_family, ctx->store_K,
            (unsigned long long)ctx->store_seed);
  return HGX_OK;
}

extern "C" int hgx_store_append(hgx_ctx *ctx) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, ctx->smp_family == 0 || ctx->smp_family == 1, HGX_ESTATE,
            "the records are not a hgx_sample_fobe / hgx_sample_hobe stream");
  HGX_CHECK(ctx, ctx->N <= (int32_t)kRowMask && ctx->E <= (int32_t)kRowMask,
            HGX_EUNSUP, "the record store holds graphs of < 2^28 nodes and edges");
  const int family = ctx->smp_family, K = ctx->K;
  BlockTab t;
  block_table(ctx, family, t);
  const int nb = ctx->n_rec_blocks;
  HGX_CHECK(ctx, (family == 1 && nb == 4) || (family == 0 && (nb == 4 || nb == 9)),
            HGX_ESTATE, "unexpected kind blocks (%d) for sampler family %d", nb,
            family);
  HGX_TRY(store_adopt(ctx, family, K, ctx->smp_seed));
  const int64_t n = ctx->n_rec;
  if (n == 0) return HGX_OK;
  for (int i = 0; i <= kMaxBlocks; i++)
    t.bound[i] = ctx->rec_bounds[std::min(i, nb)];
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->n_store + n > ctx->cap_store)
    HGX_TRY(store_grow(ctx, std::max(ctx->n_store + n, ctx->cap_store + ctx->cap_store / 4)));
  HGX_TRY(hgx_ensure(ctx, ctx->s0, 32));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s0.p, 0, 32, ctx->stream));
  hipLaunchKernelGGL(store_pack, dim3(grid_for(n, 256)), dim3(256), 0, ctx->stream,
                     ctx->rec_idx.as<int>(), ctx->rec_tgt.as<float>(), n, K, t,
                     csr_of(ctx), ctx->store_seed,
                     ctx->store.as<uint32_t>() + 3 * ctx->n_store, ctx->s0.as<int>());
  HGX_LAUNCH_CHECK(ctx);
  int ev[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  HGX_HIP(ctx, hipMemcpyAsync(ev, ctx->s0.p, 32, hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int err = ev[0];
  HGX_CHECK(ctx, !(err & 2), HGX_EUNSUP, "a record row id exceeds 2^28");
  HGX_CHECK(ctx, err == 0, HGX_ESTATE,
            "a sampled record does not reload bit for bit from its stored form "
            "(mismatch bits 0x%x: 4 ids, 8 targets, 16 neighbours, 32 rows; "
            "64 << kind block; first: record %d, block %d, row %d, column %d)",
            err, ev[2], ev[3], ev[4], ev[5]);
  ctx->n_store += n;
  ctx->st_hist_ok = false;
  return HGX_OK;
}

extern "C" int hgx_store_info(hgx_ctx *ctx, int64_t *n, int *family, int *K,
                              uint64_t *seed) {
  if (!ctx) return HGX_EINVAL;
  if (n) *n = ctx->n_store;
  if (family) *family = ctx->store_family;
  if (K) *K = ctx->store_K;
  if (seed) *seed = ctx->store_seed;
  return HGX_OK;
}

extern "C" int hgx_store_read(hgx_ctx *ctx, int64_t start, int64_t n, void *dst,
                              int dst_device) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, start >= 0 && n >= 0 && start + n <= ctx->n_store, HGX_EINVAL,
            "store range [%lld, %lld) outside [0, %lld)", (long long)start,
            (long long)(start + n), (long long)ctx->n_store);
  HGX_CHECK(ctx, n == 0 || dst, HGX_EINVAL, "null destination");
  if (n == 0) return HGX_OK;
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  HGX_HIP(ctx, hipMemcpyAsync(dst, ctx->store.as<uint32_t>() + 3 * start,
                              sizeof(uint32_t) * 3 * n,
                              dst_device ? hipMemcpyDeviceToDevice
                                         : hipMemcpyDeviceToHost,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return HGX_OK;
}

extern "C" int hgx_store_write(hgx_ctx *ctx, int64_t n, const void *src,
                               int src_device, int family, int K, uint64_t seed) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, family == 0 || family == 1, HGX_EINVAL, "family must be 0 or 1");
  HGX_CHECK(ctx, K >= 1 && K <= 16, HGX_EUNSUP, "num_neighbors %d outside [1,16]", K);
  HGX_CHECK(ctx, n >= 0 && (n == 0 || src), HGX_EINVAL, "bad source");
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_TRY(store_adopt(ctx, family, K, seed));
  if (n == 0) return HGX_OK;
  if (!src_device) {  // host records: validate before they reach the device
    const uint32_t *h = static_cast<const uint32_t *>(src);
    BlockTab t;
    block_table(ctx, family, t);
    for (int64_t i = 0; i < n; i++) {
      const int b = (int)(h[3 * i] >> kRowBits);
      const int64_t row = h[3 * i] & kRowMask;
      HGX_CHECK(ctx, b < t.nb, HGX_EINVAL, "record %lld: block %d", (long long)i, b);
      const bool node_row = t.kind[b] == REC_NN || t.kind[b] == REC_NE_NODE;
      HGX_CHECK(ctx, row < (node_row ? ctx->N : ctx->E), HGX_EINVAL,
                "record %lld: row %lld out of range", (long long)i, (long long)row);
      if (!t.neg[b]) {
        const bool node_col = t.kind[b] == REC_NN || t.kind[b] == REC_NE_EDGE;
        HGX_CHECK(ctx, h[3 * i + 1] < (uint32_t)(node_col ? ctx->N : ctx->E),
                  HGX_EINVAL, "record %lld: column out of range", (long long)i);
      }
    }
  }
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  if (ctx->n_store + n > ctx->cap_store)
    HGX_TRY(store_grow(ctx, std::max(ctx->n_store + n, ctx->cap_store + ctx->cap_store / 4)));
  HGX_HIP(ctx, hipMemcpyAsync(ctx->store.as<uint32_t>() + 3 * ctx->n_store, src,
                              sizeof(uint32_t) * 3 * n,
                              src_device ? hipMemcpyDeviceToDevice
                                         : hipMemcpyHostToDevice,
                              ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->n_store += n;
  ctx->st_hist_ok = false;
  return HGX_OK;
}

extern "C" int hgx_store_plan(hgx_ctx *ctx, uint64_t epoch_seed, int64_t budget,
                              int *n_chunks, int32_t *bin_bounds, int64_t *counts) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, budget >= 1, HGX_EINVAL, "budget must be >= 1");
  HGX_CHECK(ctx, n_chunks && bin_bounds && counts, HGX_EINVAL, "null output");
  HGX_CHECK(ctx, ctx->n_store > 0, HGX_ESTATE, "the record store is empty");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  uint64_t k1, k2;
  epoch_keys(epoch_seed, k1, k2);
  HGX_TRY(hgx_ensure(ctx, ctx->st_hist, sizeof(unsigned) * kBins));
  HGX_HIP(ctx, hipMemsetAsync(ctx->st_hist.p, 0, sizeof(unsigned) * kBins, ctx->stream));
  hipLaunchKernelGGL(store_hist, dim3(grid_for(ctx->n_store, 1024, 1024)), dim3(1024),
                     0, ctx->stream, ctx->store.as<uint32_t>(), ctx->n_store, k1, k2,
                     ctx->st_hist.as<unsigned>());
  HGX_LAUNCH_CHECK(ctx);
  std::vector<unsigned> &h = ctx->st_hist_host;
  h.assign(kBins, 0u);
  HGX_HIP(ctx, hipMemcpyAsync(h.data(), ctx->st_hist.p, sizeof(unsigned) * kBins,
                              hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->st_hist_seed = epoch_seed;
  ctx->st_hist_ok = true;
  // greedy: consecutive bins while the chunk stays within budget (a bin
  // larger than the budget is a chunk of its own)
  int nc = 0;
  bin_bounds[0] = 0;
  int64_t cur = 0;
  for (int b = 0; b < kBins; b++) {
    if (cur > 0 && cur + (int64_t)h[b] > budget) {
      counts[nc] = cur;
      bin_bounds[++nc] = b;
      cur = 0;
    }
    cur += h[b];
  }
  counts[nc] = cur;
  bin_bounds[++nc] = kBins;
  int64_t tot = 0;
  for (int c = 0; c < nc; c++) tot += counts[c];
  HGX_CHECK(ctx, tot == ctx->n_store, HGX_EHIP, "store histogram lost records");
  *n_chunks = nc;
  ctx->store_carry = 0;  // a new epoch: no batch tail carried over
  return HGX_OK;
}

extern "C" int hgx_store_load(hgx_ctx *ctx, uint64_t epoch_seed, int32_t bin_lo,
                              int32_t bin_hi, int batch, int last,
                              int64_t *n_records) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, 0 <= bin_lo && bin_lo < bin_hi && bin_hi <= kBins, HGX_EINVAL,
            "bins [%d, %d) outside [0, %d)", bin_lo, bin_hi, kBins);
  HGX_CHECK(ctx, batch >= 1, HGX_EINVAL, "batch must be >= 1");
  HGX_CHECK(ctx, ctx->n_store > 0, HGX_ESTATE, "the record store is empty");
  HGX_CHECK(ctx, ctx->N > 0, HGX_ESTATE, "no incidence uploaded");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int K = ctx->store_K, R = 4 + 2 * K;
  BlockTab t;
  block_table(ctx, ctx->store_family, t);
  uint64_t k1, k2;
  epoch_keys(epoch_seed, k1, k2);
  // 1. the chunk's entries and their keys
  HGX_TRY(hgx_ensure(ctx, ctx->s0, 16));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s0.p, 0, 16, ctx->stream));
  // the chunk's size from the epoch's key histogram (hgx_store_plan's, or
  // computed here for a load without a plan of this epoch)
  if (!ctx->st_hist_ok || ctx->st_hist_seed != epoch_seed) {
    HGX_TRY(hgx_ensure(ctx, ctx->st_hist, sizeof(unsigned) * kBins));
    HGX_HIP(ctx, hipMemsetAsync(ctx->st_hist.p, 0, sizeof(unsigned) * kBins, ctx->stream));
    hipLaunchKernelGGL(store_hist, dim3(grid_for(ctx->n_store, 1024, 1024)), dim3(1024),
                       0, ctx->stream, ctx->store.as<uint32_t>(), ctx->n_store, k1, k2,
                       ctx->st_hist.as<unsigned>());
    HGX_LAUNCH_CHECK(ctx);
    ctx->st_hist_host.assign(kBins, 0u);
    HGX_HIP(ctx, hipMemcpyAsync(ctx->st_hist_host.data(), ctx->st_hist.p,
                                sizeof(unsigned) * kBins, hipMemcpyDeviceToHost,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ctx->st_hist_seed = epoch_seed;
    ctx->st_hist_ok = true;
  }
  const std::vector<unsigned> &h = ctx->st_hist_host;
  int64_t m = 0;
  for (int b = bin_lo; b < bin_hi; b++) m += h[b];
  const int64_t carry = ctx->store_carry;
  HGX_CHECK(ctx, carry + m < (int64_t)INT32_MAX, HGX_EUNSUP,
            "%lld records in one load exceed the trainer's 2^31 limit",
            (long long)(carry + m));
  HGX_TRY(hgx_ensure(ctx, ctx->st_sel, sizeof(uint32_t) * 3 * (size_t)(m + 1)));
  size_t sort_tmp = 0;
  unsigned long long *kin = nullptr, *kout = nullptr;
  int *vin = nullptr, *vout = nullptr;
  HGX_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, kin, kout, vin,
                                                  vout, (int)m, 0, 64, ctx->stream));
  const size_t koff = (sizeof(unsigned long long) * 2 * (size_t)(m + 1) + 255) / 256 * 256;
  HGX_TRY(hgx_ensure(ctx, ctx->st_keys, koff + sort_tmp + 256));
  HGX_TRY(hgx_ensure(ctx, ctx->st_vals, sizeof(int) * 2 * (size_t)(m + 1)));
  kin = ctx->st_keys.as<unsigned long long>();
  kout = kin + (m + 1);
  vin = ctx->st_vals.as<int>();
  vout = vin + (m + 1);
  if (m > 0) {
    hipLaunchKernelGGL(store_select, dim3(grid_for(ctx->n_store, 256 * kSelItems, 4096)),
                       dim3(256), 0,
                       ctx->stream, ctx->store.as<uint32_t>(), ctx->n_store, k1, k2,
                       (uint32_t)bin_lo, (uint32_t)bin_hi, ctx->st_sel.as<uint32_t>(),
                       kin, vin, ctx->s0.as<unsigned long long>());
    HGX_LAUNCH_CHECK(ctx);
    size_t tmp = sort_tmp;
    HGX_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(ctx->st_keys.as<char>() + koff, tmp,
                                                    kin, kout, vin, vout, (int)m, 0, 64,
                                                    ctx->stream));
  }
  // 2. the batch tail of the previous load goes first
  if (carry > 0) {
    HGX_TRY(hgx_ensure(ctx, ctx->st_tmp, sizeof(int) * (size_t)carry * (R + 3)));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->st_tmp.p, ctx->rec_idx.as<int>() + ctx->n_rec * R,
                                sizeof(int) * carry * R, hipMemcpyDeviceToDevice,
                                ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->st_tmp.as<int>() + carry * R,
                                ctx->rec_tgt.as<float>() + ctx->n_rec * 3,
                                sizeof(float) * carry * 3, hipMemcpyDeviceToDevice,
                                ctx->stream));
    HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  const int64_t total = carry + m;
  HGX_TRY(hgx_ensure(ctx, ctx->rec_idx, sizeof(int32_t) * (total * R + 1)));
  HGX_TRY(hgx_ensure(ctx, ctx->rec_tgt, sizeof(float) * (total * 3 + 1)));
  if (carry > 0) {
    HGX_HIP(ctx, hipMemcpyAsync(ctx->rec_idx.p, ctx->st_tmp.p, sizeof(int) * carry * R,
                                hipMemcpyDeviceToDevice, ctx->stream));
    HGX_HIP(ctx, hipMemcpyAsync(ctx->rec_tgt.p, ctx->st_tmp.as<int>() + carry * R,
                                sizeof(float) * carry * 3, hipMemcpyDeviceToDevice,
                                ctx->stream));
  }
  // 3. the chunk's trainer records in key order
  if (m > 0) {
    hipLaunchKernelGGL(store_expand, dim3(grid_for(m, 256)), dim3(256), 0, ctx->stream,
                       ctx->st_sel.as<uint32_t>(), vout, m, carry, t, K, ctx->store_seed,
                       csr_of(ctx), ctx->rec_idx.as<int>(), ctx->rec_tgt.as<float>(),
                       ctx->s0.as<int>() + 2);
    HGX_LAUNCH_CHECK(ctx);
  }
  unsigned long long got[2] = {0, 0};
  HGX_HIP(ctx, hipMemcpyAsync(got, ctx->s0.p, 16, hipMemcpyDeviceToHost, ctx->stream));
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  HGX_CHECK(ctx, (int64_t)(got[0]) == m || m == 0, HGX_EHIP,
            "store selection found %llu of %lld records", got[0], (long long)m);
  HGX_CHECK(ctx, (got[1] & 0xffffffffull) == 0, HGX_EVALUE,
            "a stored record names rows outside the graph or a node-edge "
            "endpoint without neighbours");
  // 4. whole batches now; the tail waits for the next load unless last
  const int64_t keep = last ? 0 : total % batch;
  ctx->n_rec = total - keep;
  ctx->store_carry = keep;
  ctx->K = K;
  ctx->rec_bounds[0] = 0;
  ctx->rec_bounds[1] = ctx->n_rec;
  ctx->n_rec_blocks = 1;
  ctx->smp_family = -1;
  ctx->rec_in_order = true;
  if (n_records) *n_records = ctx->n_rec;
  return HGX_OK;
}
