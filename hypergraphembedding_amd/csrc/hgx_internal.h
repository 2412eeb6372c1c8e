// Internal state of libhgx.so (MI355X / gfx950). See include/hgx.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hgx.h"

// Device buffer owned by a context; grows on demand, never shrinks.
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// Rows longer than `thresh` incidences, split into pieces of `thresh`: the
// alg-dist half sweep reduces each piece on its own wave (seg_partial) and
// finishes the row from the piece partials (long_finish); the narrow kernel
// skips them. Without this one power-law edge (~2% of all incidences at C4)
// would sit on a single lane group for the whole sweep.
struct LongRows {
  DevBuf seg;   // int2 {row, piece} per piece
  DevBuf off;   // nlong + 1: first piece of each long row
  DevBuf rows;  // nlong long-row ids
  DevBuf part;  // nseg x ks float partials [sum w, sum w*src]
  int nlong = 0, nseg = 0, thresh = 0;
};
constexpr int kLongRow = 512;

// Per-context tuning (hgx_set_tuning). None of these changes the math or
// the distribution of a result; they pick between exact implementations.
struct Tuning {
  // 2/3-hop sample rows with more expansion paths than this are sampled by
  // rejection (0: always expand)
  int64_t sample_reject_w = 1 << 15;
  // 3-hop rejection proposal: 0 auto, 1 paths (Karp-Luby), 2 uniform columns
  int sample_mode3 = 0;
  // mode 0: a node row of the 3-hop pattern (A A^T A) takes uniform columns
  // when its path count W is at least the column count times
  // 2^sample_mode3_shift (paths otherwise); an edge row (A^T A A^T) by
  // sample_mode3_shift_e. Defaults from a sweep on the C4 graph
  int sample_mode3_shift = 1;
  int sample_mode3_shift_e = 1;
  // trainer: 1 fused one-launch batch step where a batch packs, 0 the
  // two-kernel step for every batch
  int train_fused = 1;
  // trainer step at dp = 128: lanes per record (0 auto, 32: float4 per lane,
  // 64: float2 per lane)
  int train_lanes = 0;
  // trainer step workgroup size (0 auto; 128 / 256 at 32 lanes, 256 / 512 at
  // 64 lanes x float2; other values fall back to the geometry's default)
  int train_tb = 0;
  // alg-dist: long-row threshold (0: kLongRow) and coordinate row width
  // (0: round_up(k + 1, 4))
  int alg_long = 0;
  int alg_ks = 0;
  // alg-dist edge half: 0 gather the new node rows through col_e, 1 push
  // form (the node half writes per-incidence contributions in edge-major
  // order, the edge half streams them; single GPU, k <= 15)
  int alg_push = 0;
  // combiner MLP training: 1 the label head computed inside the launch that
  // forms the joint layers' deltas (one launch per batch fewer), 0 its own
  // launch
  int mlp_fuse_head = 1;
  // combiner MLP training: 1 batch b + 1's input rows gathered (with their
  // dropout) by extra workgroups of batch b's hidden-layer launch (2: of its
  // joint-layer launch), so its first layer and weight gradient read a dense
  // operand; 0 both gather
  int mlp_prefetch = 1;
  // combiner MLP training: where the weight gradients of the layers after the
  // pre layers run. 0 every gradient in one launch after the pre-layer
  // deltas; 1 two launches (those layers', then the pre layers')
  int mlp_wgrad_split = 0;
  // trainer: chunk c + 1 prepared (train_prep / train_place) on a second
  // stream while chunk c trains (1), on the same stream one chunk ahead
  // (2: queued before chunk c's batches, so the host never waits on the
  // batches for the next chunk's MULTI flags), or in line before it (0);
  // with train_prep_cus > 0 the two streams of form 1 get disjoint CU masks,
  // that many CUs for the preparation
  int train_prep_overlap = 0;
  int train_prep_cus = 0;
};

struct hgx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;      // stream every launch goes to
  hipStream_t own_stream = nullptr;  // created by hgx_create
  std::string err;

  // ---- incidence (compressed, both orientations, sorted columns) ----
  int32_t N = 0, E = 0;
  int64_t nnz = 0;
  DevBuf rp_n, col_n, rp_e, col_e;
  // alg-dist row-blocks (<= 64 whole rows, <= 256 incidences each; a longer
  // row is a block of its own): row starts, nblk + 1 entries
  DevBuf blk_n, blk_e;
  int nblk_n = 0, nblk_e = 0;
  LongRows long_n, long_e;
  double avg_deg_n = 0, avg_deg_e = 0;
  int32_t max_deg_n = 0, max_deg_e = 0;

  // ---- algebraic distance: rows of KS floats = [w, x_0..x_{k-1}, pad] ----
  int k = 0, ks = 0;
  DevBuf X[2], Y[2];
  int xcur = 0, ycur = 0;
  DevBuf mm;            // per iteration [2][ks] int32 (max, ~min) encodings
  // push form (tuning alg_push): tpos[t] = edge-major position of node-major
  // incidence t (built once per incidence), contrib = nnz x ks rows
  DevBuf tpos, contrib;
  bool tpos_ok = false;
  // sharded (node-row) mode: own node rows [row0,row1), local edge sub-CSR
  // of those rows, caller-owned exchange buffers (reduced by the caller).
  int32_t row0 = 0, row1 = 0;
  DevBuf rp_el, col_el, blk_sn, blk_el;
  int nblk_sn = 0, nblk_el = 0;
  LongRows long_sn, long_el;
  // edge-range pipelining of the exchange (hgx_alg_shard_ranges): local edge
  // rows split into n_elr contiguous ranges, each with its own long rows
  static constexpr int kMaxEdgeRanges = 16;
  LongRows long_elr[kMaxEdgeRanges];
  int32_t elr_bound[kMaxEdgeRanges + 1] = {};
  int n_elr = 0;
  float *ext_partial = nullptr;  // E x ks
  // compact exchange (hgx_alg_shard_wire): shared edges' [sum w, sum w x]
  // rows of k + 1 floats; per edge its wire row (>= 0), -1 private to this
  // rank (finished from ext_partial), -2 another rank's private edge
  float *ext_wire = nullptr;
  int64_t n_wire = 0;
  DevBuf wire_slot;
  int *ext_mm = nullptr;         // iters x 2 x ks
  int ext_iters = 0;
  double alg_ms = 0, alg_bytes = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;

  // weighted-Jaccard features (node-major / edge-major values on A's
  // pattern) and the centroid CSRs built from them
  DevBuf feat_n, feat_e, cn_p, cn_j, cn_v, ce_p, ce_j, ce_v;
  int64_t cn_nnz = 0, ce_nnz = 0;
  bool features_ok = false, centroids_ok = false;

  // sampler diagnostics of the last hgx_sample_* call
  int64_t sample_union_rows = 0, sample_fallback_rows = 0;
  int64_t sample_uniform_rows = 0;
  Tuning tune;

  // HOBE per-incidence distance weights (node-major, edge-major) and each
  // edge's largest weight, built from the current alg coords
  DevBuf hw_n, hw_e, hw_self;
  DevBuf bloom_off, bloom_bits;  // per-edge member filters (hgx_sample.hip)
  bool bloom_ok = false;

  // ---- records (SamplesToModelInput layout) ----
  int64_t n_rec = 0;
  int K = 0;
  DevBuf rec_idx, rec_tgt;
  // record kind blocks of the stream in the reference's order (e.g. nn, ee,
  // ne node rows, ne edge rows): block i = [rec_bounds[i], rec_bounds[i+1])
  static constexpr int kMaxRecBlocks = 16;
  int64_t rec_bounds[kMaxRecBlocks + 1] = {0};
  int n_rec_blocks = 0;

  // the last sampler call that wrote the records (hgx_store_append packs
  // them): family 0 FOBE (BooleanSamples), 1 HOBE (AlgebraicDistanceSamples),
  // -1 any other writer; its seed (every draw is keyed by it)
  int smp_family = -1;
  uint64_t smp_seed = 0;
  // records written by hgx_store_load are already in their epoch order (a
  // slice of the store's global permutation): hgx_train keeps that order
  // instead of shuffling; every other record writer clears it
  bool rec_in_order = false;

  // ---- compact record store (hgx_store_*, streamed epochs) ----
  // 12 B per record: {block << 28 | row, column (negatives: rank in row),
  // target bits}; everything else of the record is re-derived on load
  DevBuf store;
  int64_t n_store = 0, cap_store = 0;
  int store_family = -1, store_K = 0, store_blocks = 0;
  uint64_t store_seed = 0;
  // records of the last hgx_store_load past ctx->n_rec: the batch tail the
  // next load puts first
  int64_t store_carry = 0;
  // the last hgx_store_plan's key histogram (host copy) and its epoch seed:
  // hgx_store_load of that epoch reads its chunk sizes from it
  std::vector<unsigned> st_hist_host;
  uint64_t st_hist_seed = 0;
  bool st_hist_ok = false;
  DevBuf st_sel, st_keys, st_vals, st_tmp, st_hist;  // hgx_store_load scratch

  // ---- model ----
  int d = 0, dp = 0;
  int64_t node_rows = 0, edge_rows = 0;
  DevBuf ntab, etab, nacc, eacc;
  double train_ms = 0, train_epoch_ms = 0;
  double train_loss_sum = 0;  // sum of per-record losses, last epoch
  int64_t train_records = 0, train_batches = 0;
  int64_t train_fused = 0, train_split = 0;
  int64_t train_multi = 0;  // step batches in the MULTI pending-slot form

  // ---- scratch ----
  DevBuf s0, s1, s2, s3, s4, s5, s6, s7;
  // trainer streams of the overlapped chunk preparation (batch steps,
  // preparation), created for train_prep_cus = tstream_cus
  hipStream_t tstream[2] = {nullptr, nullptr};
  int tstream_cus = -1;
};

// Diagnostic knobs of the A/B experiments under tools/ (ablations, kernel
// geometry): the environment is read only in a build with -DHGX_DEBUG_KNOBS
// (tools/build_variant.sh); the release library always takes the default,
// so no environment variable changes what it computes.
inline int hgx_debug_env(const char *name, int dflt) {
#ifdef HGX_DEBUG_KNOBS
  const char *e = getenv(name);
  return e && e[0] ? atoi(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}
inline const char *hgx_debug_env_str(const char *name) {
#ifdef HGX_DEBUG_KNOBS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

int hgx_fail(hgx_ctx *ctx, int code, const char *fmt, ...);
// alg-dist row-block partition of rows [r0, r1) of a CSR (host side)
int hgx_make_row_blocks(hgx_ctx *ctx, const int32_t *rp, int32_t r0, int32_t r1,
                        DevBuf &blk, int &nblk);
// long rows of rows [r0, r1) of a CSR (host side)
int hgx_make_long_rows(hgx_ctx *ctx, const int32_t *rp, int32_t r0, int32_t r1,
                       LongRows &out);
int hgx_ensure(hgx_ctx *ctx, DevBuf &b, size_t bytes);
void hgx_release(DevBuf &b);

#define HGX_HIP(ctx, expr)                                                   \
  do {                                                                       \
    hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess)                                                    \
      return hgx_fail((ctx), HGX_EHIP, "%s failed: %s (%s:%d)", #expr,        \
                      hipGetErrorString(e_), __FILE__, __LINE__);            \
  } while (0)

#define HGX_CHECK(ctx, cond, code, ...)                                      \
  do {                                                                       \
    if (!(cond)) return hgx_fail((ctx), (code), __VA_ARGS__);                \
  } while (0)

#define HGX_TRY(expr)                                                        \
  do {                                                                       \
    int rc_ = (expr);                                                        \
    if (rc_ != HGX_OK) return rc_;                                           \
  } while (0)

#define HGX_LAUNCH_CHECK(ctx) HGX_HIP(ctx, hipGetLastError())

// ---- device helpers shared by the kernels ----
namespace hgx {

// Order-preserving float <-> signed int32 so a per-dim min/max reduces with
// atomicMax on device and all_reduce(MAX) on int32 across ranks. Max slots
// hold f2ord(x); min slots hold ~f2ord(x) (bitwise not: order-reversing,
// no overflow). Empty slot = INT_MIN.
__device__ __forceinline__ int f2ord(float f) {
  unsigned u = __float_as_uint(f);
  unsigned s = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return (int)(s ^ 0x80000000u);
}
__device__ __forceinline__ float ord2f(int e) {
  unsigned s = (unsigned)e ^ 0x80000000u;
  unsigned u = (s & 0x80000000u) ? (s & 0x7fffffffu) : ~s;
  return __uint_as_float(u);
}

// splitmix64 finaliser: counter-based uniform bits for the samplers.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// rand64's counter-independent part: rand64(seed, stream, ctr) =
// mix64(rand64_key(seed, stream) + ctr), for loops that hoist it
__host__ __device__ __forceinline__ uint64_t rand64_key(uint64_t seed, uint64_t stream) {
  return mix64(seed ^ mix64(stream + 0x632be59bd9b4e019ull));
}
__host__ __device__ __forceinline__ uint64_t rand64(uint64_t seed,
                                                    uint64_t stream,
                                                    uint64_t ctr) {
  return mix64(rand64_key(seed, stream) + ctr);
}
// uniform integer in [0, n) (multiply-high on 64 random bits: bias < n/2^64)
__device__ __forceinline__ uint32_t bounded(uint64_t r, uint32_t n) {
  return (uint32_t)__umul64hi(r, (uint64_t)n);
}

// record kinds of the samplers' kind blocks (ids written per kind:
// nn ln/rn, ee le/re, node-edge from node rows ln = row / re = column,
// node-edge from edge rows re = row / ln = column)
enum RecKind { REC_NN = 0, REC_EE, REC_NE_NODE, REC_NE_EDGE };

// _sample_neighbors (hg2v_sample.py:49-51) of one node-edge record: K nodes
// of its edge (col_e[nb, nb + nl)) and K edges of its node (col_n[eb,
// eb + el)), with replacement, written +1 shifted to out[0, 2K). Every draw
// is keyed by (seed, block stream, the record's row, `key`): key = the
// record's column for sampled pairs (distinct within a row), its rank in
// the row for negatives (drawn with replacement). The sampler and the
// record store's loader (hgx_store_load) call this one function, so a
// stored record reloads with the neighbours it was sampled with.
__device__ __forceinline__ void draw_record_neighbors(
    uint64_t seed, uint64_t stream, int row, uint64_t key, int K, int nb,
    int nl, int eb, int el, const int *col_e, const int *col_n, int *out) {
  const uint64_t rk = rand64_key(seed, (stream << 32) | (uint32_t)row);
  for (int k = 0; k < K; k++) {
    const uint64_t h = mix64(rk + key * 64 + k);
    const uint64_t h2 = mix64(rk + key * 64 + 32 + k);
    out[k] = col_e[nb + bounded(h, (uint32_t)nl)] + 1;
    out[K + k] = col_n[eb + bounded(h2, (uint32_t)el)] + 1;
  }
}

// Sum over aligned groups of G lanes (G a power of two <= 64); every lane of
// the group gets the sum. Steps inside a 16-lane DPP row are single VALU ops
// (quad_perm xor1 / xor2, row_half_mirror, row_mirror pair lanes whose
// partial sums are disjoint). The 16- and 32-lane steps are gfx950's
// v_permlane16_swap / v_permlane32_swap (VALU half exchanges, no LDS pipe):
// with x in two registers, the swap leaves x_i in one and x_{i^16} (x_{i^32})
// in the other on every lane, so their sum is the xor-shuffle step's value
// bit for bit (float addition commutes). Inline asm with two "+v" operands
// keeps them in distinct registers (the builtin with one value for both
// operands gave wrong sums); s_nop 1 covers the VALU-write -> permlane hazard.
template <int ctrl>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), ctrl,
                                         0xF, 0xF, false));
}
template <int G>
__device__ __forceinline__ float group_allreduce_sum(float x) {
  if (G >= 2) x += dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
  if (G >= 4) x += dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
  if (G >= 8) x += dpp_f<0x141>(x);  // row_half_mirror
  if (G >= 16) x += dpp_f<0x140>(x); // row_mirror
  if (G >= 32) {
    float a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    x = a + b;
  }
  if (G >= 64) {
    float a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    x = a + b;
  }
  return x;
}

// group_allreduce_sum<64> of N values at once, bit for bit the same sums:
// every DPP step of all N values, then the N v_permlane16_swaps back to
// back, then the N v_permlane32_swaps (four per asm block: 8 operands),
// instead of N dependent chains each ordered behind the previous one's
// volatile swaps.
#define HGX_SWAP4(op)                                                        \
  asm volatile("s_nop 1\n\t" op " %0, %1\n\t" op " %2, %3\n\t" op       \
               " %4, %5\n\t" op " %6, %7"                                  \
               : "+v"(a[i]), "+v"(b[i]), "+v"(a[i + 1]), "+v"(b[i + 1]),      \
                 "+v"(a[i + 2]), "+v"(b[i + 2]), "+v"(a[i + 3]), "+v"(b[i + 3]))
template <int N>
__device__ __forceinline__ void wave_allreduce_sum_n(float (&x)[N]) {
  static_assert(N % 4 == 0, "groups of four");
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp_f<0xB1>(x[i]);
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp_f<0x4E>(x[i]);
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp_f<0x141>(x[i]);
#pragma unroll
  for (int i = 0; i < N; i++) x[i] += dpp_f<0x140>(x[i]);
  float a[N], b[N];
#pragma unroll
  for (int i = 0; i < N; i++) a[i] = b[i] = x[i];
#pragma unroll
  for (int i = 0; i < N; i += 4) HGX_SWAP4("v_permlane16_swap_b32");
#pragma unroll
  for (int i = 0; i < N; i++) a[i] = b[i] = a[i] + b[i];
#pragma unroll
  for (int i = 0; i < N; i += 4) HGX_SWAP4("v_permlane32_swap_b32");
#pragma unroll
  for (int i = 0; i < N; i++) x[i] = a[i] + b[i];
}
#undef HGX_SWAP4

// Whole-wave min / max without LDS traffic: the four in-row DPP steps, then
// the four row results by v_readlane (wave-uniform result). ds_bpermute
// shuffles go through the CU's LDS pipe: at a kernel tail where every
// resident wave reduces ~20 values at once they queued for microseconds.
// (a lane whose DPP source is disabled keeps its own value: neutral for
// min / max)
template <int ctrl>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(x, x, ctrl, 0xF, 0xF, false);
}
template <int ctrl>
__device__ __forceinline__ float dpp_keep_f(float x) {
  return __builtin_bit_cast(float, dpp_i<ctrl>(__builtin_bit_cast(int, x)));
}
__device__ __forceinline__ float wave_max(float x) {
  x = fmaxf(x, dpp_keep_f<0xB1>(x));
  x = fmaxf(x, dpp_keep_f<0x4E>(x));
  x = fmaxf(x, dpp_keep_f<0x141>(x));
  x = fmaxf(x, dpp_keep_f<0x140>(x));
  const int b = __builtin_bit_cast(int, x);
  return fmaxf(fmaxf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)),
                     __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))),
               fmaxf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)),
                     __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48))));
}
__device__ __forceinline__ float wave_min(float x) { return -wave_max(-x); }
__device__ __forceinline__ int wave_max_i(int x) {
  x = max(x, dpp_i<0xB1>(x));
  x = max(x, dpp_i<0x4E>(x));
  x = max(x, dpp_i<0x141>(x));
  x = max(x, dpp_i<0x140>(x));
  return max(max(__builtin_amdgcn_readlane(x, 0), __builtin_amdgcn_readlane(x, 16)),
             max(__builtin_amdgcn_readlane(x, 32), __builtin_amdgcn_readlane(x, 48)));
}

}  // namespace hgx
