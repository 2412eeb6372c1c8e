/*
 * hgx.h -- C ABI of libhgx.so, the MI355X (gfx950) FOBE/HOBE hot path.
 *
 * Plain pointers and sizes only. The caller owns every host buffer; the
 * library owns all device memory, one HIP stream per context (a context is
 * thread-compatible: use one per thread) and no global state.
 *
 * Every call returns 0 on success or a negative HGX_E* code; the message is
 * in hgx_last_error(ctx). The Python host package (hypergraphembedding_amd,
 * _hgx._raise) maps
 *   HGX_EINVAL   -> AssertionError (the reference's precondition style,
 *                   e.g. embedding.py:83-85, hg2v_sample.py:646-647)
 *   HGX_EZERODIV -> ZeroDivisionError (algebraic_distance.py:49 on an
 *                   isolated row)
 *   HGX_EVALUE   -> ValueError (np.random.choice on an empty row,
 *                   hg2v_sample.py:49-51)
 *   HGX_ENUMERIC -> FloatingPointError (trainer fixed-point range left)
 *   the rest (EHIP, ENOMEM, ESTATE, EUNSUP) -> RuntimeError.
 *
 * Each entry point names the reference interface it replaces
 * (JSybrandt/HypergraphEmbedding, hypergraph_embedding/<file>:<line>).
 */
#ifndef HGX_H_
#define HGX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGX_OK 0
#define HGX_EINVAL -1    /* precondition violated (AssertionError)          */
#define HGX_EHIP -2      /* HIP / RCCL runtime error                        */
#define HGX_ENOMEM -3    /* device allocation failed                        */
#define HGX_EZERODIV -4  /* isolated node/edge in algebraic distance        */
#define HGX_ESTATE -5    /* call out of order (e.g. no incidence uploaded)  */
#define HGX_EUNSUP -6    /* shape outside what this build supports          */
#define HGX_EVALUE -7    /* ValueError in the reference (np.random.choice on
                            an empty row, hg2v_sample.py:49-51)             */
#define HGX_ENUMERIC -8  /* trainer: a gradient left the batch step's fixed-
                            point range (diverged run, NaN)                 */

#define HGX_LOSS_KLD 0   /* BooleanModel: kullback_leibler_divergence       */
#define HGX_LOSS_MSE 1   /* UnweightedFloatModel: mean_squared_error        */
#define HGX_ACT_SIGMOID 0
#define HGX_ACT_RELU 1

typedef struct hgx_ctx hgx_ctx;

/* ---- context ---------------------------------------------------------- */
int hgx_create(int device, hgx_ctx **out);
int hgx_destroy(hgx_ctx *ctx);
const char *hgx_last_error(const hgx_ctx *ctx);
int hgx_version(void);
/* Run on an external stream (e.g. torch.cuda.current_stream()); NULL =
 * the context's own stream. */
int hgx_set_stream(hgx_ctx *ctx, void *hip_stream);
int hgx_synchronize(hgx_ctx *ctx);
/* HIP devices visible to this library (no context needed), and the free /
 * total device memory of a context's device (hipMemGetInfo). */
int hgx_device_count(int *n);
int hgx_mem_info(hgx_ctx *ctx, int64_t *free_bytes, int64_t *total_bytes);
/* Implementation choices of this context (none changes a result's math or
 * distribution; not a reference interface). key:
 *   "sample_reject_w"  2/3-hop sample rows with more expansion paths are
 *                      sampled by rejection (default 32768; 0 = expand all)
 *   "sample_mode3"     3-hop rejection proposal: 0 auto, 1 paths
 *                      (Karp-Luby), 2 uniform columns
 *   "sample_mode3_shift" auto rule for node rows: uniform columns when a
 *                      row's path count >= columns x 2^shift (default 1,
 *                      -10..10); "sample_mode3_shift_e" the same for edge
 *                      rows (default 1)
 *   "train_fused"      1 fused one-launch batch step (default), 0 the
 *                      two-kernel step for every batch
 *   "train_lanes"      fused step at padded d = 128: lanes per record
 *                      (0 auto = 64, 32 = float4 per lane, 64 = float2)
 *   "train_tb"         fused step workgroup size (0 auto, 128, 256, 512;
 *                      a size the geometry has no form for -> its default)
 *   "alg_long"         alg-dist long-row threshold (0 = 512, else >= 64)
 *   "alg_ks"           alg-dist coordinate row width in floats (0 = auto:
 *                      round_up(k + 1, 4), widened from 12 to 16 floats
 *                      when the node + edge rows exceed 256 MiB)
 *   "alg_push"         alg-dist edge half: 0 gather (default), 1 push form
 *                      (the node half writes per-incidence contributions in
 *                      edge-major order, the edge half streams them; single
 *                      GPU, k <= 15; measured slower, kept for the record)
 *   "mlp_fuse_head"    combiner MLP training: 1 the label head computed in
 *                      the launch forming the joint layers' deltas (default,
 *                      bit-identical), 0 its own launch
 *   "mlp_prefetch"     combiner MLP training: 1 batch b + 1's dropped-out
 *                      input rows gathered by extra workgroups of batch b's
 *                      hidden-layer launch (default, bit-identical), 2 of its
 *                      joint-layer launch (measured 0.4% slower), 0 the
 *                      first layer and its weight gradient gather them
 *   "mlp_wgrad_split"  combiner MLP training: 0 every weight gradient in one
 *                      launch (default), 1 two launches (the layers after the
 *                      pre layers, then the pre layers; measured slower)
 *   "train_prep_overlap" trainer: 1 prepare chunk c + 1 (train_prep /
 *                      train_place) on a second stream while chunk c trains,
 *                      0 in line before each chunk (default); the same
 *                      batches, bit for bit
 *   "train_prep_cus"   with train_prep_overlap: CUs reserved for the
 *                      preparation stream by disjoint CU masks (0 = no masks)
 * Unknown keys and out-of-range values -> HGX_EINVAL. */
int hgx_set_tuning(hgx_ctx *ctx, const char *key, int64_t value);

/* ---- incidence --------------------------------------------------------- *
 * Replaces ToCsrMatrix / ToEdgeCsrMatrix(CompressRange(hg))
 * (hypergraph_util.py:96-135, 223-244): the compressed N x E incidence in
 * both orientations, int32 CSR with sorted columns. */
int hgx_upload_incidence(hgx_ctx *ctx, int32_t N, int32_t E, int64_t nnz,
                         const int32_t *rowptr_n, const int32_t *col_n,
                         const int32_t *rowptr_e, const int32_t *col_e);

/* ---- algebraic distance ----------------------------------------------- *
 * Replaces EmbedAlgebraicDistance's relaxation loop
 * (algebraic_distance.py:126-175, helpers 34-123): per iteration the node
 * half, then the edge half on the NEW node coords, then the joint per-dim
 * min-max rescale to [0,1]. Coordinates are fp32 on device.
 *   hgx_alg_dist: upload node_xy (N x k) / edge_xy (E x k), run `iters`
 *   iterations, download the rescaled result into the same buffers.
 * The split calls keep the coords resident for benchmarking / HOBE:
 *   hgx_alg_set -> hgx_alg_run (repeatable) -> hgx_alg_get. */
int hgx_alg_dist(hgx_ctx *ctx, int k, int iters, float *node_xy,
                 float *edge_xy);
int hgx_alg_set(hgx_ctx *ctx, int k, const float *node_xy,
                const float *edge_xy);
int hgx_alg_run(hgx_ctx *ctx, int iters);
int hgx_alg_get(hgx_ctx *ctx, float *node_xy, float *edge_xy);
/* Device time (ms) of the last hgx_alg_run and its algorithmic bytes
 * (8*nnz + (8+12k)*(N+E) per iteration). */
int hgx_alg_last_stats(hgx_ctx *ctx, double *ms, double *bytes);

/* Multi-GPU, node-row sharded. Rank g owns node rows
 * [row0,row1); every rank holds all edge coords. The CALLER owns the two
 * exchange buffers (device memory, e.g. torch tensors) and runs the
 * collectives (torch.distributed "nccl" = RCCL over xGMI) between calls:
 *   begin(row0,row1, partial[E*KS] f32, mm[iters*M] i32, iters, &KS)
 *   for it: node(it); edge_partial(it); all_reduce(partial, SUM);
 *           edge_final(it); all_reduce(mm[it*M : (it+1)*M], MAX)
 *   end()   -> own node rows + all edge rows rescaled on device
 * with M = 2 * KS * HGX_MM_REPLICAS. min/max words are order-preserving
 * int32 (max slot f(x), min slot ~f(x)), so MAX is the only reduction. */
#define HGX_MM_REPLICAS 64
int hgx_alg_shard_begin(hgx_ctx *ctx, int32_t row0, int32_t row1,
                        void *d_partial, void *d_mm, int iters, int *ks_out);
int hgx_alg_shard_node(hgx_ctx *ctx, int it);
int hgx_alg_shard_edge_partial(hgx_ctx *ctx, int it);
int hgx_alg_shard_edge_final(hgx_ctx *ctx, int it);
int hgx_alg_shard_end(hgx_ctx *ctx);
/* Compact exchange (optional, after begin): only edges whose incidences sit
 * on two or more ranks go on the wire, as rows of k + 1 floats
 * [sum w, sum w x_1..k] (no padding slot). edge_slot[E] (host): wire row of
 * a shared edge (0..n_shared-1, the same on every rank), -1 an edge private
 * to this rank, -2 another rank's private edge (left unset here). The caller
 * then all-reduces d_wire (n_shared * (k + 1) floats, SUM) in place of
 * d_partial, which becomes this rank's local scratch. */
int hgx_alg_shard_wire(hgx_ctx *ctx, void *d_wire, int64_t n_shared,
                       const int32_t *edge_slot);
/* Exchange pipelining (optional, after begin / wire): split the edge rows
 * into n (1..16) contiguous ranges balanced by the incidences of the whole
 * graph, so every rank gets the same split; bounds[n + 1] receives the range
 * starts. Then per iteration
 * edge_partial_range(it, r) for r = 0..n-1 in place of edge_partial(it): the
 * caller may all-reduce range r's rows (of d_partial, or its wire rows) while
 * range r + 1 is computed, and calls edge_final(it) after all of them. The
 * reference has one monolithic pass (algebraic_distance.py:77-95). */
int hgx_alg_shard_ranges(hgx_ctx *ctx, int n, int32_t *bounds);
int hgx_alg_shard_edge_partial_range(hgx_ctx *ctx, int it, int r);

/* ---- HOBE probabilities ------------------------------------------------ *
 * _same_type_dist_calc (hg2v_sample.py:527-543) and DiffTypeDistanceSample
 * (:588-629) on the device-resident alg coords (after hgx_alg_run or
 * hgx_alg_set; values are used exactly as given, i.e. already rescaled).
 * kind: 0 node-node, 1 edge-edge, 2 node-edge. Bit-exact with numpy's
 * float32 norm (double-accumulated float products, k < 32). */
int hgx_hobe_probs(hgx_ctx *ctx, int kind, int64_t n, const int32_t *a,
                   const int32_t *b, float *out);

/* Per-incidence weights (hg2v_weighting.py): which = 0 UniformWeight
 * (195-198), 1 WeightByNeighborhood(alpha) (137-167), 2 HOBE distance weight
 * (hg2v_sample.py:540-541). Output is node-major (nnz, CSR order of col_n)
 * and edge-major (nnz, CSR order of col_e); either may be NULL. */
int hgx_incidence_weights(hgx_ctx *ctx, int which, double alpha,
                          float *node_major, float *edge_major);

/* ---- samplers ----------------------------------------------------------- *
 * Record layout = SamplesToModelInput(records, K, weighted=False)
 * (hg2v_sample.py:751-797): int32 [ln, le, rn, re, nn_0..K-1, ne_0..K-1]
 * (ids +1, 0 = absent) and float32 [nn_prob, ee_prob, ne_prob].
 * Records stay on the device for hgx_train; hgx_records_get copies out.
 *
 * BooleanSamples (hg2v_sample.py:125-242). Quotas are the reference's
 * int(weight * num_samples) (:138-146); the negative quotas may be NULL
 * (neg_samples == 0). Uniform draws come from a counter-based generator
 * keyed by `seed` (distribution-identical to the reference, not the same
 * stream). */
int hgx_sample_fobe(hgx_ctx *ctx, uint64_t seed, int K,
                    const int32_t *node_quota, const int32_t *edge_quota,
                    const int32_t *neg_node_quota,
                    const int32_t *neg_edge_quota, int64_t *n_records);
/* AlgebraicDistanceSamples (hg2v_sample.py:632-717) on the device alg
 * coords: quota S for every row, nn/ee/ne probabilities as above. */
int hgx_sample_hobe(hgx_ctx *ctx, uint64_t seed, int K, int S,
                    int64_t *n_records);
/* The same on a subset of rows: quota per node row / edge row instead of S
 * (both NULL -> S everywhere, i.e. hgx_sample_hobe). Used to sample the
 * rows one rank owns and for bounded slices of large graphs. */
int hgx_sample_hobe_rows(hgx_ctx *ctx, uint64_t seed, int K,
                         const int32_t *node_quota, const int32_t *edge_quota,
                         int S, int64_t *n_records);
/* The reference's record stream bit for bit (rng="mt19937"): the same
 * samplers drawing from numpy's global legacy RandomState, whose MT19937
 * state (np.random.get_state(): 624 key words and the position) is passed
 * in and updated in place to the state the reference leaves behind.
 * hgx_sample_fobe_mt replaces BooleanSamples (hg2v_sample.py:125-242, the
 * quotas as for hgx_sample_fobe); hgx_sample_hobe_mt replaces
 * AlgebraicDistanceSamples(run_in_parallel=False) (:632-717): its
 * neighbour draws come from the worker's copy of the stream (:604-605), so
 * the returned state is the parent's after its last pair draw. The host
 * walks the stream (the bounded draws' accepted values, in order); the
 * device orders the pattern rows (scipy's SMMP column order), runs every
 * row's Fisher-Yates and writes the records (csrc/hgx_mt.hip). Such a
 * stream is not keyed, so hgx_store_append refuses it. */
int hgx_sample_fobe_mt(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                       const int32_t *node_quota, const int32_t *edge_quota,
                       const int32_t *neg_node_quota,
                       const int32_t *neg_edge_quota, int64_t *n_records);
int hgx_sample_hobe_mt(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                       int S, int64_t *n_records);
/* WeightedJaccardSamples(run_in_parallel=False) (hg2v_sample.py:395-510)
 * drawing numpy's stream, the per-row quotas int(weight * S) as for
 * hgx_sample_jaccard (declared below) and its probabilities. */
int hgx_sample_jaccard_mt(hgx_ctx *ctx, uint32_t *mt_key, int32_t *mt_pos, int K,
                          const int32_t *node_quota, const int32_t *edge_quota,
                          int64_t *n_records);
/* ---- weighted-Jaccard samples (HG2V_ADJ_JAC / HG2V_NEIGH_JAC) --------- *
 * Replaces WeightedJaccardSamples (hg2v_sample.py:395-510) with
 * SparseWeightedJaccard (:250-273) and GetAllCentroids (:276-326).
 * Features: node2features / edge2features values on A's pattern (A's CSR
 * order, A^T's CSR order), e.g. UniformWeight / WeightByNeighborhood
 * (hg2v_weighting.py:137-198). Quotas are per row, int(weight * S). */
int hgx_features_set(hgx_ctx *ctx, const float *node_major,
                     const float *edge_major);
int hgx_sample_jaccard(hgx_ctx *ctx, uint64_t seed, int K,
                       const int32_t *node_quota, const int32_t *edge_quota,
                       int64_t *n_records);
/* kind 0 node-node, 1 edge-edge (SameTypeJaccardSample, :329-341), 2
 * node-edge (DiffTypeJaccardSample, :343-392) for pairs (a[i], b[i]). */
int hgx_jaccard_probs(hgx_ctx *ctx, int kind, int64_t n, const int32_t *a,
                      const int32_t *b, float *out);
/* The centroid CSR (which 0: node rows over nodes, 1: edge rows over
 * edges); any output may be NULL (sizes first). */
int hgx_jaccard_centroids(hgx_ctx *ctx, int which, int64_t *nnz,
                          int64_t *rowptr, int32_t *col, float *val);
/* Of the last hgx_sample_* call: 2-hop rows sampled from the union by
 * rejection (rows whose expansion exceeds the sample_reject_w tuning,
 * default 32768) and rows that fell back to expansion. */
int hgx_sample_last_stats(hgx_ctx *ctx, int64_t *union_rows,
                          int64_t *fallback_rows);
/* Of the last hgx_sample_* call: 3-hop rows sampled by uniform-column
 * rejection (a subset of union_rows). */
int hgx_sample_uniform_rows(hgx_ctx *ctx, int64_t *rows);
int hgx_records_set(hgx_ctx *ctx, int64_t n, int K, const int32_t *idx,
                    const float *tgt);
/* the records of `src` copied device to device into `dst` (same device) */
int hgx_records_copy(hgx_ctx *dst, hgx_ctx *src);
int hgx_records_info(hgx_ctx *ctx, int64_t *n, int *K);
int hgx_records_get(hgx_ctx *ctx, int32_t *idx, float *tgt);
/* Kind blocks of the stream in the reference's record order (hgx_sample_*:
 * nn, ee, ne node rows, ne edge rows [, the five negative blocks]; one block
 * after hgx_records_set): block i = [bounds[i], bounds[i+1]), at most 16
 * blocks (bounds holds nblocks + 1 entries). */
int hgx_records_blocks(hgx_ctx *ctx, int *nblocks, int64_t *bounds);
/* Device-to-device record copies for collectives over caller-owned device
 * buffers (e.g. RCCL all-gather of row-sharded samples):
 * export the n x (4+2K) ids and n x 3 targets; import a stream (nblocks 0 ->
 * one block). */
int hgx_records_export(hgx_ctx *ctx, void *d_idx, void *d_tgt);
int hgx_records_import(hgx_ctx *ctx, int64_t n, int K, const void *d_idx,
                       const void *d_tgt, int nblocks, const int64_t *bounds);

/* ---- compact record store: streams larger than HBM -------------------- *
 * The reference materialises every SimilarityRecord once and fits with
 * Keras' shuffle=True: each epoch a uniform permutation of the whole
 * stream in batches of 256 (embedding.py:277-302). The store keeps each
 * sampled record as 12 bytes (kind block and row, column or rank in row,
 * target); the rest of the record (neighbour lists, negatives' columns) is
 * re-derived from the sampler's keyed draws, bit for bit.
 *   hgx_store_reset(capacity)   empty the store, reserve `capacity` records
 *   hgx_store_append()          pack the records of the last
 *                               hgx_sample_fobe / hgx_sample_hobe(_rows)
 *                               call (HGX_ESTATE for any other stream; every
 *                               record is checked to reload bit for bit);
 *                               graphs of < 2^28 nodes and edges
 *   hgx_store_read / _write     raw 3 x uint32 entries to / from host or
 *                               device memory (multi-GPU: ranks exchange
 *                               what they sampled); write takes the
 *                               sampler family (0 FOBE, 1 HOBE), K, seed
 *   hgx_store_plan(epoch_seed, budget)
 *                               the epoch's order: records sorted by a
 *                               bijective mix of (identity, epoch_seed), so
 *                               the order does not depend on where records
 *                               sit in the store; the key space cut into
 *                               chunks of <= budget records, as bin ranges
 *                               of HGX_STORE_BINS bins (bin_bounds:
 *                               n_chunks + 1 entries, counts: n_chunks;
 *                               both arrays of HGX_STORE_BINS + 1)
 *   hgx_store_load(epoch_seed, bin_lo, bin_hi, batch, last)
 *                               the chunk's records as the context's record
 *                               stream, in epoch order, after the batch
 *                               tail the previous load kept (so batches
 *                               follow the global order); unless `last`,
 *                               the stream's own tail (< batch records) is
 *                               kept for the next load. hgx_train then
 *                               trains the records in that order (no
 *                               shuffle). n_records = records to train.
 *   hgx_store_release()         free the store, its load scratch and the
 *                               loaded records (the embedders call it when
 *                               fit_store returns or raises). */
#define HGX_STORE_BINS 16384
int hgx_store_reset(hgx_ctx *ctx, int64_t capacity);
int hgx_store_append(hgx_ctx *ctx);
int hgx_store_info(hgx_ctx *ctx, int64_t *n, int *family, int *K,
                   uint64_t *seed);
int hgx_store_read(hgx_ctx *ctx, int64_t start, int64_t n, void *dst,
                   int dst_device);
int hgx_store_write(hgx_ctx *ctx, int64_t n, const void *src, int src_device,
                    int family, int K, uint64_t seed);
int hgx_store_plan(hgx_ctx *ctx, uint64_t epoch_seed, int64_t budget,
                   int *n_chunks, int32_t *bin_bounds, int64_t *counts);
int hgx_store_load(hgx_ctx *ctx, uint64_t epoch_seed, int32_t bin_lo,
                   int32_t bin_hi, int batch, int last, int64_t *n_records);
int hgx_store_release(hgx_ctx *ctx);

/* ---- hg2v_weighting distance / span weights ------------------------------ *
 * hg2v_weighting.py:34-64 (WeightBySameTypeDistance), 67-103
 * (WeightByDistance), 170-192 + 236-293 (WeightByAlgebraicSpan,
 * ComputeSpans). The vectors are the alg coordinates on the context
 * (hgx_alg_set of the reference embedding's node / edge rows). `norm`:
 * np.linalg.norm (HGX_NORM_L2: numpy's float32 sdot arithmetic) or its
 * ord=inf (HGX_NORM_INF). Values are the reference's after
 * ZeroOneScaleValues -> OneMinusValues -> AlphaScaleValues, float32 (the
 * reference's arrays of protobuf float fields are float32); zeros are
 * returned (the reference's lil_matrix drops them). */
#define HGX_NORM_L2 0
#define HGX_NORM_INF 1
/* first order: per incidence, in A's (node_major) and A^T's (edge_major)
 * CSR order (either may be NULL) */
int hgx_weight_distance(hgx_ctx *ctx, int norm, double alpha, float *node_major,
                        float *edge_major);
/* second order: the A A^T (side 0, node rows) or A^T A (side 1) pattern,
 * diagonal included, as CSR over compressed ids (rows sorted, columns
 * ascending). col == val == NULL: only *nnz (and rowptr[R+1] if given);
 * HGX_EUNSUP when the pattern's expansion exceeds 2^31 paths. */
int hgx_weight_same_type(hgx_ctx *ctx, int side, int norm, double alpha,
                         int64_t *nnz, int64_t *rowptr, int32_t *col, float *val);
/* spans (ComputeSpans) and the span weights per incidence (node_major[v,e]
 * = edge e's value, edge_major[e,v] = node v's); any output may be NULL */
int hgx_weight_span(hgx_ctx *ctx, double alpha, float *node_span,
                    float *edge_span, float *node_major, float *edge_major);

/* ---- diagnostics ----------------------------------------------------------- *
 * Random-row gather rate of the device: rows of `row_floats` floats drawn
 * uniformly from a table of `table_bytes`, quads of lanes one row, in_flight
 * (4, 8, 16) rows per lane; best of `reps` launches, in rows per second.
 * The ceiling bench.py holds the C4 alg-dist gather against. */
int hgx_probe_gather(hgx_ctx *ctx, int64_t table_bytes, int row_floats,
                     int in_flight, int reps, double *rows_per_s);

/* ---- model + trainer ---------------------------------------------------- *
 * Replaces BooleanModel / UnweightedFloatModel (hg2v_model.py:51-203) and
 * the model.fit loop (embedding.py:269-305): two tables of (rows x d) fp32,
 * row 0 = padding, Keras Adagrad (a += g^2; p -= lr*g/(sqrt(a)+eps),
 * duplicate rows of a batch summed), loss = sum over the three heads of the
 * batch mean, EarlyStopping(monitor=loss, min_delta, patience=0).
 *   init_tables NULL -> uniform(-0.05, 0.05) from `seed` on device. */
int hgx_model_init(hgx_ctx *ctx, int d, int64_t node_rows, int64_t edge_rows,
                   uint64_t seed, const float *node_tab, const float *edge_tab);
int hgx_model_get(hgx_ctx *ctx, float *node_tab, float *edge_tab);
/* Rows `rows[0..n)` of the node (table 0) or edge (table 1) table into
 * out[n x d]: the touched rows of a 10M-row table without downloading it
 * (KerasModelToEmbedding reads rows idx + 1, hg2v_model.py:31-48). */
int hgx_model_get_rows(hgx_ctx *ctx, int table, int64_t n, const int64_t *rows,
                       float *out);
/* perms: NULL -> a fresh device shuffle per epoch keyed by shuffle_seed,
 * else max_epochs x n int64 permutations (Keras' np.random.shuffle order).
 * epoch_loss: max_epochs floats (may be NULL). */
int hgx_train(hgx_ctx *ctx, int batch, int max_epochs, float lr, float eps,
              int loss, int act, float min_delta, uint64_t shuffle_seed,
              const int64_t *perms, float *epoch_loss, int *epochs_run);
/* Device time (ms) of the last hgx_train spent in the per-batch kernels
 * (the K1+K2 replays, HIP events on the context stream; excludes the
 * per-epoch shuffle and batch preparation) and the records / batches they
 * processed. */
int hgx_train_last_stats(hgx_ctx *ctx, double *ms, int64_t *records,
                         int64_t *batches);
/* Of the last hgx_train: batches run by the one-launch deferred-row step
 * (train_step: rows in several records of a batch summed as fixed point and
 * applied by the next launch, the padding row likewise) and batches that
 * took the two-kernel step (train_fwd_bwd + train_update; tuning
 * "train_fused" 0 forces it). Same Keras semantics either way
 * (embedding.py:269-305, hg2v_model.py:51-203). They differ in how a row's
 * slot gradients are summed: the two-kernel step adds them in fp32, the
 * deferred-row step rounds each slot gradient (after the 1/batch factor) to
 * the nearest multiple of 2^-44 and adds them exactly as 64-bit integers
 * (order-free, bitwise reproducible): a quantisation of 2^-45 absolute per
 * slot, so values below 2^-45 (~2.8e-14) vanish. The padding row's
 * gradients are summed in fp32 per record (steps holding a float2 of the row
 * per lane, d = 128 by default) or per workgroup of records (float4 per
 * lane, d = 256) before that rounding. A slot gradient
 * of magnitude >= 32 fails the call with HGX_ENUMERIC. */
int hgx_train_path_stats(hgx_ctx *ctx, int64_t *fused_batches,
                         int64_t *split_batches);
/* Of the last hgx_train: step batches launched in the MULTI pending-slot form
 * (a record of theirs names two rows deferred by the previous batch). */
int hgx_train_multi_pending(hgx_ctx *ctx, int64_t *batches);
/* Sum of the per-record losses (all three heads) of the last epoch of the
 * last hgx_train, in double: epoch loss = sum / records. Consecutive
 * hgx_train calls continue the same model state (tables and Adagrad
 * accumulators persist; the padding row is written back at the end of each
 * call), so a stream too large to keep resident trains as a sequence of
 * one-epoch calls over resident chunks, the caller adding up these sums
 * (hg2v_model.Hg2vModel.fit_store over hgx_store_load's chunks). */
int hgx_train_last_loss(hgx_ctx *ctx, double *loss_sum);

/* ---- dense MLP engine (combiners + link-prediction classifier) --------- *
 * Replaces the Keras models of
 *   HGX_MLP_LP_CLASSIFIER       _TrainNodeEdgeEmbeddingClassifier +
 *                               NodeEdgeEmbeddingPrediction
 *                               (evaluation_util.py:471-552):
 *                               [node | edge] -> Dense(in, relu) -> Dense(1,
 *                               sigmoid); in = embedding.dim
 *   HGX_MLP_NE_SUPERVISED       CombineEmbeddingsViaNodeEdgeClassifier(...,
 *                               with_auto_encoder=False)
 *                               (combine_embeddings_util.py:80-174); in =
 *                               input_size, out = desired_dim
 *   HGX_MLP_NE_SEMI_SUPERVISED  the same with with_auto_encoder=True
 * Layers (Keras creation order; hgx_mlp_layers gives each kernel's K x N):
 *   classifier: hidden, label
 *   combiners:  pre_node, pre_edge, joint_node, joint_edge,
 *               [post_node, post_edge, recovered_node, recovered_edge,]
 *               hidden, label
 * Weights travel flat: per layer the kernel (K x N, row-major) then the bias
 * (N). Training = Keras fit: MSE, Adagrad(lr, eps, zero accumulators; a
 * set_weights restarts them), batches sequential, Dropout(0.5) on the
 * combiner inputs (mask from `seed`), EarlyStopping(monitor=loss,
 * min_delta, patience=0). perms: NULL -> device shuffle per epoch, else
 * max_epochs x n permutations. Samples reference table rows. */
#define HGX_MLP_LP_CLASSIFIER 0
#define HGX_MLP_NE_SUPERVISED 1
#define HGX_MLP_NE_SEMI_SUPERVISED 2
typedef struct hgx_mlp hgx_mlp;
int hgx_mlp_create(hgx_ctx *ctx, int kind, int in_dim, int out_dim,
                   hgx_mlp **out);
int hgx_mlp_destroy(hgx_mlp *m);
int hgx_mlp_layers(const hgx_mlp *m, int *n_layers, int32_t *shapes);
int hgx_mlp_set_weights(hgx_mlp *m, const float *flat);
int hgx_mlp_get_weights(hgx_mlp *m, float *flat);
/* node_tab: node_rows x in_dim, edge_tab: edge_rows x in_dim (row-major) */
int hgx_mlp_set_tables(hgx_mlp *m, int64_t node_rows, const float *node_tab,
                       int64_t edge_rows, const float *edge_tab);
/* (node row, edge row, label) per sample */
int hgx_mlp_set_samples(hgx_mlp *m, int64_t n, const int32_t *node_row,
                        const int32_t *edge_row, const float *label);
int hgx_mlp_fit(hgx_mlp *m, int batch, int max_epochs, float lr, float eps,
                float min_delta, uint64_t seed, const int64_t *perms,
                float *epoch_loss, int *epochs_run);
/* output 0: the label head per (node, edge) pair (n floats);
 * 1 / 2: JointNode of node rows / JointEdge of edge rows (n x out_dim).
 * Inference: no dropout. */
int hgx_mlp_predict(hgx_mlp *m, int output, int64_t n, const int32_t *node_row,
                    const int32_t *edge_row, float *out);
/* Device time (ms, HIP events over the batch launches) of the last fit,
 * samples and batches trained, algorithmic flops (fwd + bwd + weight
 * gradients of the unpadded layers). */
int hgx_mlp_last_stats(const hgx_mlp *m, double *ms, int64_t *samples,
                       int64_t *batches, double *flops);

/* ---- host utilities (bench / test data; not reference entry points) --- *
 * Power-law synthetic incidence of SURVEY.md §8(d) (C4/C5): node degree
 * 1 + Poisson(mean_degree - 1), distinct edges per node drawn with
 * probability proportional to rank^-exponent; edges no node picked are
 * dropped and the rest renumbered (*E_out). Call with col_n == NULL to get
 * rowptr_n (N+1) and *nnz, then again with col_n (nnz) to fill the sorted
 * columns. Deterministic for `seed`. No context, no device. */
int hgx_synth_powerlaw(int32_t N, int32_t E, double mean_degree,
                       double exponent, uint64_t seed, int32_t *rowptr_n,
                       int32_t *col_n, int64_t *nnz, int32_t *E_out);
/* Native hypergraph.proto reader (Hypergraph, hypergraph.proto:6-23): the
 * serialized message -> the compressed incidence of
 * CompressRange(hg) (hypergraph_util.py:223-244) over every node's `edges`
 * list (Relabel, :208-212), duplicates dropped, plus weights (default 1).
 * Parse, read sizes, fill (rowptr_n N+1, col_n nnz, ids/weights N or E;
 * any pointer may be NULL), free. Errors: hgx_host_last_error(). */
typedef struct hgx_hg hgx_hg;
int hgx_proto_parse_hypergraph(const uint8_t *buf, int64_t len, hgx_hg **out,
                               int32_t *N, int32_t *E, int64_t *nnz);
int hgx_proto_hypergraph_fill(const hgx_hg *h, int32_t *rowptr_n,
                              int32_t *col_n, int64_t *node_ids,
                              int64_t *edge_ids, float *node_weight,
                              float *edge_weight);
void hgx_proto_hypergraph_free(hgx_hg *h);
/* Native HypergraphEmbedding writer (hypergraph.proto:26-35): rows of
 * node_tab (n_nodes x d) keyed by node_ids, likewise edges, dim, and
 * method_name (NULL = unset), entries in ascending id order. out == NULL
 * returns the size in *len; then call again with cap >= *len. */
int hgx_proto_write_embedding(int64_t n_nodes, const int64_t *node_ids,
                              const float *node_tab, int64_t n_edges,
                              const int64_t *edge_ids, const float *edge_tab,
                              int d, const char *method_name, uint8_t *out,
                              int64_t cap, int64_t *len);
/* Native HypergraphEmbedding reader (hypergraph.proto:26-35): one buffer
 * holding one message, or several shards of one embedding concatenated
 * (protobuf's wire format merges them: map entries union, a repeated key
 * keeps its last entry, the last dim / method_name wins). Any size, no
 * 2 GiB message limit. Parse -> sizes (entries per map, `width` = values per
 * entry, the same for every entry, and the dim field, 0 if unset); fill
 * (ids ascending, tables n x width row-major; any pointer may be NULL;
 * method_name NUL-terminated, cap >= hgx_proto_embedding_method_len + 1);
 * free. Replaces HypergraphEmbedding.ParseFromString for embeddings
 * written by runner.py:363-364 or by write_embedding's shards. */
typedef struct hgx_emb hgx_emb;
int hgx_proto_parse_embedding(const uint8_t *buf, int64_t len, hgx_emb **out,
                              int64_t *n_nodes, int64_t *n_edges,
                              int64_t *width, int32_t *dim);
int hgx_proto_embedding_fill(const hgx_emb *h, int64_t *node_ids,
                             float *node_tab, int64_t *edge_ids,
                             float *edge_tab, char *method_name, int64_t cap);
int64_t hgx_proto_embedding_method_len(const hgx_emb *h);
void hgx_proto_embedding_free(hgx_emb *h);
/* Hypergraph writer (test / bench data): compressed incidence + original
 * ids -> wire bytes (repeated fields unpacked, proto2's default). */
int hgx_proto_write_hypergraph(int32_t N, int32_t E, const int32_t *rowptr_n,
                               const int32_t *col_n, const int32_t *rowptr_e,
                               const int32_t *col_e, const int64_t *node_ids,
                               const int64_t *edge_ids, uint8_t *out,
                               int64_t cap, int64_t *len);
/* ---- link prediction, Python `random` semantics (host) ------------------ *
 * state: the 625 ints of random.getstate()[1] (MT19937 words + position),
 * advanced in place exactly as CPython's `random` would be.
 * SampleMissingConnections (evaluation_util.py:125-158): nodes / edges are
 * list positions (the map iteration order the caller saw); rowptr/col = each
 * node's edges as sorted edge positions. Outputs the distinct accepted
 * (node, edge) positions in insertion order (num_samples capacity). */
int hgx_pyrandom_sample_missing(uint32_t *state, int32_t n_nodes,
                                int32_t n_edges, const int64_t *rowptr,
                                const int32_t *col, int64_t num_samples,
                                int32_t *node_pos, int32_t *edge_pos,
                                int64_t *n_out);
/* RemoveRandomConnections (evaluation_util.py:84-122): pairs in the
 * reference's node_edges order, current degrees (decremented in place);
 * outputs the indices of the removed pairs in removal order. */
int hgx_pyrandom_remove_connections(uint32_t *state, int64_t n_pairs,
                                    const int32_t *pair_node,
                                    const int32_t *pair_edge,
                                    int32_t *node_deg, int32_t *edge_size,
                                    double probability, int64_t *removed,
                                    int64_t *n_removed);
const char *hgx_lp_last_error(void);
/* Message of the last failed host utility call on this thread. */
const char *hgx_host_last_error(void);
/* CSR transpose by counting sort (rows of the result sorted). */
int hgx_csr_transpose(int32_t nrow, int32_t ncol, const int32_t *rowptr,
                      const int32_t *col, int32_t *rowptr_t, int32_t *col_t);

#ifdef __cplusplus
}
#endif
#endif /* HGX_H_ */
