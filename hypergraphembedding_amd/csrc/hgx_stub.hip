// TEMPORARY: entry points not implemented yet.
#include "hgx_internal.h"
#define STUB(ctx) return hgx_fail(ctx, HGX_EUNSUP, "%s not implemented yet", __func__)
extern "C" int hgx_sample_fobe(hgx_ctx *ctx, uint64_t, int, const int32_t *, const int32_t *, const int32_t *, const int32_t *, int64_t *) { STUB(ctx); }
extern "C" int hgx_sample_hobe(hgx_ctx *ctx, uint64_t, int, int, int64_t *) { STUB(ctx); }
extern "C" int hgx_records_set(hgx_ctx *ctx, int64_t, int, const int32_t *, const float *) { STUB(ctx); }
extern "C" int hgx_records_info(hgx_ctx *ctx, int64_t *, int *) { STUB(ctx); }
extern "C" int hgx_records_get(hgx_ctx *ctx, int32_t *, float *) { STUB(ctx); }
extern "C" int hgx_model_init(hgx_ctx *ctx, int, int64_t, int64_t, uint64_t, const float *, const float *) { STUB(ctx); }
extern "C" int hgx_model_get(hgx_ctx *ctx, float *, float *) { STUB(ctx); }
extern "C" int hgx_train(hgx_ctx *ctx, int, int, float, float, int, int, float, uint64_t, const int64_t *, float *, int *) { STUB(ctx); }
extern "C" int hgx_train_last_stats(hgx_ctx *ctx, double *, int64_t *, int64_t *) { STUB(ctx); }
