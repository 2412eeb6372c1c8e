// TEMPORARY: entry points not implemented yet.
#include "hgx_internal.h"
#define STUB(ctx) return hgx_fail(ctx, HGX_EUNSUP, "%s not implemented yet", __func__)
extern "C" int hgx_sample_fobe(hgx_ctx *ctx, uint64_t, int, const int32_t *, const int32_t *, const int32_t *, const int32_t *, int64_t *) { STUB(ctx); }
extern "C" int hgx_sample_hobe(hgx_ctx *ctx, uint64_t, int, int, int64_t *) { STUB(ctx); }
