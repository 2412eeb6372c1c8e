// Random-row gather ceiling of the device (diagnostic).
//
// The alg-dist half sweep (hgx_algdist.hip) is a gather over random rows of
// a coordinate table: per incidence one KS-float row (64 B at C4, where the
// tables spill the Infinity Cache). Its bound is the rate at which the
// memory system serves random 64-B rows, not HBM's stream bandwidth. This
// probe measures that rate on the same box: quads of lanes gather random
// rows (each lane one float4 of the row, F rows in flight per lane, like
// algdist_half_quad), rows drawn by a per-lane xorshift (no index stream),
// from a table of `table_bytes`, best of `reps` launches. bench.py reports
// the C4 relaxation's achieved gathers/s against it.
#include <algorithm>

#include "hgx_internal.h"

namespace {

template <int F>
__global__ __launch_bounds__(256) void gather_probe(const float4 *__restrict__ tab,
                                                    uint64_t nrows, int rq,
                                                    uint64_t iters,
                                                    float *__restrict__ out) {
  const int sub = threadIdx.x & 3;
  const uint64_t grp = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 2;
  float acc = 0.f;
  uint64_t x = grp * 0x9e3779b97f4a7c15ull + 12345;
  for (uint64_t i = 0; i < iters; i += F) {
    float4 v[F];
#pragma unroll
    for (int u = 0; u < F; u++) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      const uint64_t r = x % nrows;
      v[u] = sub < rq ? tab[r * rq + sub] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < F; u++) acc += v[u].x + v[u].w;
  }
  if (acc == 1234.5f) out[0] = acc;  // keeps the loads
}

}  // namespace

extern "C" int hgx_probe_gather(hgx_ctx *ctx, int64_t table_bytes,
                                int row_floats, int in_flight, int reps,
                                double *rows_per_s) {
  if (!ctx) return HGX_EINVAL;
  HGX_CHECK(ctx, row_floats == 4 || row_floats == 8 || row_floats == 12 ||
                     row_floats == 16,
            HGX_EINVAL, "row_floats must be 4, 8, 12 or 16");
  HGX_CHECK(ctx, in_flight == 4 || in_flight == 8 || in_flight == 16,
            HGX_EINVAL, "in_flight must be 4, 8 or 16");
  HGX_CHECK(ctx, table_bytes >= 4096 && table_bytes <= (int64_t)64 << 30 &&
                     reps >= 1 && rows_per_s,
            HGX_EINVAL, "bad probe arguments");
  HGX_HIP(ctx, hipSetDevice(ctx->device));
  const int rq = row_floats / 4;
  const uint64_t nrows = (uint64_t)table_bytes / (16ull * rq);
  // the context's scratch s7 holds the table (zeros: the values are not used)
  HGX_TRY(hgx_ensure(ctx, ctx->s7, (size_t)table_bytes + 64));
  HGX_HIP(ctx, hipMemsetAsync(ctx->s7.p, 0, (size_t)table_bytes + 64, ctx->stream));
  int dev = 0, ncu = 256;
  HGX_HIP(ctx, hipGetDevice(&dev));
  HGX_HIP(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = ncu * 8, threads = 256;
  const uint64_t groups = (uint64_t)blocks * threads / 4;
  const uint64_t iters = ((1ull << 28) / groups + in_flight - 1) / in_flight * in_flight;
  float *out = reinterpret_cast<float *>((char *)ctx->s7.p + table_bytes);
  hipEvent_t a, b;
  HGX_HIP(ctx, hipEventCreate(&a));
  HGX_HIP(ctx, hipEventCreate(&b));
  float best = 1e30f;
  int rc = HGX_OK;
  for (int rep = 0; rep < reps + 1 && rc == HGX_OK; rep++) {  // +1: warm
    (void)hipEventRecord(a, ctx->stream);
    const float4 *tab = ctx->s7.as<float4>();
    if (in_flight == 4)
      hipLaunchKernelGGL(gather_probe<4>, dim3(blocks), dim3(threads), 0,
                         ctx->stream, tab, nrows, rq, iters, out);
    else if (in_flight == 8)
      hipLaunchKernelGGL(gather_probe<8>, dim3(blocks), dim3(threads), 0,
                         ctx->stream, tab, nrows, rq, iters, out);
    else
      hipLaunchKernelGGL(gather_probe<16>, dim3(blocks), dim3(threads), 0,
                         ctx->stream, tab, nrows, rq, iters, out);
    if (hipGetLastError() != hipSuccess) rc = hgx_fail(ctx, HGX_EHIP, "probe launch");
    (void)hipEventRecord(b, ctx->stream);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (rep > 0) best = std::min(best, ms);
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  HGX_HIP(ctx, hipStreamSynchronize(ctx->stream));
  hgx_release(ctx->s7);  // the probe's table is not kept
  if (rc != HGX_OK) return rc;
  *rows_per_s = (double)groups * (double)iters / (best * 1e-3);
  return HGX_OK;
}
