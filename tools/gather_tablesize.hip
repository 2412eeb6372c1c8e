// Microbenchmark: random 48-B row gathers (the alg-dist row: [1/len, k=10
// coords, pad] = 12 floats) by table size, from L2-resident
// through Infinity-Cache (MALL) resident to HBM. Decides whether cache
// blocking of the C4 alg-dist sweep (node table 480 MB, edge table 240 MB)
// can beat the random-line rate measured by gather_granularity.hip.
// Each group of 4 lanes gathers one row (lanes 0..2 one float4 each), 4 rows
// in flight per lane, like algdist_half_narrow. Same number of row gathers
// for every size.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/gt tools/gather_tablesize.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void gather48(const float4 *__restrict__ tab, uint64_t nrows,
                         uint64_t iters, float *out) {
  const int lane = threadIdx.x & 63;
  const int sub = lane & 3;
  const uint64_t grp = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 2;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  uint64_t x = grp * 0x9e3779b97f4a7c15ull + 12345;
  for (uint64_t i = 0; i < iters; i += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      const uint64_t r = x % nrows;
      v[u] = sub < 3 ? tab[r * 3 + sub] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      acc.x += v[u].x;
      acc.y += v[u].y;
    }
  }
  if (acc.x == 1234.5f) out[0] = acc.y;
}

int main() {
  const size_t maxbytes = 4ull << 30;
  float4 *tab;
  float *out;
  if (hipMalloc(&tab, maxbytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(tab, 0, maxbytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int blocks = 256 * 8, threads = 256;
  const uint64_t rows_total = 1ull << 28;
  const uint64_t groups = (uint64_t)blocks * threads / 4;
  const uint64_t iters = rows_total / groups;
  for (size_t mb : {2, 8, 32, 64, 128, 192, 256, 384, 512, 1024, 4096}) {
    const uint64_t nrows = (mb << 20) / 48;
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(gather48, dim3(blocks), dim3(threads), 0, 0, tab, nrows,
                         iters, out);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    const double rows = (double)groups * iters;
    printf("table %5zu MB: %.3f ms  %.1f G rows/s  %.0f GB/s (48 B/row)\n", mb, best,
           rows / best / 1e6, rows * 48 / best / 1e6);
  }
  return 0;
}
