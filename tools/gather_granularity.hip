// Microbenchmark: cost of random gathers from a table far larger than the
// Infinity Cache, by chunk size. Each wave gathers random aligned chunks of
// C bytes (C/16 lanes per chunk, 16 B per lane); the same number of chunks
// for every C. If a 64-B chunk costs as much as a 128-B one, the memory
// system moves whole 128-B lines for small gathers (informs the alg-dist row
// layout). Build: hipcc --offload-arch=gfx950 -O3 -o
// /tmp/gg tools/gather_granularity.hip ; run: /tmp/gg
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void gather(const float4 *__restrict__ tab, uint64_t nchunk_tab,
                       int lanes_per_chunk, uint64_t iters, float *out) {
  const int lane = threadIdx.x & 63;
  const int sub = lane % lanes_per_chunk;
  const uint64_t wid = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
  const uint64_t grp = wid * (64 / lanes_per_chunk) + lane / lanes_per_chunk;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  uint64_t x = grp * 0x9e3779b97f4a7c15ull + 12345;
  for (uint64_t i = 0; i < iters; i += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      const uint64_t c = x % nchunk_tab;
      v[u] = tab[c * lanes_per_chunk + sub];
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
  const size_t bytes = 4ull << 30;  // 4 GiB table
  float4 *tab;
  float *out;
  if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(tab, 0, bytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int blocks = 256 * 8, threads = 256;
  const uint64_t chunks_total = 1ull << 28;  // same chunk count for every C
  for (int C : {16, 32, 64, 128, 256}) {
    const int lpc = C / 16;
    const uint64_t groups = (uint64_t)blocks * threads / lpc;
    const uint64_t iters = chunks_total / groups;
    const uint64_t nchunk_tab = bytes / C;
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(gather, dim3(blocks), dim3(threads), 0, 0, tab,
                         nchunk_tab, lpc, iters, out);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, a, b);
      const double n = (double)groups * iters;
      if (rep)
        printf("chunk %4d B: %.2f ms  %.1f G chunks/s  useful %.2f TB/s  "
               "as 64-B lines %.2f TB/s  as 128-B lines %.2f TB/s\n",
               C, ms, n / ms / 1e6, n * C / ms / 1e9,
               n * ((C + 63) / 64) * 64 / ms / 1e9,
               n * ((C + 127) / 128) * 128 / ms / 1e9);
    }
  }
  return 0;
}
