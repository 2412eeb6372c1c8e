// Skeleton A/B for the trainer's batch step (diagnostic, tools/ only): is a
// persistent step on ONE XCD (hand-offs inside that XCD's L2, no kernel
// boundary) faster than one launch per batch over the whole chip?
//
// Per "batch" both forms do the trainer's memory skeleton: 256 records, one
// per wave, 64 workgroups of 4 waves; round trip 1 = each wave's 20 record
// words; round trip 2 = 28 table rows of 512 B (14 slots x {param, acc})
// gathered at random rows of a 200 MB table; then 28 row stores (the
// updates). No arithmetic.
//   launch:  one kernel per batch, 64 workgroups anywhere on the chip.
//   persist: one kernel, 512 workgroups launched, only those with
//            blockIdx % 8 == 0 stay (64 workgroups, one XCD under the
//            round-robin placement; checked with HW_REG_XCC_ID, the run is
//            void if they differ); batch b + 1 starts when all 64 have
//            stored batch b: every storing wave waits for its stores
//            (vmcnt 0), workgroup barrier, one agent-scope atomic add per
//            workgroup to a per-parity counter, the others poll it with an
//            sc1 load (bounded: gives up and flags after ~2^22 polls), then
//            a workgroup barrier; the record words and rows of the next
//            batch are read with sc1 loads (L1 bypassed; the stores of the
//            same XCD sit in its L2).
// Prints us per batch for each form.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kWG = 64, kTB = 256, kRecW = 20, kSlots = 28, kRowF = 128;

__device__ __forceinline__ int ld_int_sc1(const int *p) {
  int v;
  asm volatile("global_load_dword %0, %1, off sc1\n s_waitcnt vmcnt(0)"
               : "=v"(v) : "v"(p) : "memory");
  return v;
}

__device__ __forceinline__ float2 ld_f2_sc1(const float2 *p) {
  float2 v;
  asm volatile("global_load_dwordx2 %0, %1, off sc1"
               : "=v"(v) : "v"(p) : "memory");
  return v;
}

__device__ void batch_body(int b, const int *words, float2 *tab, int nrows,
                           bool sc1) {
  const int wave = blockIdx.x / (sc1 ? 8 : 1) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int *w = words + ((size_t)b * kWG * 4 + wave) * kRecW;
  int myw;
  if (sc1) myw = ld_int_sc1(w + (lane < kRecW ? lane : 0));
  else myw = w[lane < kRecW ? lane : 0];
  float2 v[kSlots];
#pragma unroll
  for (int s = 0; s < kSlots; s++) {
    const int r = (unsigned)__builtin_amdgcn_readlane(myw, s % kRecW) * 2654435761u % nrows;
    const float2 *p = tab + (size_t)r * (kRowF / 2) + lane;
    if (sc1) v[s] = ld_f2_sc1(p);
    else v[s] = *p;
  }
  if (sc1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < kSlots; s++) {
    const int r = ((unsigned)__builtin_amdgcn_readlane(myw, s % kRecW) * 40503u + s) % nrows;
    tab[(size_t)r * (kRowF / 2) + lane] = make_float2(v[s].x + 1.f, v[s].y);
  }
}

__global__ __launch_bounds__(kTB) void step_launch(int b, const int *words,
                                                   float2 *tab, int nrows) {
  batch_body(b, words, tab, nrows, false);
}

__global__ __launch_bounds__(kTB) void step_persist(int nb, const int *words,
                                                    float2 *tab, int nrows,
                                                    int *ctr, int *xcc,
                                                    int *bad) {
  if (blockIdx.x % 8 != 0) return;
  const int me = blockIdx.x / 8;
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    int id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    xcc[me] = id & 0xf;
  }
  for (int b = 0; b < nb; b++) {
    batch_body(b, words, tab, nrows, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      int *c = ctr + (b & 1) * 64;
      __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int want = kWG * (b / 2 + 1);
      int spins = 0, ok = 1;
      while (ld_int_sc1(c) < want) {
        if (++spins > (1 << 22)) {
          ok = 0;
          atomicOr(bad, 1);
          break;
        }
      }
      s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) return;
  }
}

int main(int argc, char **argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 4000;
  const int nrows = 400000;  // 200 MB of 512-B rows
  std::vector<int> h((size_t)nb * kWG * 4 * kRecW);
  srand(1);
  for (auto &x : h) x = rand();
  int *words, *ctr, *xcc, *bad;
  float2 *tab;
  hipMalloc(&words, h.size() * 4);
  hipMemcpy(words, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&tab, (size_t)nrows * kRowF * 4);
  hipMemset(tab, 0, (size_t)nrows * kRowF * 4);
  hipMalloc(&ctr, 128 * 4);
  hipMalloc(&xcc, kWG * 4);
  hipMalloc(&bad, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; rep++) {
    // launch per batch
    hipEventRecord(e0);
    for (int b = 0; b < nb; b++)
      hipLaunchKernelGGL(step_launch, dim3(kWG), dim3(kTB), 0, 0, b, words, tab, nrows);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms_l = 0;
    hipEventElapsedTime(&ms_l, e0, e1);
    // persistent on one XCD
    hipMemset(ctr, 0, 128 * 4);
    hipMemset(bad, 0, 4);
    hipEventRecord(e0);
    hipLaunchKernelGGL(step_persist, dim3(kWG * 8), dim3(kTB), 0, 0, nb, words, tab,
                       nrows, ctr, xcc, bad);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms_p = 0;
    hipEventElapsedTime(&ms_p, e0, e1);
    int hx[kWG], hb = 0;
    hipMemcpy(hx, xcc, sizeof(hx), hipMemcpyDeviceToHost);
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    int same = 1;
    for (int i = 1; i < kWG; i++) same &= hx[i] == hx[0];
    printf("{\"batches\": %d, \"launch_us_per_batch\": %.3f, "
           "\"persist_one_xcd_us_per_batch\": %.3f, \"one_xcd\": %d, "
           "\"poll_timeout\": %d}\n",
           nb, ms_l * 1e3 / nb, ms_p * 1e3 / nb, same, hb);
  }
  return 0;
}
