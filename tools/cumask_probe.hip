// CU-mask probe (r03): which CUs a stream created with
// hipExtStreamCreateWithCUMask dispatches to, and whether a dependent chain
// of short 64-workgroup kernels on one masked stream keeps its per-kernel
// time while an LDS-heavy 1024-workgroup kernel runs on a disjoint mask.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_ab/cumask_probe tools/cumask_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void where(unsigned *out, int spin) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) {
  }
  if (threadIdx.x == 0) out[blockIdx.x] = (xcc & 0xf) << 16 | (hw & 0xffff);
}

// a step-like kernel: 64 workgroups, one dependent gather round trip per wave
// plus stores (the trainer's memory skeleton, small)
__global__ __launch_bounds__(256) void stepk(const float2 *tab, float2 *out, const int *ids,
                                             int b) {
  const int w = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x % 64;
  const int *ri = ids + ((size_t)b * 256 + w) * 16;
  const int rv = ri[lane % 16];
  float2 acc = make_float2(0.f, 0.f);
#pragma unroll
  for (int s = 0; s < 14; s++) {
    const int r = __builtin_amdgcn_readlane(rv, s);
    const float2 v = tab[(size_t)r * 64 + lane];
    acc.x += v.x;
    acc.y += v.y;
  }
#pragma unroll
  for (int s = 0; s < 14; s++) {
    const int r = __builtin_amdgcn_readlane(rv, s);
    out[(size_t)r * 64 + lane] = acc;
  }
}

// a prep-like kernel: LDS bitonic sort of 4096 64-bit keys per workgroup
__global__ __launch_bounds__(256) void prepk(unsigned long long *o, int rounds) {
  __shared__ unsigned long long k[4096];
  for (int r = 0; r < rounds; r++) {
    for (int i = threadIdx.x; i < 4096; i += 256)
      k[i] = (unsigned long long)((i * 2654435761u) ^ (blockIdx.x + r)) << 20 | i;
    __syncthreads();
    for (int size = 2; size <= 4096; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = threadIdx.x; t < 2048; t += 256) {
          const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
          const bool up = (lo & size) == 0;
          const unsigned long long x = k[lo], y = k[hi];
          if ((x > y) == up) {
            k[lo] = y;
            k[hi] = x;
          }
        }
        __syncthreads();
      }
  }
  if (threadIdx.x == 0) o[blockIdx.x] = k[blockIdx.x % 4096];
}

static void mask_range(std::vector<uint32_t> &m, int lo, int hi) {  // bits [lo, hi)
  std::fill(m.begin(), m.end(), 0u);
  for (int i = lo; i < hi; i++) m[i / 32] |= 1u << (i % 32);
}

static void probe(const char *name, const std::vector<uint32_t> &m) {
  hipStream_t s;
  printf("probe %s: mask words %zu, first %08x\n", name, m.size(), m[0]);
  CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
  const int nwg = 2048;
  unsigned *d;
  CK(hipMalloc(&d, nwg * 4));
  hipLaunchKernelGGL(where, dim3(nwg), dim3(64), 0, s, d, 2000);  // 20 us each
  CK(hipStreamSynchronize(s));
  std::vector<unsigned> h(nwg);
  CK(hipMemcpy(h.data(), d, nwg * 4, hipMemcpyDeviceToHost));
  std::set<unsigned> cus;
  std::set<int> xccs;
  int per_xcc[16] = {0};
  for (unsigned v : h) {
    const unsigned xcc = v >> 16, hw = v & 0xffff;
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    const unsigned key = xcc << 8 | se << 5 | sh << 4 | cu;
    if (!cus.count(key)) per_xcc[xcc]++;
    cus.insert(key);
    xccs.insert((int)xcc);
  }
  printf("%-28s distinct CUs %3zu, XCCs %zu, CUs per XCC:", name, cus.size(), xccs.size());
  for (int x = 0; x < 8; x++) printf(" %d", per_xcc[x]);
  printf("\n");
  CK(hipFree(d));
  CK(hipStreamDestroy(s));
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  printf("CUs: %d\n", ncu);
  const int W = (ncu + 31) / 32;
  std::vector<uint32_t> m(W);
  mask_range(m, 0, ncu);
  probe("all", m);
  mask_range(m, 0, 32);
  probe("bits 0..31", m);
  mask_range(m, 0, 8);
  probe("bits 0..7", m);
  mask_range(m, 32, ncu);
  probe("bits 32..", m);
  std::fill(m.begin(), m.end(), 0u);
  for (int i = 0; i < ncu; i += 8) m[i / 32] |= 1u << (i % 32);
  probe("every 8th bit", m);
  std::fill(m.begin(), m.end(), 0u);
  for (int i = 0; i < ncu; i++)
    if (i % 8 != 0) m[i / 32] |= 1u << (i % 32);
  probe("all but every 8th", m);

  // interference: a chain of 4096 stepk launches alone / beside prepk
  const int NB = 4096, ROWS = 200000;
  float2 *tab, *out;
  int *ids;
  unsigned long long *po;
  CK(hipMalloc(&tab, sizeof(float2) * (size_t)ROWS * 64));
  CK(hipMalloc(&out, sizeof(float2) * (size_t)ROWS * 64));
  CK(hipMalloc(&ids, sizeof(int) * (size_t)NB * 256 * 16));
  CK(hipMalloc(&po, 8 * 4096));
  CK(hipMemset(tab, 0, sizeof(float2) * (size_t)ROWS * 64));
  {
    std::vector<int> h((size_t)NB * 256 * 16);
    unsigned x = 12345;
    for (auto &v : h) {
      x = x * 1664525u + 1013904223u;
      v = (int)((x >> 8) % ROWS);
    }
    CK(hipMemcpy(ids, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  struct Cfg {
    const char *name;
    int split;  // 0: plain streams; k: prep on every k-th CU bit, step on the rest
    bool prep;
  } cfgs[] = {{"plain, alone", 0, false},     {"plain, beside prep", 0, true},
              {"masked 1/8, alone", 8, false}, {"masked 1/8, beside prep", 8, true},
              {"masked 1/4, beside prep", 4, true}, {"plain, alone", 0, false}};
  for (const Cfg &c : cfgs) {
    hipStream_t ss, sp;
    if (c.split) {
      std::vector<uint32_t> ms(W, 0u), mp(W, 0u);
      for (int i = 0; i < ncu; i++) (i % c.split ? ms : mp)[i / 32] |= 1u << (i % 32);
      CK(hipExtStreamCreateWithCUMask(&ss, W, ms.data()));
      CK(hipExtStreamCreateWithCUMask(&sp, W, mp.data()));
    } else {
      CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
      CK(hipStreamCreateWithFlags(&sp, hipStreamNonBlocking));
    }
    hipEvent_t e0, e1, p0, p1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&p0));
    CK(hipEventCreate(&p1));
    for (int rep = 0; rep < 2; rep++) {
      CK(hipDeviceSynchronize());
      if (c.prep) {
        CK(hipEventRecord(p0, sp));
        hipLaunchKernelGGL(prepk, dim3(1024), dim3(256), 0, sp, po, 24);
        CK(hipEventRecord(p1, sp));
      }
      CK(hipEventRecord(e0, ss));
      for (int b = 0; b < NB; b++) hipLaunchKernelGGL(stepk, dim3(64), dim3(256), 0, ss, tab, out, ids, b);
      CK(hipEventRecord(e1, ss));
      CK(hipDeviceSynchronize());
      float ms = 0.f, pms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (c.prep) CK(hipEventElapsedTime(&pms, p0, p1));
      if (rep == 1)
        printf("%-26s step %.3f us per launch over %d; prep kernel %.1f us\n", c.name,
               1e3f * ms / NB, NB, 1e3f * pms);
    }
    CK(hipStreamDestroy(ss));
    CK(hipStreamDestroy(sp));
  }
  return 0;
}
