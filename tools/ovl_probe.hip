// Overlapped-preparation probe (r03): the trainer's host pattern with a
// step-like kernel chain (64 workgroups, one gather round trip) and a
// prep-like kernel (LDS bitonic sort, 1024 workgroups) per chunk of 1024
// steps. Which part of the two-stream pattern slows the chain?
//   inline   one stream: [prep][host sync][1024 steps] per chunk
//   ovl      prep c+1 on stream P (waits for steps c-1), D2H copy of 4 KB of
//            flags to pinned memory, event; host waits for it, steps of c on
//            stream S after a stream wait on that event (the trainer's form)
//   ovl-nocopy / ovl-noprep / ovl-nowait: the same minus one part
//   extra streams: the same with 12 idle streams created first (HW queue
//   sharing: GPU_MAX_HW_QUEUES = 4)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_ab/ovl_probe tools/ovl_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

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

__global__ __launch_bounds__(256) void prepk(unsigned long long *o, int *flags) {
  __shared__ unsigned long long k[4096];
  for (int i = threadIdx.x; i < 4096; i += 256)
    k[i] = (unsigned long long)((i * 2654435761u) ^ blockIdx.x) << 20 | i;
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
  if (threadIdx.x == 0) {
    o[blockIdx.x] = k[blockIdx.x % 4096];
    flags[blockIdx.x] = (int)(k[7] & 1);
  }
}

int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int CB = 1024, NCH = 12, ROWS = 200000;
  float2 *tab, *out;
  int *ids, *dflags;
  unsigned long long *po;
  CK(hipMalloc(&tab, sizeof(float2) * (size_t)ROWS * 64));
  CK(hipMalloc(&out, sizeof(float2) * (size_t)ROWS * 64));
  CK(hipMalloc(&ids, sizeof(int) * (size_t)CB * 256 * 16));
  CK(hipMalloc(&po, 8 * 4096));
  CK(hipMalloc(&dflags, 4 * 2 * CB));
  CK(hipMemset(tab, 0, sizeof(float2) * (size_t)ROWS * 64));
  {
    std::vector<int> h((size_t)CB * 256 * 16);
    unsigned x = 12345;
    for (auto &v : h) {
      x = x * 1664525u + 1013904223u;
      v = (int)((x >> 8) % ROWS);
    }
    CK(hipMemcpy(ids, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  int *hflags;
  CK(hipHostMalloc((void **)&hflags, 4 * 2 * CB));
  std::vector<hipStream_t> extra;
  hipStream_t s0, S, P;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&P, hipStreamNonBlocking));
  std::vector<hipEvent_t> bev(2 * NCH), pev(NCH);
  for (auto &e : bev) CK(hipEventCreate(&e));
  for (auto &e : pev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));

  auto run = [&](const char *name, int mode, bool copy, bool prep, bool wait,
                 bool pwait = true) {
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    double steps_ms = 0;
    if (mode == 0) {
      for (int c = 0; c < NCH; c++) {
        hipLaunchKernelGGL(prepk, dim3(1024), dim3(256), 0, s0, po, dflags);
        CK(hipMemcpyAsync(hflags, dflags, 4 * CB, hipMemcpyDeviceToHost, s0));
        CK(hipStreamSynchronize(s0));
        CK(hipEventRecord(bev[2 * c], s0));
        for (int b = 0; b < CB; b++)
          hipLaunchKernelGGL(stepk, dim3(64), dim3(256), 0, s0, tab, out, ids, b + hflags[b] * 0);
        CK(hipEventRecord(bev[2 * c + 1], s0));
      }
      CK(hipStreamSynchronize(s0));
    } else {
      auto prep_ov = [&](int c) {
        const int cp = c & 1;
        if (c >= 2 && pwait) CK(hipStreamWaitEvent(P, bev[2 * (c - 2) + 1], 0));
        if (c >= 2 && !pwait) CK(hipEventSynchronize(bev[2 * (c - 2) + 1]));
        if (prep) hipLaunchKernelGGL(prepk, dim3(1024), dim3(256), 0, P, po, dflags + cp * CB);
        if (copy)
          CK(hipMemcpyAsync(hflags + cp * CB, dflags + cp * CB, 4 * CB, hipMemcpyDeviceToHost, P));
        CK(hipEventRecord(pev[c], P));
      };
      prep_ov(0);
      for (int c = 0; c < NCH; c++) {
        if (c + 1 < NCH) prep_ov(c + 1);
        CK(hipEventSynchronize(pev[c]));
        if (wait) CK(hipStreamWaitEvent(S, pev[c], 0));
        CK(hipEventRecord(bev[2 * c], S));
        const int *hb = hflags + (c & 1) * CB;
        for (int b = 0; b < CB; b++)
          hipLaunchKernelGGL(stepk, dim3(64), dim3(256), 0, S, tab, out, ids, b + hb[b] * 0);
        CK(hipEventRecord(bev[2 * c + 1], S));
      }
      CK(hipStreamSynchronize(S));
      CK(hipStreamSynchronize(P));
    }
    const double wall =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int c = 1; c < NCH; c++) {
      float m = 0.f;
      CK(hipEventElapsedTime(&m, bev[2 * c], bev[2 * c + 1]));
      steps_ms += m;
    }
    printf("%-34s step %.3f us per launch (chunks 1..), wall %.3f us per step\n", name,
           1e3 * steps_ms / ((NCH - 1) * CB), 1e3 * wall / (NCH * CB));
  };
  for (int rep = 0; rep < 2; rep++) {
    if (rep == 1) {
      for (int i = 0; i < 12; i++) {
        hipStream_t x;
        CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        extra.push_back(x);
      }
      printf("-- with 12 extra idle streams --\n");
    }
    run("inline", 0, true, true, true);
    run("ovl", 1, true, true, true);
    run("ovl-nocopy", 1, false, true, true);
    run("ovl-noprep", 1, true, false, true);
    run("ovl-nowait", 1, true, true, false);
    run("ovl-no-prep-stream-wait", 1, true, true, true, false);
    run("inline", 0, true, true, true);
  }
  return 0;
}
