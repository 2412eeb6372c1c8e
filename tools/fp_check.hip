// Device float sqrt / division rounding vs IEEE (numpy) -- tools only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
__global__ void k(const float *a, const float *b, float *o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  o[6 * i + 0] = __fsqrt_rn(a[i]);
  o[6 * i + 1] = sqrtf(a[i]);
  o[6 * i + 2] = __fdiv_rn(a[i], b[i]);
  o[6 * i + 3] = a[i] / b[i];
  o[6 * i + 4] = (float)__dsqrt_rn((double)a[i]);
  o[6 * i + 5] = __builtin_amdgcn_sqrtf(a[i]);
}
int main(int argc, char **argv) {
  const int n = 1 << 20;
  std::vector<float> a(n), b(n), o(6 * (size_t)n);
  FILE *f = fopen(argv[1], "rb");
  fread(a.data(), 4, n, f); fread(b.data(), 4, n, f); fclose(f);
  float *da, *db, *dout;
  hipMalloc(&da, 4 * n); hipMalloc(&db, 4 * n); hipMalloc(&dout, 24 * (size_t)n);
  hipMemcpy(da, a.data(), 4 * n, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, da, db, dout, n);
  hipMemcpy(o.data(), dout, 24 * (size_t)n, hipMemcpyDeviceToHost);
  f = fopen(argv[2], "wb"); fwrite(o.data(), 4, 6 * (size_t)n, f); fclose(f);
  return 0;
}
