// Latency floor of back-to-back kernels on one stream (round 4, C4 study):
// an empty kernel, a copy of one 16^3 box per workgroup, and the same with a
// dependent second load, at 1 / 8 / 64 / 512 workgroups.  Run under
// rocprofv3 --kernel-trace; each variant is launched 50 times back to back.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(double* p) {
  if (p == nullptr && threadIdx.x == 12345) p[0] = 1.0;
}
__global__ void __launch_bounds__(512) k_copy(const double* __restrict__ a, double* __restrict__ b) {
  const long long o = (long long)blockIdx.x * 4096;
  for (int q = threadIdx.x; q < 4096; q += 512) b[o + q] = a[o + q] + 1.0;
}
__global__ void __launch_bounds__(512) k_dep(const double* __restrict__ a, const int* __restrict__ idx,
                                             double* __restrict__ b) {
  const long long o = (long long)idx[blockIdx.x] * 4096;
  for (int q = threadIdx.x; q < 4096; q += 512) b[o + q] = a[o + q] + 1.0;
}

int main() {
  const int nmax = 512;
  double *a, *b;
  int* idx;
  hipMalloc(&a, sizeof(double) * 4096 * nmax);
  hipMalloc(&b, sizeof(double) * 4096 * nmax);
  hipMalloc(&idx, sizeof(int) * nmax);
  int h[nmax];
  for (int i = 0; i < nmax; i++) h[i] = (i * 37) % nmax;
  hipMemcpy(idx, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(a, 0, sizeof(double) * 4096 * nmax);
  hipStream_t st;
  hipStreamCreate(&st);
  for (int n : {1, 8, 64, 512}) {
    for (int r = 0; r < 50; r++) k_empty<<<n, 512, 0, st>>>(nullptr);
    for (int r = 0; r < 50; r++) k_copy<<<n, 512, 0, st>>>(a, b);
    for (int r = 0; r < 50; r++) k_dep<<<n, 512, 0, st>>>(a, idx, b);
  }
  hipStreamSynchronize(st);
  std::printf("done\n");
  return 0;
}
