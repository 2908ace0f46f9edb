// FETCH_SIZE / WRITE_SIZE calibration on gfx950: kernels
// whose HBM bytes are known, read by rocprofv3 --pmc.  A 2 GiB buffer (8x the
// 256 MiB Infinity Cache), each byte read once per launch:
//   rd8   one double per lane per load (global_load_dwordx2, what k_gsrb3 /
//         k_gsrb4 issue), 64 lanes = 512 contiguous bytes
//   rd16  one double2 per lane (global_load_dwordx4), the guide's calibrated case
//   wr8   one double per lane per store (global_store_dwordx2)
//   wr8nt the same, non-temporal (k_gsrb3 / k_gsrb4's stores)
//   cp8   read 8 B + write 8 B per lane (k_box_sums3<SUB>-like traffic)
// usage: fetch_probe <kernel> [launches]; prints bytes per launch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHK(x)                                                                     \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr size_t kBytes = 2ull << 30;
constexpr size_t kN = kBytes / 8;   // doubles

__global__ void __launch_bounds__(256) rd8(const double* __restrict__ a, double* __restrict__ out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < kN; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 12345.678) out[0] = s;   // (keeps the loads)
}
__global__ void __launch_bounds__(256) rd16(const double2* __restrict__ a, double* __restrict__ out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < kN / 2; i += (size_t)gridDim.x * 256) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}
__global__ void __launch_bounds__(256) wr8(double* __restrict__ a) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < kN; i += (size_t)gridDim.x * 256) a[i] = (double)i;
}
__global__ void __launch_bounds__(256) wr8nt(double* __restrict__ a) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < kN; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store((double)i, a + i);
}
__global__ void __launch_bounds__(256) cp8(double* __restrict__ a) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < kN / 2; i += (size_t)gridDim.x * 256)
    a[i + kN / 2] = a[i] + 1.0;
}

int main(int argc, char** argv) {
  const char* k = argc > 1 ? argv[1] : "rd8";
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  double *a, *out;
  CHK(hipMalloc(&a, kBytes));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(a, 0, kBytes));
  CHK(hipDeviceSynchronize());
  const int grid = 256 * 8 * 4;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < reps; r++) {
    CHK(hipEventRecord(e0));
    if (!std::strcmp(k, "rd8")) rd8<<<grid, 256>>>(a, out);
    else if (!std::strcmp(k, "rd16")) rd16<<<grid, 256>>>((const double2*)a, out);
    else if (!std::strcmp(k, "wr8")) wr8<<<grid, 256>>>(a);
    else if (!std::strcmp(k, "wr8nt")) wr8nt<<<grid, 256>>>(a);
    else if (!std::strcmp(k, "cp8")) cp8<<<grid, 256>>>(a);
    else { std::fprintf(stderr, "unknown kernel %s\n", k); return 2; }
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  const double rd = !std::strcmp(k, "rd8") || !std::strcmp(k, "rd16") ? kBytes : (!std::strcmp(k, "cp8") ? kBytes / 2 : 0);
  const double wr = !std::strncmp(k, "wr", 2) ? kBytes : (!std::strcmp(k, "cp8") ? kBytes / 2 : 0);
  std::printf("%s: read %.0f B, written %.0f B per launch; best %.3f ms = %.2f TB/s\n", k, rd, wr, best,
              (rd + wr) / (best * 1e-3) / 1e12);
  return 0;
}
