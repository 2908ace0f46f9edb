// omg_free.h — device side of the free-space boundary conditions
// (m_free_space, kernels in omg_free.hip, driver in omg_api.cpp).
#pragma once

#include "omg_internal.h"

namespace omg {

constexpr int kFreeNGauss = 89;                  // gequad terms (build_kernel.f90:893)
constexpr int kFreeItype = 8;                    // itype_scf (m_free_space.f90:60)
constexpr int kFreeNScf = 2 * kFreeItype * 64;   // integration points - 1 (build_kernel.f90:895-916)
constexpr int kFreeMaxRange = 4096;              // LDS bound of k_free_tables

// The padded FFT grid: N (x, y, z) >= 2*nx; nx = the FFT level's domain + 2
// (one ghost layer); n0 = the extents of the kernel tables.
struct FreeGrid {
  int N[3];
  int nx[3];
  int n0[3];
};

struct FreeTabArgs {
  const double* p0;   // [89][3] starting exponent per Gaussian and axis (reference order 89..1)
  const int* n_iter;  // [89][3] scf_recursion passes
  double h[3];        // grid spacing per axis
  int cube;           // hx == hy == hz (one table per Gaussian)
  int n_range;        // max(n01, n02, n03, 16)
  int n0[3];          // table lengths written
  int n0max;
  double* tab;        // out: [89][3][n0max]
  double* work;       // scratch: [89][3][n_range+1]
};

// one physical face of one box whose Dirichlet values are interpolated
struct FreeFace {
  double rmin[3];   // box%r_min
  double dr[3];     // box%dr (the level's)
  long long off;    // first of nc*nc values in the face table
  int nb, nc;
};

// interp_bc's r_min / inv_dr per face direction (x, y, z), two tangential
// dims each (m_free_space.f90:128-139)
struct FreePlaneGeom {
  double r_min[3][2];
  double inv_dr[3][2];
};

void launch_free_tables(const FreeTabArgs& A, hipStream_t st);
void launch_free_dft(const double* tab, int n0max, const FreeGrid& G, double* F, int fmax, hipStream_t st);
void launch_free_karray(const double* F, int fmax, const double* w, const FreeGrid& G, double scal,
                        double* karray, hipStream_t st);
void launch_free_gather(const LevelView& L, const int* boxes, const int* bix, int n, const FreeGrid& G,
                        double rhs_fac, double* R, hipStream_t st);
void launch_free_pack(const LevelView& L, const int* boxes, int n, double* buf, hipStream_t st);
void launch_free_scatter(const double* buf, const int* bix, int n, int nc, const FreeGrid& G, double rhs_fac,
                         double* R, hipStream_t st);
void launch_free_mul(double2* Z, const double* karray, long long n, hipStream_t st);
void launch_free_planes(const double* R, const FreeGrid& G, double* planes, hipStream_t st);
void launch_free_guess(const LevelView& L, const int* boxes, const int* bix, int n, const FreeGrid& G,
                       const double* R, hipStream_t st);
void launch_free_bc_faces(const FreeFace* faces, int n_faces, const double* planes, const FreeGrid& G,
                          const FreePlaneGeom& P, double* out, hipStream_t st);

}  // namespace omg
