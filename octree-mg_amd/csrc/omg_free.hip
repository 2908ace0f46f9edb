// omg_free.hip — free-space boundary conditions on the GPU (m_free_space).
//
// The reference's mg_poisson_free_3d (src/m_free_space.f90:36-214) solves the
// Poisson problem once on a coarse uniform level with its bundled BigDFT
// PSolver (poisson_3d_fft/, geocode 'F', itype_scf 8) and uses that solution
// for the boundary values of every level and as the initial guess.  Here that
// solve runs on the device in three parts:
//
//   Green's function (once per grid, PSolver's createKernel / Free_Kernel,
//   poisson_3d_fft/build_kernel.f90:55-199, 884-1164).  1/r is the 89-term
//   Gaussian sum of gequad (:1549-1740); each Gaussian is integrated against
//   the order-8 interpolating scaling function (scaling_function.f90:18-96,
//   back_trans_8 :328-370) and brought to its exponent by scf_recursion_8
//   (:443-479).  k_free_tables does this for all 89 Gaussians at once, one
//   workgroup each.  The kernel is separable per Gaussian, so its transform is
//   too: k_free_dft takes the 1D cosine transform of each table and
//   k_free_karray sums the 89 tensor products straight into the spectrum (no
//   3D transform of the kernel is needed).
//
//   Convolution (per right-hand side, PSolver / F_PoissonSolver,
//   psolver_main.f90:91-556, psolver_base.f90:1720-2153): the zero-padded
//   density goes through a D2Z transform (rocFFT via hipFFT, on the context
//   stream), is multiplied by the real kernel spectrum (scaled by
//   hx*hy*hz/(N1*N2*N3), PSolver's scal) and comes back with Z2D.  The density
//   is zero on the ghost layer, so the padded sizes only need N >= 2*(nx-2)
//   (the result is the linear convolution either way); they are chosen as
//   2^a 3^b 5^c 7^d, powers of two for power-of-two domains.
//
//   Use of the solution: the six boundary planes (m_free_space.f90:163-171),
//   the interpolated Dirichlet values of every physical face of every level
//   (ghost_cells_free_bc / interp_bc, :216-270) into the device boundary
//   table, and phi of the FFT level including its ghost faces (:176-183).
//
// Results agree with the reference at round-off (the transforms sum in another
// order than PSolver's FFT); the tests state that as a relative tolerance.
#include "omg_device.h"
#include "omg_free.h"

namespace omg {

namespace {

inline unsigned blocks_for(long long work, int block = 256) {
  long long g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 2048 * 8) g = 2048 * 8;
  return (unsigned)g;
}

#define FREE_STRIDE(t, total)                                                       \
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < (total); \
       t += (long long)gridDim.x * blockDim.x)

// lazy_8.inc: the order-8 interpolating filter ch(-7..7); the zero taps are
// left out (they add +-0.0 to a finite sum)
__device__ __forceinline__ double ch8(int j) {
  switch (j) {
    case -7: case 7: return -5.0 / 2048.0;
    case -5: case 5: return 49.0 / 2048.0;
    case -3: case 3: return -245.0 / 2048.0;
    case -1: case 1: return 1225.0 / 2048.0;
    case 0: return 1.0;
    default: return 0.0;
  }
}

}  // namespace

// One workgroup per Gaussian g (reference order: i_gauss = 89 .. 1).
//   1. the scaling function y_scf on 0..N_SCF by the cascade (every
//      workgroup builds its own copy in LDS: 6 levels of 10 taps);
//   2. "Stupid integration" of y_scf against exp(-p0 (x-i)^2 h^2) for
//      i = 0..n_range, cut after the first |value| < 1e-18 (1e-18 summed over
//      the three axes, 3e-18, in the anisotropic branch);
//   3. scf_recursion_8, n_iter times, each pass cut at the first exact zero.
__global__ void __launch_bounds__(256) k_free_tables(FreeTabArgs A) {
  extern __shared__ double sm[];
  const int g = blockIdx.x, tid = threadIdx.x, nt_ = blockDim.x;
  const int nd = kFreeNScf, nr = A.n_range;
  __shared__ int cut;
  // 1. cascade: x(7) = 1 at nt = 16, then nt = 32 .. 1024
  double* x = sm;
  double* y = sm + (nd + 1);
  for (int i = tid; i <= nd; i += nt_) x[i] = 0.0;
  __syncthreads();
  if (tid == 0) x[2 * kFreeItype / 2 - 1] = 1.0;
  __syncthreads();
  for (int nt = 4 * kFreeItype; nt <= nd; nt *= 2) {
    const int half = nt / 2;
    for (int i = tid; i < half; i += nt_) {
      double y0 = 0.0, y1 = 0.0;
      for (int j = -5; j <= 4; j++) {
        int ind = (i - j) % half;
        if (ind < 0) ind += half;
        y0 = y0 + ch8(2 * j) * x[ind];
        y1 = y1 + ch8(2 * j + 1) * x[ind];
      }
      y[2 * i] = y0;
      y[2 * i + 1] = y1;
    }
    __syncthreads();
    for (int i = tid; i < nt; i += nt_) x[i] = y[i];
    __syncthreads();
  }
  // x now holds y_scf(0..nd) (x(nd) stays 0, as in the reference)
  // 2. integration, every offset in parallel
  const int n_tab = A.cube ? 1 : 3;
  const double dx = (double)(2 * kFreeItype) / (double)nd;
  if (tid == 0) cut = nr + 1;
  __syncthreads();
  double* work = A.work + (long long)g * 3 * (nr + 1);
  for (int ik = tid; ik <= nr; ik += nt_) {
    double k3[3] = {0.0, 0.0, 0.0};
    for (int i = 0; i <= nd; i++) {
      double absci = ((double)(i * 2 * kFreeItype) / (double)nd - (0.5 * (2 * kFreeItype) - 1.0)) - (double)ik;
      if (A.cube) {
        absci = absci * absci * (A.h[0] * A.h[0]);
        k3[0] = k3[0] + x[i] * exp(-(A.p0[g * 3] * absci));
      } else {
        for (int d = 0; d < 3; d++) {
          const double u = -(A.p0[g * 3 + d] * absci * absci * (A.h[d] * A.h[d]));
          k3[d] = k3[d] + x[i] * exp(u);
        }
      }
    }
    for (int d = 0; d < n_tab; d++) work[d * (nr + 1) + ik] = k3[d] * dx;
    const bool small = A.cube ? fabs(k3[0]) < 1e-18 : fabs(k3[0]) + fabs(k3[1]) + fabs(k3[2]) < 3e-18;
    if (small) atomicMin(&cut, ik);
  }
  __syncthreads();
  const int c0 = cut;
  // 3. recursion per axis table, ping-pong in LDS (the cascade is done)
  double* a = sm;
  double* b = sm + (nr + 1);
  for (int d = 0; d < n_tab; d++) {
    for (int i = tid; i <= nr; i += nt_) a[i] = i <= c0 ? work[d * (nr + 1) + i] : 0.0;
    __syncthreads();
    const int n_iter = A.n_iter[g * 3 + d];
    for (int it = 0; it < n_iter; it++) {
      if (tid == 0) cut = nr + 1;
      __syncthreads();
      for (int i = tid; i <= nr; i += nt_) {
        double tot = 0.0;
        for (int j = -7; j <= 7; j += 2) {
          const int ind = 2 * i - j;
          const double k = (ind > nr || ind < -nr) ? 0.0 : a[ind < 0 ? -ind : ind];
          tot = tot + ch8(j) * k;
          if (j == -1) {   // the even tap in the middle
            const int ind0 = 2 * i;
            const double k0 = ind0 > nr ? 0.0 : a[ind0];
            tot = tot + ch8(0) * k0;
          }
        }
        b[i] = tot;
        if (tot == 0.0) atomicMin(&cut, i);
      }
      __syncthreads();
      const int c1 = cut;
      for (int i = tid; i <= nr; i += nt_) b[i] = i < c1 ? 0.5 * b[i] : 0.0;
      __syncthreads();
      double* s = a;
      a = b;
      b = s;
    }
    for (int dd = A.cube ? 0 : d; dd < (A.cube ? 3 : d + 1); dd++)
      for (int i = tid; i < A.n0[dd]; i += nt_) A.tab[((long long)g * 3 + dd) * A.n0max + i] = a[i];
    __syncthreads();
  }
}

// F[d][g][k], k = 0..N/2: the transform of the even extension of one 1D
// table on N points (it is real),
//   K(0) + 2 sum_{0 < n < N/2} K(n) cos(2 pi k n / N) + K(N/2) (-1)^k,
// with K(n) = 0 beyond the table; the solution only needs offsets |n| <= N/2.
__global__ void __launch_bounds__(256) k_free_dft(const double* tab, int n0max, FreeGrid G, double* F, int fmax) {
  const long long total = 3LL * kFreeNGauss * fmax;
  FREE_STRIDE(t, total) {
    const int k = (int)(t % fmax), g = (int)((t / fmax) % kFreeNGauss), d = (int)(t / ((long long)fmax * kFreeNGauss));
    const int N = G.N[d];
    if (k > N / 2) continue;
    const double* K = tab + ((long long)g * 3 + d) * n0max;
    const int n_end = min(G.n0[d], N / 2);   // n < n_end: the doubled terms
    double s = 0.0;
    for (int n = 1; n < n_end; n++) {
      const long long kn = ((long long)k * n) % N;
      s = s + K[n] * cospi(2.0 * (double)kn / (double)N);
    }
    double f = K[0] + 2.0 * s;
    if (N / 2 < G.n0[d]) f = f + ((k & 1) ? -K[N / 2] : K[N / 2]);
    F[((long long)d * kFreeNGauss + g) * fmax + k] = f;
  }
}

// The kernel spectrum on the D2Z half grid [z][y][x <= N1/2], times scal:
// sum over the Gaussians (reference order) of w_g Fx Fy Fz.  F is even in
// k, so one thread per (kx, ky <= N2/2, kz <= N3/2) writes up to four mirror
// images in y and z.
__global__ void __launch_bounds__(256) k_free_karray(const double* F, int fmax, const double* w, FreeGrid G,
                                                     double scal, double* karray) {
  const int h1 = G.N[0] / 2 + 1, h2 = G.N[1] / 2 + 1, h3 = G.N[2] / 2 + 1;
  const long long total = (long long)h1 * h2 * h3;
  FREE_STRIDE(t, total) {
    const int kx = (int)(t % h1);
    const int ky = (int)((t / h1) % h2), kz = (int)(t / ((long long)h1 * h2));
    const double* Fx = F;
    const double* Fy = F + (long long)kFreeNGauss * fmax;
    const double* Fz = F + 2LL * kFreeNGauss * fmax;
    double s = 0.0;
    for (int g = 0; g < kFreeNGauss; g++)
      s = s + w[g] * Fx[(long long)g * fmax + kx] * Fy[(long long)g * fmax + ky] * Fz[(long long)g * fmax + kz];
    s = s * scal;
    const int ys[2] = {ky, ky == 0 || 2 * ky == G.N[1] ? -1 : G.N[1] - ky};
    const int zs[2] = {kz, kz == 0 || 2 * kz == G.N[2] ? -1 : G.N[2] - kz};
    for (int a = 0; a < 2; a++)
      for (int b = 0; b < 2; b++)
        if (ys[a] >= 0 && zs[b] >= 0) karray[((long long)zs[b] * G.N[1] + ys[a]) * h1 + kx] = s;
  }
}

// m_free_space.f90:144-150: tmp(ix+1:ix+nc, ...) = rhs_fac * rhs of my boxes
// at the FFT level, into the zero-padded real grid [z][y][x]
__global__ void __launch_bounds__(256) k_free_gather(LevelView L, const int* boxes, const int* bix, int n,
                                                     FreeGrid G, double rhs_fac, double* R) {
  const int nc = L.nc, nc3 = nc * nc * nc;
  FREE_STRIDE(t, (long long)n * nc3) {
    const int q = (int)(t / nc3), r = (int)(t % nc3);
    const int i = r % nc + 1, j = (r / nc) % nc + 1, k = r / (nc * nc) + 1;
    const int* ix = bix + 3 * q;
    const long long p1 = (long long)(ix[0] - 1) * nc + i, p2 = (long long)(ix[1] - 1) * nc + j,
                    p3 = (long long)(ix[2] - 1) * nc + k;
    R[(p3 * G.N[1] + p2) * G.N[0] + p1] = rhs_fac * boxp(L, 2, boxes[q])[off_int(L, i, j, k)];
  }
}

// the rhs interiors of my FFT-level boxes for the other ranks (i fastest)
__global__ void __launch_bounds__(256) k_free_pack(LevelView L, const int* boxes, int n, double* buf) {
  const int nc = L.nc, nc3 = nc * nc * nc;
  FREE_STRIDE(t, (long long)n * nc3) {
    const int q = (int)(t / nc3), r = (int)(t % nc3);
    buf[t] = boxp(L, 2, boxes[q])[off_int(L, r % nc + 1, (r / nc) % nc + 1, r / (nc * nc) + 1)];
  }
}

// received boxes (ix per item) -> the padded grid, times rhs_fac
__global__ void __launch_bounds__(256) k_free_scatter(const double* buf, const int* bix, int n, int nc,
                                                      FreeGrid G, double rhs_fac, double* R) {
  const int nc3 = nc * nc * nc;
  FREE_STRIDE(t, (long long)n * nc3) {
    const int q = (int)(t / nc3), r = (int)(t % nc3);
    const int i = r % nc + 1, j = (r / nc) % nc + 1, k = r / (nc * nc) + 1;
    const int* ix = bix + 3 * q;
    const long long p1 = (long long)(ix[0] - 1) * nc + i, p2 = (long long)(ix[1] - 1) * nc + j,
                    p3 = (long long)(ix[2] - 1) * nc + k;
    R[(p3 * G.N[1] + p2) * G.N[0] + p1] = rhs_fac * buf[t];
  }
}

// spectrum *= kernel spectrum (real)
__global__ void __launch_bounds__(256) k_free_mul(double2* Z, const double* karray, long long n) {
  FREE_STRIDE(t, n) {
    const double k = karray[t];
    double2 z = Z[t];
    z.x = z.x * k;
    z.y = z.y * k;
    Z[t] = z;
  }
}

// m_free_space.f90:163-171: bc_x0 = 0.5 (pot(1,:,:) + pot(2,:,:)), ... from
// the solution on the nx grid (the first nx points of each padded axis)
__global__ void __launch_bounds__(256) k_free_planes(const double* R, FreeGrid G, double* planes) {
  const int n1 = G.nx[0], n2 = G.nx[1], n3 = G.nx[2];
  const long long s1 = n2 * (long long)n3, s2 = n1 * (long long)n3, s3 = n1 * (long long)n2;
  auto at = [&](int i, int j, int k) { return R[((long long)k * G.N[1] + j) * G.N[0] + i]; };
  FREE_STRIDE(t, 2 * (s1 + s2 + s3)) {
    long long u = t;
    int nb = 0;
    const long long sz[3] = {s1, s2, s3};
    while (u >= sz[nb / 2]) {
      u -= sz[nb / 2];
      nb++;
    }
    double v;
    if (nb < 2) {   // x faces: plane (j, k)
      const int j = (int)(u % n2), k = (int)(u / n2);
      v = nb == 0 ? 0.5 * (at(0, j, k) + at(1, j, k)) : 0.5 * (at(n1 - 2, j, k) + at(n1 - 1, j, k));
    } else if (nb < 4) {   // y faces: plane (i, k)
      const int i = (int)(u % n1), k = (int)(u / n1);
      v = nb == 2 ? 0.5 * (at(i, 0, k) + at(i, 1, k)) : 0.5 * (at(i, n2 - 2, k) + at(i, n2 - 1, k));
    } else {   // z faces: plane (i, j)
      const int i = (int)(u % n1), j = (int)(u / n1);
      v = nb == 4 ? 0.5 * (at(i, j, 0) + at(i, j, 1)) : 0.5 * (at(i, j, n3 - 2) + at(i, j, n3 - 1));
    }
    planes[t] = v;
  }
}

// m_free_space.f90:176-183: phi(0:nc+1, ...) of my FFT-level boxes = the
// solution at ix-1 .. ix+nc (interior and face ghosts; edges are not stored)
__global__ void __launch_bounds__(256) k_free_guess(LevelView L, const int* boxes, const int* bix, int n,
                                                    FreeGrid G, const double* R) {
  const int nc = L.nc, s = nc + 2, s3 = s * s * s;
  FREE_STRIDE(t, (long long)n * s3) {
    const int q = (int)(t / s3), r = (int)(t % s3);
    const int i = r % s, j = (r / s) % s, k = r / (s * s);
    const int nbnd = (i == 0 || i == s - 1) + (j == 0 || j == s - 1) + (k == 0 || k == s - 1);
    if (nbnd >= 2) continue;
    const int* ix = bix + 3 * q;
    const long long p1 = (long long)(ix[0] - 1) * nc + i, p2 = (long long)(ix[1] - 1) * nc + j,
                    p3 = (long long)(ix[2] - 1) * nc + k;
    boxp(L, 1, boxes[q])[off_cell(L, i, j, k)] = R[(p3 * G.N[1] + p2) * G.N[0] + p1];
  }
}

// ghost_cells_free_bc + interp_bc (m_free_space.f90:216-270) for one physical
// face per workgroup: mg_get_face_coords (m_data_structures.f90:495-539),
// then bilinear interpolation in the stored plane
__global__ void __launch_bounds__(256) k_free_bc_faces(const FreeFace* faces, const double* planes, FreeGrid G,
                                                       FreePlaneGeom P, double* out) {
  const FreeFace& f = faces[blockIdx.x];
  const int nc = f.nc, nb = f.nb, d = (nb - 1) / 2;
  const int t1 = d == 0 ? 1 : 0, t2 = d == 2 ? 1 : 2;   // tangential dims ixs
  double rmin[3] = {f.rmin[0], f.rmin[1], f.rmin[2]};
  if (nb % 2 == 0) rmin[d] = rmin[d] + f.dr[d] * (double)nc;
  const long long plane_off[6] = {0,
                                  (long long)G.nx[1] * G.nx[2],
                                  2LL * G.nx[1] * G.nx[2],
                                  2LL * G.nx[1] * G.nx[2] + (long long)G.nx[0] * G.nx[2],
                                  2LL * G.nx[1] * G.nx[2] + 2LL * G.nx[0] * G.nx[2],
                                  2LL * G.nx[1] * G.nx[2] + 2LL * G.nx[0] * G.nx[2] + (long long)G.nx[0] * G.nx[1]};
  const double* pl = planes + plane_off[nb - 1];
  const int na = G.nx[t1];
  for (int q = threadIdx.x; q < nc * nc; q += blockDim.x) {
    const int i = q % nc + 1, j = q / nc + 1;
    const double x1 = rmin[t1] + ((double)i - 0.5) * f.dr[t1];
    const double x2 = rmin[t2] + ((double)j - 0.5) * f.dr[t2];
    const double fr1 = (x1 - P.r_min[d][0]) * P.inv_dr[d][0];
    const double fr2 = (x2 - P.r_min[d][1]) * P.inv_dr[d][1];
    const int i1 = (int)ceil(fr1), i2 = (int)ceil(fr2);
    const double l1 = (double)i1 - fr1, l2 = (double)i2 - fr2;
    const double w11 = l1 * l2, w21 = (1.0 - l1) * l2, w12 = l1 * (1.0 - l2), w22 = (1.0 - l1) * (1.0 - l2);
    // 1-based plane indices (i1, i2) .. (i1+1, i2+1), first index fastest
    auto P_ = [&](int a, int b) { return pl[(a - 1) + (long long)na * (b - 1)]; };
    double v = w11 * P_(i1, i2);
    v = v + w21 * P_(i1 + 1, i2);
    v = v + w12 * P_(i1, i2 + 1);
    v = v + w22 * P_(i1 + 1, i2 + 1);
    out[f.off + (i - 1) + (long long)nc * (j - 1)] = v;
  }
}

// ---------------------------------------------------------------------------
// launchers

void launch_free_tables(const FreeTabArgs& A, hipStream_t st) {
  const size_t lds = sizeof(double) * (size_t)std::max(2 * (kFreeNScf + 1), 2 * (A.n_range + 1));
  k_free_tables<<<kFreeNGauss, 256, lds, st>>>(A);
}

void launch_free_dft(const double* tab, int n0max, const FreeGrid& G, double* F, int fmax, hipStream_t st) {
  k_free_dft<<<blocks_for(3LL * kFreeNGauss * fmax), 256, 0, st>>>(tab, n0max, G, F, fmax);
}

void launch_free_karray(const double* F, int fmax, const double* w, const FreeGrid& G, double scal,
                        double* karray, hipStream_t st) {
  const long long n = (long long)(G.N[0] / 2 + 1) * (G.N[1] / 2 + 1) * (G.N[2] / 2 + 1);
  k_free_karray<<<blocks_for(n), 256, 0, st>>>(F, fmax, w, G, scal, karray);
}

void launch_free_gather(const LevelView& L, const int* boxes, const int* bix, int n, const FreeGrid& G,
                        double rhs_fac, double* R, hipStream_t st) {
  if (n == 0) return;
  k_free_gather<<<blocks_for((long long)n * L.nc * L.nc * L.nc), 256, 0, st>>>(L, boxes, bix, n, G, rhs_fac, R);
}

void launch_free_pack(const LevelView& L, const int* boxes, int n, double* buf, hipStream_t st) {
  if (n == 0) return;
  k_free_pack<<<blocks_for((long long)n * L.nc * L.nc * L.nc), 256, 0, st>>>(L, boxes, n, buf);
}

void launch_free_scatter(const double* buf, const int* bix, int n, int nc, const FreeGrid& G, double rhs_fac,
                         double* R, hipStream_t st) {
  if (n == 0) return;
  k_free_scatter<<<blocks_for((long long)n * nc * nc * nc), 256, 0, st>>>(buf, bix, n, nc, G, rhs_fac, R);
}

void launch_free_mul(double2* Z, const double* karray, long long n, hipStream_t st) {
  k_free_mul<<<blocks_for(n), 256, 0, st>>>(Z, karray, n);
}

void launch_free_planes(const double* R, const FreeGrid& G, double* planes, hipStream_t st) {
  const long long n = 2LL * ((long long)G.nx[1] * G.nx[2] + (long long)G.nx[0] * G.nx[2] +
                             (long long)G.nx[0] * G.nx[1]);
  k_free_planes<<<blocks_for(n), 256, 0, st>>>(R, G, planes);
}

void launch_free_guess(const LevelView& L, const int* boxes, const int* bix, int n, const FreeGrid& G,
                       const double* R, hipStream_t st) {
  if (n == 0) return;
  const long long s = L.nc + 2;
  k_free_guess<<<blocks_for(n * s * s * s), 256, 0, st>>>(L, boxes, bix, n, G, R);
}

void launch_free_bc_faces(const FreeFace* faces, int n_faces, const double* planes, const FreeGrid& G,
                          const FreePlaneGeom& P, double* out, hipStream_t st) {
  if (n_faces == 0) return;
  k_free_bc_faces<<<n_faces, 256, 0, st>>>(faces, planes, G, P, out);
}

}  // namespace omg
