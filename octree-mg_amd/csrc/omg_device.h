// omg_device.h — the device data layout and the shared device helpers.
//
// Box storage (one variable of one box, `stride` doubles, 512-B aligned):
//
//   [ colour 0 interior | colour 1 interior | 6 ghost faces ]
//
// The reference stores cc(0:nc+1,0:nc+1,0:nc+1) with i fastest.  Here the
// interior is split by the global red-black colour e = (i+j+k) & 1 (even box
// sizes make it global), each colour packed row by row:
//     off(i,j,k) = e*HV + ((i-1)>>1) + H*((j-1) + nc*(k-1)),   H = ceil(nc/2)
// and the six ghost faces follow, each split by the colour of the ghost cell:
//     off(nb,a,c) = 2*HV + (nb-1)*FS + e*HF*nc + ((a-1)>>1) + HF*(c-1)
// with (a,c) the tangential indices of the face (x faces: (j,k); y: (i,k);
// z: (i,j)), exactly the reference's face arrays (m_ghost_cells.f90:456-663).
// A red-black substep then streams one colour of phi, the matching colour of
// rhs and half of each ghost face, all contiguous.  Edge and corner ghost
// cells are not stored: no operator of the reference ever reads them (7-point
// stencils, face interpolation, sparse prolongation only touch face ghosts).
#pragma once

#include "omg_internal.h"

namespace omg {

__device__ __forceinline__ double* boxp(const LevelView& L, int iv, int b) {
  return (iv == 1 ? L.phi : L.data + (long long)(iv - 1) * L.vstride) + (long long)b * L.stride;
}

// interior cell (1 <= i,j,k <= nc)
__device__ __forceinline__ int off_int(const LevelView& L, int i, int j, int k) {
  return ((i + j + k) & 1) * L.hv + ((i - 1) >> 1) + L.h * ((j - 1) + L.nc * (k - 1));
}
// ghost cell of face nb (1..6) at tangential (a, c)
__device__ __forceinline__ int off_gh(const LevelView& L, int nb, int a, int c) {
  const int g = (nb & 1) ? 0 : L.nc + 1;
  return 2 * L.hv + (nb - 1) * L.fs + ((g + a + c) & 1) * (L.hf * L.nc) + ((a - 1) >> 1) + L.hf * (c - 1);
}
// any stored cell: interior or face ghost (never an edge/corner)
__device__ __forceinline__ int off_cell(const LevelView& L, int i, int j, int k) {
  const int n1 = L.nc + 1;
  if (i == 0) return off_gh(L, 1, j, k);
  if (i == n1) return off_gh(L, 2, j, k);
  if (j == 0) return off_gh(L, 3, i, k);
  if (j == n1) return off_gh(L, 4, i, k);
  if (k == 0) return off_gh(L, 5, i, j);
  if (k == n1) return off_gh(L, 6, i, j);
  return off_int(L, i, j, k);
}
// cell at normal index `layer` of face nb, tangential (a, c)
__device__ __forceinline__ int off_face_cell(const LevelView& L, int nb, int layer, int a, int c) {
  const int d = (nb + 1) >> 1;
  if (d == 1) return off_cell(L, layer, a, c);
  if (d == 2) return off_cell(L, a, layer, c);
  return off_cell(L, a, c, layer);
}
// decode a stored offset q (0 <= q < 2*HV + 6*FS) into (i,j,k); false for
// padding slots of odd box sizes
__device__ __forceinline__ bool cell_of(const LevelView& L, int q, int& i, int& j, int& k) {
  const int nc = L.nc;
  if (q < 2 * L.hv) {
    const int e = q >= L.hv, r = q - e * L.hv;
    const int ih = r % L.h, row = r / L.h;
    j = row % nc + 1;
    k = row / nc + 1;
    i = 2 * ih + 1 + ((1 + j + k + e) & 1);
    return i <= nc;
  }
  const int r0 = q - 2 * L.hv, nb = r0 / L.fs + 1, r1 = r0 % L.fs;
  const int e = r1 >= L.hf * nc, r = r1 - e * L.hf * nc;
  const int ah = r % L.hf, c = r / L.hf + 1;
  const int g = (nb & 1) ? 0 : nc + 1;
  const int a = 2 * ah + 1 + ((1 + g + c + e) & 1);
  if (a > nc) return false;
  const int d = (nb + 1) >> 1;
  if (d == 1) { i = g; j = a; k = c; }
  else if (d == 2) { i = a; j = g; k = c; }
  else { i = a; j = c; k = g; }
  return true;
}

// The same layout with a compile-time (even) box size, for LDS-tiled kernels
// that stage a whole stored box.
template <int NC>
struct Tl {
  static constexpr int H = NC / 2, HV = H * NC * NC, FH = H * NC, FS = 2 * FH, NST = 2 * HV + 6 * FS;
  __device__ static __forceinline__ int oint(int i, int j, int k) {
    return ((i + j + k) & 1) * HV + ((i - 1) >> 1) + H * ((j - 1) + NC * (k - 1));
  }
  __device__ static __forceinline__ int ogh(int nb, int a, int c) {
    const int g = (nb & 1) ? 0 : NC + 1;
    return 2 * HV + (nb - 1) * FS + ((g + a + c) & 1) * FH + ((a - 1) >> 1) + H * (c - 1);
  }
  __device__ static __forceinline__ int ocell(int i, int j, int k) {
    if (i == 0) return ogh(1, j, k);
    if (i == NC + 1) return ogh(2, j, k);
    if (j == 0) return ogh(3, i, k);
    if (j == NC + 1) return ogh(4, i, k);
    if (k == 0) return ogh(5, i, j);
    if (k == NC + 1) return ogh(6, i, j);
    return oint(i, j, k);
  }
  // interior slot q (< 2*HV) -> (i, j, k)
  __device__ static __forceinline__ void decode(int q, int& i, int& j, int& k) {
    const int e = q >= HV, r = q - e * HV, ih = r % H, row = r / H;
    j = row % NC + 1;
    k = row / NC + 1;
    i = 2 * ih + 1 + ((1 + j + k + e) & 1);
  }
};

// max of two |res| values (non-negative, or NaN) on their IEEE bit patterns:
// the same result as fmax for numbers, but NaN and Inf propagate (fmax drops
// a NaN operand), so a diverged field reaches the max residual
__device__ __forceinline__ double amax(double a, double b) {
  return (unsigned long long)__double_as_longlong(a) >= (unsigned long long)__double_as_longlong(b) ? a : b;
}

__device__ __forceinline__ void atomic_max_nonneg(unsigned long long* p, double v) {
  // |res| >= 0: IEEE bit patterns of non-negative doubles order like uint64
  atomicMax(p, (unsigned long long)__double_as_longlong(v));
}

// Max |res| over a launch (max_residual_lvl, exact in any order). A
// multi-workgroup launch issues one device-scope atomic per workgroup, spread
// over kMaxSlots slots kMaxSlotStride words apart: the 32K workgroups of a
// 512^3 level queueing on one address cost 2.4 ms per pass. launch_max_fold
// folds the slots into one word and zeroes them again. A one-workgroup launch
// (the coarse tail) keeps one atomic per wave on maxbits[0].
template <int BS>
__device__ __forceinline__ void launch_max(unsigned long long* maxbits, double mx) {
  for (int off = 32; off > 0; off >>= 1) mx = amax(mx, __shfl_down(mx, off, 64));
  if (gridDim.x == 1) {
    if ((threadIdx.x & 63) == 0) atomic_max_nonneg(maxbits, mx);
    return;
  }
  __shared__ double wmax[BS / 64];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < BS / 64; w++) mx = amax(mx, wmax[w]);
    atomic_max_nonneg(maxbits + (blockIdx.x % kMaxSlots) * kMaxSlotStride, mx);
  }
}

template <int OP>
struct OpCoef {
  double ix, iy, iz, fac, lambda;
  __device__ __forceinline__ OpCoef(const LevelView& L, double lam) {
    ix = L.idr2[0];
    iy = L.idr2[1];
    iz = L.idr2[2];
    lambda = lam;
    // box_gs_lpl fac = 0.5/sum(idr2) (m_laplacian.f90:64-65);
    // box_gs_helmh fac = 1/(2*sum(idr2)+lambda) (m_helmholtz.f90:58-59)
    if (OP == OP_HELM)
      fac = 1.0 / (2 * ((ix + iy) + iz) + lambda);
    else
      fac = 0.5 / ((ix + iy) + iz);
  }
};

// The 7 values of a stencil: centre and x-/x+/y-/y+/z-/z+ neighbours.
struct Nbr7 {
  double c, xm, xp, ym, yp, zm, zp;
};

__device__ __forceinline__ Nbr7 load7(const LevelView& L, const double* u, int i, int j, int k) {
  Nbr7 s;
  s.c = u[off_int(L, i, j, k)];
  s.xm = u[off_cell(L, i - 1, j, k)];
  s.xp = u[off_cell(L, i + 1, j, k)];
  s.ym = u[off_cell(L, i, j - 1, k)];
  s.yp = u[off_cell(L, i, j + 1, k)];
  s.zm = u[off_cell(L, i, j, k - 1)];
  s.zp = u[off_cell(L, i, j, k + 1)];
  return s;
}

// box_lpl / box_helmh (m_laplacian.f90:183-189, m_helmholtz.f90:141-148)
template <int OP>
__device__ __forceinline__ double op_value(const OpCoef<OP>& K, const Nbr7& s) {
  double v = K.ix * (s.xm + s.xp - 2 * s.c) + K.iy * (s.ym + s.yp - 2 * s.c) +
             K.iz * (s.zm + s.zp - 2 * s.c);
  if (OP == OP_HELM) v = v - K.lambda * s.c;
  return v;
}

// box_gs_lpl / box_gs_helmh cell update (m_laplacian.f90:104-108)
template <int OP>
__device__ __forceinline__ double gs_value(const OpCoef<OP>& K, const Nbr7& s, double f) {
  return K.fac * (K.ix * (s.xp + s.xm) + K.iy * (s.yp + s.ym) + K.iz * (s.zp + s.zm) - f);
}

// Operators with a cell coefficient: harmonic face means of eps.
// box_ahelmh (m_ahelmholtz.f90:215-234) and box_gs_ahelmh with the 3D a0(5:6)
// index fixed (:143-156) use eps1..3 (vars 5..7, one per direction);
// box_vlpl / box_gs_vlpl (m_vlaplacian.f90:51-189) and box_vhelmh /
// box_gs_vhelmh (m_vhelmholtz.f90:61-205) one eps (var 5) for all.
constexpr bool is_varop(int OP) { return OP == OP_AHELM || OP == OP_VLPL || OP == OP_VHELM; }

struct AEps {
  double a0[3], a[6];
};
template <int OP>
__device__ __forceinline__ AEps load_eps(const LevelView& L, int b, int i, int j, int k) {
  const double* e1 = boxp(L, 5, b);
  const double* e2 = boxp(L, OP == OP_AHELM ? 6 : 5, b);
  const double* e3 = boxp(L, OP == OP_AHELM ? 7 : 5, b);
  AEps E;
  const int o = off_int(L, i, j, k);
  E.a0[0] = e1[o];
  E.a0[1] = e2[o];
  E.a0[2] = e3[o];
  E.a[0] = e1[off_cell(L, i - 1, j, k)];
  E.a[1] = e1[off_cell(L, i + 1, j, k)];
  E.a[2] = e2[off_cell(L, i, j - 1, k)];
  E.a[3] = e2[off_cell(L, i, j + 1, k)];
  E.a[4] = e3[off_cell(L, i, j, k - 1)];
  E.a[5] = e3[off_cell(L, i, j, k + 1)];
  return E;
}

template <int OP>
__device__ __forceinline__ double aop_value(const OpCoef<OP>& K, const Nbr7& s, const AEps& E) {
  const double uu[6] = {s.xm, s.xp, s.ym, s.yp, s.zm, s.zp};
  const double i2[6] = {K.ix, K.ix, K.iy, K.iy, K.iz, K.iz};
  double acc = 0.0;
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const double a0 = E.a0[q >> 1];
    acc += 2 * i2[q] * a0 * E.a[q] / (a0 + E.a[q]) * (uu[q] - s.c);
  }
  if (OP == OP_VLPL) return acc;
  return acc - K.lambda * s.c;
}

template <int OP>
__device__ __forceinline__ double ags_value(const OpCoef<OP>& K, const Nbr7& s, const AEps& E, double f) {
  const double uu[6] = {s.xm, s.xp, s.ym, s.yp, s.zm, s.zp};
  const double i2[6] = {K.ix, K.ix, K.iy, K.iy, K.iz, K.iz};
  double cc[6], scu = 0.0, sc = 0.0;
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const double a0 = E.a0[q >> 1];
    cc[q] = 2 * a0 * E.a[q] / (a0 + E.a[q]) * i2[q];
  }
#pragma unroll
  for (int q = 0; q < 6; q++) scu += cc[q] * uu[q];
#pragma unroll
  for (int q = 0; q < 6; q++) sc += cc[q];
  if (OP == OP_VLPL) return (scu - f) / sc;
  return (scu - f) / (sc + K.lambda);
}

}  // namespace omg
