// omg_kernels.hip — gfx950 kernels of the octree-mg V-cycle hot path.
//
// Every kernel covers one whole octree level (all boxes this rank owns there)
// in one launch.  Arithmetic is fp64 and keeps the reference's association
// order term by term (compiled with -ffp-contract=off, so no FMA contraction),
// which makes every result bit-identical to the reference CPU solver.
// Reference routines are cited as path:line of FermiQ/octree-mg.
#include "omg_kernels.h"

namespace omg {

// ---------------------------------------------------------------------------
// helpers
__device__ __forceinline__ long long cix(int s, int i, int j, int k) {
  return i + (long long)s * (j + (long long)s * k);
}
__device__ __forceinline__ double* boxp(const LevelView& L, int iv, int b) {
  return L.data + (long long)(iv - 1) * L.vstride + (long long)b * L.stride;
}
// cell of face nb (1..6) at normal index `layer` and tangential (a, c)
__device__ __forceinline__ long long fcix(int s, int nb, int layer, int a, int c) {
  const int d = (nb + 1) >> 1;  // 1,1,2,2,3,3
  if (d == 1) return cix(s, layer, a, c);
  if (d == 2) return cix(s, a, layer, c);
  return cix(s, a, c, layer);
}

__device__ __forceinline__ void atomic_max_nonneg(unsigned long long* p, double v) {
  // |res| >= 0: IEEE bit patterns of non-negative doubles order like uint64
  atomicMax(p, (unsigned long long)__double_as_longlong(v));
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

// Operator value at one interior cell (box_lpl m_laplacian.f90:180-192,
// box_helmh m_helmholtz.f90:138-151, box_ahelmh m_ahelmholtz.f90:215-234).
template <int OP>
__device__ __forceinline__ double op_at(const LevelView& L, int b, const OpCoef<OP>& K, int s,
                                        long long c) {
  const double* u = boxp(L, 1, b);
  const long long sj = s, sk = (long long)s * s;
  const double u0 = u[c];
  if (OP == OP_AHELM) {
    const double* e1 = boxp(L, 5, b);
    const double* e2 = boxp(L, 6, b);
    const double* e3 = boxp(L, 7, b);
    const double a0[6] = {e1[c], e1[c], e2[c], e2[c], e3[c], e3[c]};
    const double uu[6] = {u[c - 1], u[c + 1], u[c - sj], u[c + sj], u[c - sk], u[c + sk]};
    const double aa[6] = {e1[c - 1], e1[c + 1], e2[c - sj], e2[c + sj], e3[c - sk], e3[c + sk]};
    const double i2[6] = {K.ix, K.ix, K.iy, K.iy, K.iz, K.iz};
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < 6; q++) acc += 2 * i2[q] * a0[q] * aa[q] / (a0[q] + aa[q]) * (uu[q] - u0);
    return acc - K.lambda * u0;
  }
  double v = K.ix * (u[c - 1] + u[c + 1] - 2 * u0) + K.iy * (u[c - sj] + u[c + sj] - 2 * u0) +
             K.iz * (u[c - sk] + u[c + sk] - 2 * u0);
  if (OP == OP_HELM) v = v - K.lambda * u0;
  return v;
}

// One Gauss-Seidel cell update in place (box_gs_lpl m_laplacian.f90:104-108,
// box_gs_helmh m_helmholtz.f90:98-102, box_gs_ahelmh m_ahelmholtz.f90:143-156
// with the 3D a0(5:6) index fixed).
template <int OP>
__device__ __forceinline__ void gs_update(const LevelView& L, int b, const OpCoef<OP>& K, int s,
                                          long long c) {
  double* u = boxp(L, 1, b);
  const double* f = boxp(L, 2, b);
  const long long sj = s, sk = (long long)s * s;
  if (OP == OP_AHELM) {
    const double* e1 = boxp(L, 5, b);
    const double* e2 = boxp(L, 6, b);
    const double* e3 = boxp(L, 7, b);
    const double a0[6] = {e1[c], e1[c], e2[c], e2[c], e3[c], e3[c]};
    const double uu[6] = {u[c - 1], u[c + 1], u[c - sj], u[c + sj], u[c - sk], u[c + sk]};
    const double aa[6] = {e1[c - 1], e1[c + 1], e2[c - sj], e2[c + sj], e3[c - sk], e3[c + sk]};
    const double i2[6] = {K.ix, K.ix, K.iy, K.iy, K.iz, K.iz};
    double cc[6], scu = 0.0, sc = 0.0;
#pragma unroll
    for (int q = 0; q < 6; q++) cc[q] = 2 * a0[q] * aa[q] / (a0[q] + aa[q]) * i2[q];
#pragma unroll
    for (int q = 0; q < 6; q++) scu += cc[q] * uu[q];
#pragma unroll
    for (int q = 0; q < 6; q++) sc += cc[q];
    u[c] = (scu - f[c]) / (sc + K.lambda);
    return;
  }
  u[c] = K.fac * (K.ix * (u[c + 1] + u[c - 1]) + K.iy * (u[c + sj] + u[c - sj]) +
                  K.iz * (u[c + sk] + u[c - sk]) - f[c]);
}

// ---------------------------------------------------------------------------
// Red-black Gauss-Seidel substep over a level: cell (i,j,k) is updated iff
// (i+j+k+cntr) is even (m_laplacian.f90:101-103).  One thread per updated
// cell; ghost cells are read, never written.
template <int OP>
__global__ void __launch_bounds__(256) k_gsrb(LevelView L, double lambda, int cntr) {
  const int nc = L.nc, s = nc + 2, slots = (nc + 1) >> 1;
  const long long per_box = (long long)slots * nc * nc;
  const long long total = per_box * L.n;
  const OpCoef<OP> K(L, lambda);
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(t / per_box);
    const int r = (int)(t - (long long)b * per_box);
    const int m = r % slots, row = r / slots;
    const int j = row % nc + 1, k = row / nc + 1;
    const int i = 2 - ((cntr ^ (k + j)) & 1) + 2 * m;
    if (i > nc) continue;
    gs_update<OP>(L, b, K, s, cix(s, i, j, k));
  }
}

// Lexicographic Gauss-Seidel (the reference's default mg_smoother_gs), exact
// order: one workgroup per box sweeps hyperplanes i+j+k = d in increasing d.
// Within a plane all updates are independent and see planes < d updated and
// planes > d old — the same values the i-fastest loop nest reads.
template <int OP>
__global__ void __launch_bounds__(256) k_gs_lex(LevelView L, double lambda) {
  const int nc = L.nc, s = nc + 2;
  const OpCoef<OP> K(L, lambda);
  for (int b = blockIdx.x; b < L.n; b += gridDim.x) {
    for (int d = 3; d <= 3 * nc; d++) {
      for (int p = threadIdx.x; p < nc * nc; p += blockDim.x) {
        const int j = p % nc + 1, k = p / nc + 1, i = d - j - k;
        if (i >= 1 && i <= nc) gs_update<OP>(L, b, K, s, cix(s, i, j, k));
      }
      __syncthreads();
    }
  }
}

// Operator into variable i_out (mg_apply_op / box_op), interior cells.
template <int OP>
__global__ void __launch_bounds__(256) k_box_op(LevelView L, double lambda, int i_out) {
  const int nc = L.nc, s = nc + 2;
  const long long per_box = (long long)nc * nc * nc, total = per_box * L.n;
  const OpCoef<OP> K(L, lambda);
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(t / per_box);
    const int r = (int)(t - (long long)b * per_box);
    const int i = r % nc + 1, j = (r / nc) % nc + 1, k = r / (nc * nc) + 1;
    const long long c = cix(s, i, j, k);
    boxp(L, i_out, b)[c] = op_at<OP>(L, b, K, s, c);
  }
}

// residual_box (m_multigrid.f90:426-436): res = rhs - L(phi); optionally the
// max |res| of the level (max_residual_lvl :296-311, exact in any order).
template <int OP>
__global__ void __launch_bounds__(256) k_residual(LevelView L, double lambda,
                                                  unsigned long long* maxbits) {
  const int nc = L.nc, s = nc + 2;
  const long long per_box = (long long)nc * nc * nc, total = per_box * L.n;
  const OpCoef<OP> K(L, lambda);
  double mx = 0.0;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(t / per_box);
    const int r = (int)(t - (long long)b * per_box);
    const int i = r % nc + 1, j = (r / nc) % nc + 1, k = r / (nc * nc) + 1;
    const long long c = cix(s, i, j, k);
    const double lv = op_at<OP>(L, b, K, s, c);
    const double res = boxp(L, 2, b)[c] - lv;
    boxp(L, 4, b)[c] = res;
    mx = fmax(mx, fabs(res));
  }
  if (maxbits) {
    for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_down(mx, off, 64));
    if ((threadIdx.x & 63) == 0) atomic_max_nonneg(maxbits, mx);
  }
}

// ---------------------------------------------------------------------------
// Ghost cells (mg_fill_ghost_cells_lvl, m_ghost_cells.f90:131-175): one thread
// per ghost-face cell of every box; diagonal ghosts are never touched.
__global__ void __launch_bounds__(256) k_fill_gc(LevelView L, int iv, LevelView C, const RBRec* rb,
                                                 GcBC bc, const double* recv) {
  const int nc = L.nc, s = nc + 2, nc2 = nc * nc;
  const long long total = (long long)L.n * 6 * nc2;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int cell = (int)(t % nc2);
    const int f = (int)(t / nc2);
    const int b = f / 6, nb = f % 6 + 1;
    const int a = cell % nc + 1, c = cell / nc + 1;
    const bool low = (nb & 1);
    const int g = low ? 0 : nc + 1, x1 = low ? 1 : nc, x2 = low ? 2 : nc - 1;
    double* u = boxp(L, iv, b);
    const int kind = L.nbk[f], arg = L.nba[f];
    double val;
    if (kind == NB_LOCAL) {
      // copy_from_nb / box_gc_for_neighbor (m_ghost_cells.f90:330-346,456-497)
      val = boxp(L, iv, arg)[fcix(s, nb, low ? nc : 1, a, c)];
    } else if (kind == NB_REMOTE) {
      // fill_buffered_nb (m_ghost_cells.f90:424-454)
      val = recv[(long long)arg * nc2 + (a - 1) + (long long)nc * (c - 1)];
    } else if (kind == NB_PHYS) {
      // physical boundary: box_set_gc + bc_to_gc (m_ghost_cells.f90:264-283,665-766)
      double bv;
      int type;
      if (bc.phi_stored && iv == 1) {
        bv = boxp(L, 2, b)[fcix(s, nb, g, a, c)];
        type = arg;
      } else if (bc.face_off && bc.face_off[f] >= 0) {
        bv = bc.face_data[bc.face_off[f] + (a - 1) + (long long)nc * (c - 1)];
        type = bc.face_type[f];
      } else {
        bv = bc.value[nb - 1];
        type = bc.type[nb - 1];
      }
      double c0, c1, c2;
      if (type == -10) {
        c0 = 2; c1 = -1; c2 = 0;
      } else if (type == -11) {
        c0 = L.dr[(nb - 1) >> 1] * (low ? -1.0 : 1.0); c1 = 1; c2 = 0;
      } else {
        c0 = 0; c1 = 2; c2 = -1;
      }
      val = c0 * bv + c1 * u[fcix(s, nb, x1, a, c)] + c2 * u[fcix(s, nb, x2, a, c)];
    } else {
      // refinement boundary: box_gc_for_fine_neighbor + sides_rb
      // (m_ghost_cells.f90:287-328,500-577,769-861)
      const RBRec R = rb[arg];
      const double* cu = boxp(C, iv, R.coarse_idx);
      const int d = (nb + 1) >> 1;
      const int t1 = (d == 1) ? 1 : 0, t2 = (d == 3) ? 1 : 2;  // tangential dims (0-based)
      const int clayer = low ? nc : 1;                          // coarse face toward us
      const int i = (a + 1) >> 1, j = (c + 1) >> 1;
      auto T = [&](int p, int q) {
        return cu[fcix(s, nb, clayer, R.dix[t1] + p, R.dix[t2] + q)];
      };
      const double tc = T(i, j);
      const double g1 = 0.125 * (T(i + 1, j) - T(i - 1, j));
      const double g2 = 0.125 * (T(i, j + 1) - T(i, j - 1));
      double gv = ((a - 1) & 1) ? tc + g1 : tc - g1;
      gv = ((c - 1) & 1) ? gv + g2 : gv - g2;
      val = 0.5 * gv + 0.75 * u[fcix(s, nb, x1, a, c)] - 0.25 * u[fcix(s, nb, x2, a, c)];
    }
    u[fcix(s, nb, g, a, c)] = val;
  }
}

// Halo pack: box_gc_for_neighbor of (box, nb) for every send item (box*6+nb-1).
__global__ void __launch_bounds__(256) k_pack_faces(LevelView L, int iv, const int* items, int n_items,
                                                    double* buf) {
  const int nc = L.nc, s = nc + 2, nc2 = nc * nc;
  const long long total = (long long)n_items * nc2;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / nc2), cell = (int)(t % nc2);
    const int it = items[q], b = it / 6, nb = it % 6 + 1;
    const int a = cell % nc + 1, c = cell / nc + 1;
    buf[t] = boxp(L, iv, b)[fcix(s, nb, (nb & 1) ? 1 : nc, a, c)];
  }
}

// ---------------------------------------------------------------------------
// Restriction (restrict_onto, m_restrict.f90:165-214): coarse cell =
// 0.125 * SUM(2x2x2 fine cells) accumulated column-major from +0.0.
__device__ __forceinline__ double restrict_cell(const double* fu, int s, int i, int j, int k) {
  double acc = 0.0;
#pragma unroll
  for (int kk = 0; kk < 2; kk++)
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int ii = 0; ii < 2; ii++) acc += fu[cix(s, 2 * i - 1 + ii, 2 * j - 1 + jj, 2 * k - 1 + kk)];
  return 0.125 * acc;
}

__global__ void __launch_bounds__(256) k_restrict(LevelView F, LevelView Cv, int iv, const int* pairs,
                                                  int n_pairs, const int* parent_local, const int* dixp) {
  const int nc = F.nc, s = nc + 2, hnc = nc / 2, sc = Cv.nc + 2;
  const long long per = (long long)hnc * hnc * hnc, total = per * n_pairs;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int cb = pairs[q], pb = parent_local[cb], dp = dixp[cb];
    const int i = r % hnc + 1, j = (r / hnc) % hnc + 1, k = r / (hnc * hnc) + 1;
    const double v = restrict_cell(boxp(F, iv, cb), s, i, j, k);
    boxp(Cv, iv, pb)[cix(sc, (dp & 1023) + i, ((dp >> 10) & 1023) + j, (dp >> 20) + k)] = v;
  }
}

// restrict_set_buffer (m_restrict.f90:116-163): restricted child into buffer.
__global__ void __launch_bounds__(256) k_restrict_pack(LevelView F, int iv, const int* items, int n_items,
                                                       double* buf) {
  const int nc = F.nc, s = nc + 2, hnc = nc / 2;
  const long long per = (long long)hnc * hnc * hnc, total = per * n_items;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int i = r % hnc + 1, j = (r / hnc) % hnc + 1, k = r / (hnc * hnc) + 1;
    buf[t] = restrict_cell(boxp(F, iv, items[q]), s, i, j, k);
  }
}

// restrict_onto's remote branch: items = (parent local idx, packed dix) pairs.
__global__ void __launch_bounds__(256) k_restrict_unpack(LevelView Cv, int iv, const int* items,
                                                         int n_items, int hnc, const double* buf) {
  const int sc = Cv.nc + 2;
  const long long per = (long long)hnc * hnc * hnc, total = per * n_items;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int pb = items[2 * q], dp = items[2 * q + 1];
    const int i = r % hnc + 1, j = (r / hnc) % hnc + 1, k = r / (hnc * hnc) + 1;
    boxp(Cv, iv, pb)[cix(sc, (dp & 1023) + i, ((dp >> 10) & 1023) + j, (dp >> 20) + k)] = buf[t];
  }
}

// ---------------------------------------------------------------------------
// update_coarse's parent loop (m_multigrid.f90:369-383): rhs = L(phi) + res
// on the interior, old = phi on the full box.
template <int OP>
__global__ void __launch_bounds__(256) k_coarse_rhs(LevelView Cv, double lambda, const int* parents,
                                                    int n_par) {
  const int nc = Cv.nc, s = nc + 2;
  const long long per = (long long)s * s * s, total = per * n_par;
  const OpCoef<OP> K(Cv, lambda);
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / per);
    const long long c = t % per;
    const int b = parents[q];
    const int i = (int)(c % s), j = (int)((c / s) % s), k = (int)(c / ((long long)s * s));
    if (i >= 1 && i <= nc && j >= 1 && j <= nc && k >= 1 && k <= nc) {
      const double lv = op_at<OP>(Cv, b, K, s, c);
      boxp(Cv, 2, b)[c] = lv + boxp(Cv, 4, b)[c];
    }
    boxp(Cv, 3, b)[c] = boxp(Cv, 1, b)[c];
  }
}

// correct_children's parent loop (m_multigrid.f90:392-399): res = phi - old.
__global__ void __launch_bounds__(256) k_sub_parents(LevelView Cv, const int* parents, int n_par) {
  const int s = Cv.nc + 2;
  const long long per = (long long)s * s * s, total = per * n_par;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = parents[t / per];
    const long long c = t % per;
    boxp(Cv, 4, b)[c] = boxp(Cv, 1, b)[c] - boxp(Cv, 3, b)[c];
  }
}

// mg_prolong_sparse (m_prolong.f90:159-240) value at fine cell (fi,fj,fk).
__device__ __forceinline__ double prolong_cell(const double* cu, int sc, int dx, int dy, int dz,
                                               int fi, int fj, int fk) {
  const int ic = ((fi + 1) >> 1) + dx, jc = ((fj + 1) >> 1) + dy, kc = ((fk + 1) >> 1) + dz;
  const long long c = cix(sc, ic, jc, kc);
  const long long sj = sc, sk = (long long)sc * sc;
  const double f0 = 0.25 * cu[c];
  const double fx = 0.25 * cu[(fi & 1) ? c - 1 : c + 1];
  const double fy = 0.25 * cu[(fj & 1) ? c - sj : c + sj];
  const double fz = 0.25 * cu[(fk & 1) ? c - sk : c + sk];
  return f0 + fx + fy + fz;
}

// mg_prolong + prolong_onto (m_prolong.f90:51-85,124-156) for local parents.
__global__ void __launch_bounds__(256) k_prolong(LevelView Cv, LevelView F, int iv, int iv_to, int add,
                                                 const int* pairs, int n_pairs, const int* parent_local,
                                                 const int* dixp) {
  const int nc = F.nc, s = nc + 2, sc = Cv.nc + 2;
  const long long per = (long long)nc * nc * nc, total = per * n_pairs;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int fb = pairs[q], pb = parent_local[fb], dp = dixp[fb];
    const int i = r % nc + 1, j = (r / nc) % nc + 1, k = r / (nc * nc) + 1;
    const double v = prolong_cell(boxp(Cv, iv, pb), sc, dp & 1023, (dp >> 10) & 1023, dp >> 20, i, j, k);
    double* dst = boxp(F, iv_to, fb) + cix(s, i, j, k);
    *dst = add ? *dst + v : v;
  }
}

// prolong_set_buffer (m_prolong.f90:91-121): items = (parent idx, packed dix).
__global__ void __launch_bounds__(256) k_prolong_pack(LevelView Cv, int iv, int nc, const int* items,
                                                      int n_items, double* buf) {
  const int sc = Cv.nc + 2;
  const long long per = (long long)nc * nc * nc, total = per * n_items;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int pb = items[2 * q], dp = items[2 * q + 1];
    const int i = r % nc + 1, j = (r / nc) % nc + 1, k = r / (nc * nc) + 1;
    buf[t] = prolong_cell(boxp(Cv, iv, pb), sc, dp & 1023, (dp >> 10) & 1023, dp >> 20, i, j, k);
  }
}

__global__ void __launch_bounds__(256) k_prolong_unpack(LevelView F, int iv_to, int add, const int* items,
                                                        int n_items, const double* buf) {
  const int nc = F.nc, s = nc + 2;
  const long long per = (long long)nc * nc * nc, total = per * n_items;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int i = r % nc + 1, j = (r / nc) % nc + 1, k = r / (nc * nc) + 1;
    double* dst = boxp(F, iv_to, items[q]) + cix(s, i, j, k);
    *dst = add ? *dst + buf[t] : buf[t];
  }
}

// ---------------------------------------------------------------------------
// get_sum (m_multigrid.f90:278-294): per-leaf sequential interior sums ...
__global__ void __launch_bounds__(256) k_box_sums(LevelView L, int iv, const int* leaves, int n_leaves,
                                                  double* out) {
  const int nc = L.nc, s = nc + 2;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n_leaves; q += gridDim.x * blockDim.x) {
    const double* u = boxp(L, iv, leaves[q]);
    double acc = 0.0;
    for (int k = 1; k <= nc; k++)
      for (int j = 1; j <= nc; j++) {
        const double* row = u + cix(s, 0, j, k);
        for (int i = 1; i <= nc; i++) acc += row[i];
      }
    out[q] = acc;
  }
}

// ... then acc = acc + w * box_sum in my_leaves order, one thread (exact order).
__global__ void k_seq_sum(const double* box_sums, int n, double w, double* acc) {
  __shared__ double stage[1024];
  double a = *acc;
  for (int base = 0; base < n; base += 1024) {
    const int m = min(1024, n - base);
    for (int q = threadIdx.x; q < m; q += blockDim.x) stage[q] = box_sums[base + q];
    __syncthreads();
    if (threadIdx.x == 0)
      for (int q = 0; q < m; q++) a = a + w * stage[q];
    __syncthreads();
  }
  if (threadIdx.x == 0) *acc = a;
}

// subtract_mean's update (m_multigrid.f90:262-275).
__global__ void __launch_bounds__(256) k_subtract(LevelView L, int iv, const double* mean, int ghosts) {
  const int nc = L.nc, s = nc + 2;
  const long long per = (long long)s * s * s, total = per * L.n;
  const double m = *mean;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(t / per);
    const long long c = t % per;
    if (!ghosts) {
      const int i = (int)(c % s), j = (int)((c / s) % s), k = (int)(c / ((long long)s * s));
      if (i < 1 || i > nc || j < 1 || j > nc || k < 1 || k > nc) continue;
    }
    double* u = boxp(L, iv, b) + c;
    *u = *u - m;
  }
}

// Whole-box copy / zero of one variable (FMG's old = phi and phi = 0).
__global__ void __launch_bounds__(256) k_copy_var(LevelView L, int src, int dst) {
  const long long per = (long long)(L.nc + 2) * (L.nc + 2) * (L.nc + 2), total = per * L.n;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(t / per);
    const long long c = t % per;
    boxp(L, dst, b)[c] = src > 0 ? boxp(L, src, b)[c] : 0.0;
  }
}

// ---------------------------------------------------------------------------
// launchers
static inline unsigned grid_for(long long work, int block = 256) {
  long long g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 2048 * 8) g = 2048 * 8;
  return (unsigned)g;
}

void launch_gsrb(const LevelView& L, int op, double lambda, int cntr, hipStream_t st) {
  const long long work = (long long)((L.nc + 1) / 2) * L.nc * L.nc * L.n;
  if (work == 0) return;
  const unsigned g = grid_for(work);
  switch (op) {
    case OP_HELM: k_gsrb<OP_HELM><<<g, 256, 0, st>>>(L, lambda, cntr); break;
    case OP_AHELM: k_gsrb<OP_AHELM><<<g, 256, 0, st>>>(L, lambda, cntr); break;
    default: k_gsrb<OP_LPL><<<g, 256, 0, st>>>(L, lambda, cntr); break;
  }
}

void launch_gs_lex(const LevelView& L, int op, double lambda, hipStream_t st) {
  if (L.n == 0) return;
  const unsigned g = (unsigned)std::min(L.n, 65535);
  const int block = L.nc * L.nc >= 256 ? 256 : ((L.nc * L.nc + 63) / 64) * 64;
  switch (op) {
    case OP_HELM: k_gs_lex<OP_HELM><<<g, block, 0, st>>>(L, lambda); break;
    case OP_AHELM: k_gs_lex<OP_AHELM><<<g, block, 0, st>>>(L, lambda); break;
    default: k_gs_lex<OP_LPL><<<g, block, 0, st>>>(L, lambda); break;
  }
}

void launch_box_op(const LevelView& L, int op, double lambda, int i_out, hipStream_t st) {
  const long long work = (long long)L.nc * L.nc * L.nc * L.n;
  if (work == 0) return;
  const unsigned g = grid_for(work);
  switch (op) {
    case OP_HELM: k_box_op<OP_HELM><<<g, 256, 0, st>>>(L, lambda, i_out); break;
    case OP_AHELM: k_box_op<OP_AHELM><<<g, 256, 0, st>>>(L, lambda, i_out); break;
    default: k_box_op<OP_LPL><<<g, 256, 0, st>>>(L, lambda, i_out); break;
  }
}

void launch_residual(const LevelView& L, int op, double lambda, unsigned long long* maxbits,
                     hipStream_t st) {
  const long long work = (long long)L.nc * L.nc * L.nc * L.n;
  if (work == 0) return;
  const unsigned g = grid_for(work);
  switch (op) {
    case OP_HELM: k_residual<OP_HELM><<<g, 256, 0, st>>>(L, lambda, maxbits); break;
    case OP_AHELM: k_residual<OP_AHELM><<<g, 256, 0, st>>>(L, lambda, maxbits); break;
    default: k_residual<OP_LPL><<<g, 256, 0, st>>>(L, lambda, maxbits); break;
  }
}

void launch_fill_gc(const LevelView& L, int iv, const LevelView& C, const RBRec* rb, const GcBC& bc,
                    const double* recv, hipStream_t st) {
  const long long work = (long long)L.n * 6 * L.nc * L.nc;
  if (work == 0) return;
  k_fill_gc<<<grid_for(work), 256, 0, st>>>(L, iv, C, rb, bc, recv);
}

void launch_pack_faces(const LevelView& L, int iv, const int* items, int n, double* buf, hipStream_t st) {
  const long long work = (long long)n * L.nc * L.nc;
  if (work == 0) return;
  k_pack_faces<<<grid_for(work), 256, 0, st>>>(L, iv, items, n, buf);
}

void launch_restrict(const LevelView& F, const LevelView& C, int iv, const int* pairs, int n_pairs,
                     const int* parent_local, const int* dixp, hipStream_t st) {
  const int h = F.nc / 2;
  const long long work = (long long)h * h * h * n_pairs;
  if (work == 0) return;
  k_restrict<<<grid_for(work), 256, 0, st>>>(F, C, iv, pairs, n_pairs, parent_local, dixp);
}

void launch_restrict_pack(const LevelView& F, int iv, const int* items, int n, double* buf,
                          hipStream_t st) {
  const int h = F.nc / 2;
  const long long work = (long long)h * h * h * n;
  if (work == 0) return;
  k_restrict_pack<<<grid_for(work), 256, 0, st>>>(F, iv, items, n, buf);
}

void launch_restrict_unpack(const LevelView& C, int iv, const int* items, int n, int hnc,
                            const double* buf, hipStream_t st) {
  const long long work = (long long)hnc * hnc * hnc * n;
  if (work == 0) return;
  k_restrict_unpack<<<grid_for(work), 256, 0, st>>>(C, iv, items, n, hnc, buf);
}

void launch_coarse_rhs(const LevelView& C, int op, double lambda, const int* parents, int n_par,
                       hipStream_t st) {
  const long long s = C.nc + 2, work = s * s * s * n_par;
  if (work == 0) return;
  const unsigned g = grid_for(work);
  switch (op) {
    case OP_HELM: k_coarse_rhs<OP_HELM><<<g, 256, 0, st>>>(C, lambda, parents, n_par); break;
    case OP_AHELM: k_coarse_rhs<OP_AHELM><<<g, 256, 0, st>>>(C, lambda, parents, n_par); break;
    default: k_coarse_rhs<OP_LPL><<<g, 256, 0, st>>>(C, lambda, parents, n_par); break;
  }
}

void launch_sub_parents(const LevelView& C, const int* parents, int n_par, hipStream_t st) {
  const long long s = C.nc + 2, work = s * s * s * n_par;
  if (work == 0) return;
  k_sub_parents<<<grid_for(work), 256, 0, st>>>(C, parents, n_par);
}

void launch_prolong(const LevelView& C, const LevelView& F, int iv, int iv_to, int add, const int* pairs,
                    int n_pairs, const int* parent_local, const int* dixp, hipStream_t st) {
  const long long work = (long long)F.nc * F.nc * F.nc * n_pairs;
  if (work == 0) return;
  k_prolong<<<grid_for(work), 256, 0, st>>>(C, F, iv, iv_to, add, pairs, n_pairs, parent_local, dixp);
}

void launch_prolong_pack(const LevelView& C, int iv, int nc, const int* items, int n, double* buf,
                         hipStream_t st) {
  const long long work = (long long)nc * nc * nc * n;
  if (work == 0) return;
  k_prolong_pack<<<grid_for(work), 256, 0, st>>>(C, iv, nc, items, n, buf);
}

void launch_prolong_unpack(const LevelView& F, int iv_to, int add, const int* items, int n,
                           const double* buf, hipStream_t st) {
  const long long work = (long long)F.nc * F.nc * F.nc * n;
  if (work == 0) return;
  k_prolong_unpack<<<grid_for(work), 256, 0, st>>>(F, iv_to, add, items, n, buf);
}

void launch_box_sums(const LevelView& L, int iv, const int* leaves, int n, double* out, hipStream_t st) {
  if (n == 0) return;
  k_box_sums<<<grid_for(n, 64), 64, 0, st>>>(L, iv, leaves, n, out);
}

void launch_seq_sum(const double* box_sums, int n, double w, double* acc, hipStream_t st) {
  if (n == 0) return;
  k_seq_sum<<<1, 256, 0, st>>>(box_sums, n, w, acc);
}

void launch_subtract(const LevelView& L, int iv, const double* mean, int ghosts, hipStream_t st) {
  const long long s = L.nc + 2, work = s * s * s * L.n;
  if (work == 0) return;
  k_subtract<<<grid_for(work), 256, 0, st>>>(L, iv, mean, ghosts);
}

void launch_copy_var(const LevelView& L, int src, int dst, hipStream_t st) {
  const long long s = L.nc + 2, work = s * s * s * L.n;
  if (work == 0) return;
  k_copy_var<<<grid_for(work), 256, 0, st>>>(L, src, dst);
}

}  // namespace omg
