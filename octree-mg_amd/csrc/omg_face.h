// omg_face.h — device helpers for the ghost-face work of the tiled kernels.
#pragma once

#include "omg_device.h"
#include "omg_kernels.h"

namespace omg {

// Bijective blockIdx -> box map giving each XCD one contiguous run of boxes
// (workgroups are dealt round-robin over the 8 XCDs), so Morton-close
// neighbour boxes share an L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_box(int bid, int nb) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7, pos = bid >> 3;
  return x * q + min(x, r) + pos;
}

// physical ghost (set_ghost_cells + bc_to_gc, m_ghost_cells.f90:264-283, 682-766)
__device__ __forceinline__ double phys_ghost(const LevelView& L, const GcBC& bc, int b, long long f, int nb,
                                             int arg, int a, int c, int gi, double x1v, double x2v) {
  double bv;
  int type;
  if (bc.phi_stored) {
    bv = L.data[L.vstride + (long long)b * L.stride + gi];
    type = arg;
  } else if (bc.face_off && bc.face_off[f] >= 0) {
    bv = bc.face_data[bc.face_off[f] + (a - 1) + (long long)L.nc * (c - 1)];
    type = bc.face_type[f];
  } else {
    bv = bc.value[nb - 1];
    type = bc.type[nb - 1];
  }
  double c0, c1, c2;
  if (type == -10) {
    c0 = 2; c1 = -1; c2 = 0;
  } else if (type == -11) {
    c0 = L.dr[(nb - 1) >> 1] * ((nb & 1) ? -1.0 : 1.0); c1 = 1; c2 = 0;
  } else {
    c0 = 0; c1 = 2; c2 = -1;
  }
  return c0 * bv + c1 * x1v + c2 * x2v;
}

// Ghost fill of phi for box b whose final interior is staged in LDS `sb`
// (Tl<NC> layout): same-GPU faces pushed (colours mask), physical ghosts
// recomputed, remote faces packed.  Refinement boundaries are not handled
// here (levels that have them take the generic kernels).
template <int NC>
__device__ __forceinline__ void tile_face_fill(const LevelView& L, int b, const double* sb, int colours,
                                               const GcBC& bc, double* sendbuf) {
  using TL = Tl<NC>;
  double* u = L.phi + (long long)b * L.stride;
  for (int p = threadIdx.x; p < 6 * NC * NC; p += blockDim.x) {
    const int nb = p / (NC * NC) + 1, cell = p % (NC * NC);
    const int a = cell % NC + 1, c = cell / NC + 1;
    const long long fidx = (long long)b * 6 + nb - 1;
    const int kind = L.nbk[fidx], arg = L.nba[fidx];
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1, x1 = low ? 1 : NC, x2 = low ? 2 : NC - 1;
    int i1, j1, k1;
    if (d == 1) { i1 = x1; j1 = a; k1 = c; }
    else if (d == 2) { i1 = a; j1 = x1; k1 = c; }
    else { i1 = a; j1 = c; k1 = x1; }
    const double v1 = sb[TL::oint(i1, j1, k1)];
    if (kind == NB_LOCAL) {
      if ((colours >> ((i1 + j1 + k1) & 1)) & 1)
        L.phi[(long long)arg * L.stride + TL::ogh(low ? nb + 1 : nb - 1, a, c)] = v1;
    } else if (kind == NB_REMOTE) {
      sendbuf[(long long)L.sendpos[fidx] * NC * NC + (a - 1) + NC * (c - 1)] = v1;
    } else if (kind == NB_PHYS) {
      const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
      const int gi = TL::ogh(nb, a, c);
      u[gi] = phys_ghost(L, bc, b, fidx, nb, arg, a, c, gi, v1, sb[TL::oint(i2, j2, k2)]);
    }
  }
}

}  // namespace omg
