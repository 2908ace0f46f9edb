// omg_face.h — device helpers for the ghost-face work of the tiled kernels.
#pragma once

#include <cstddef>
#include <type_traits>

#include "omg_device.h"
#include "omg_kernels.h"

namespace omg {

typedef double v2d __attribute__((ext_vector_type(2)));
// pointer types of __builtin_amdgcn_global_load_lds (LDS-DMA)
typedef __attribute__((address_space(1))) void glb_void;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ v2d ld_nt(const double* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
}
__device__ __forceinline__ void st_nt(double* p, double x, double y) {
  v2d t = {x, y};
  __builtin_nontemporal_store(t, reinterpret_cast<v2d*>(p));
}
__device__ __forceinline__ void st_v2(double* p, double x, double y) {
  *reinterpret_cast<v2d*>(p) = v2d{x, y};
}

// The seven stencil values of two neighbouring same-colour cells of one row
// (colour indices ih, ih+1, ih even) of colour e, from a stored box in LDS:
// `so` = the other colour's interior, `gb` = the other colour's half of ghost
// face 1, consecutive faces `fstride` apart.  Five 16-B and one 8-B LDS read.
template <int NC>
__device__ __forceinline__ void pair_stencil(const double* so, const double* gb, int fstride, int e, int q,
                                             Nbr7& s0, Nbr7& s1) {
  constexpr int H = NC / 2;
  const int ih = q % H, row = q / H, j = row % NC + 1, k = row / NC + 1;
  const int p = (1 + j + k + e) & 1;   // i = 2*ih + 1 + p for the first cell
  const double2 xc = *reinterpret_cast<const double2*>(so + ih + H * row);
  const int xgi = ((j - 1) >> 1) + H * (k - 1);
  const double xs = *(p ? (ih + 2 == H ? gb + fstride + xgi : so + ih + 2 + H * row)
                        : (ih == 0 ? gb + xgi : so + ih - 1 + H * row));
  const double2 ym = *reinterpret_cast<const double2*>(j > 1 ? so + ih + H * (row - 1)
                                                           : gb + 2 * fstride + ih + H * (k - 1));
  const double2 yp = *reinterpret_cast<const double2*>(j < NC ? so + ih + H * (row + 1)
                                                            : gb + 3 * fstride + ih + H * (k - 1));
  const double2 zm = *reinterpret_cast<const double2*>(k > 1 ? so + ih + H * (row - NC)
                                                           : gb + 4 * fstride + ih + H * (j - 1));
  const double2 zp = *reinterpret_cast<const double2*>(k < NC ? so + ih + H * (row + NC)
                                                            : gb + 5 * fstride + ih + H * (j - 1));
  s0.xm = p ? xc.x : xs;
  s0.xp = p ? xc.y : xc.x;
  s1.xm = p ? xc.y : xc.x;
  s1.xp = p ? xs : xc.y;
  s0.ym = ym.x; s1.ym = ym.y;
  s0.yp = yp.x; s1.yp = yp.y;
  s0.zm = zm.x; s1.zm = zm.y;
  s0.zp = zp.x; s1.zp = zp.y;
}


// The face topology of one box (Level::d_topo): per face the kind (NbKind,
// bits 29-31) and a 29-bit argument: NB_LOCAL the neighbour's local index,
// NB_PHYS minus the boundary code of the neighbour slot, NB_REMOTE the halo
// send slot, NB_RB the coarse neighbour's local index (bits 0-24) and the
// child offset halves (bits 25-27: x, y, z), NB_RBREM none; word 6 = mask of
// the non-local faces.  A box program loads it once, first: 32 B from a
// uniform address before any store, i.e. two scalar loads that complete
// while the bulk loads stream, so the epilogue's pushes and ghost fills find
// every face's kind and target in registers (before round 4 they issued
// dependent loads of nbk / nba after the update).
struct FaceTopo {
  // two int4 values, not an int array: a runtime index into an array (even
  // through a select chain, which the compiler folds into one address)
  // keeps it in scratch memory (ScratchSize 36 in every tiled kernel)
  int4 x, y;
  __device__ __forceinline__ int word(int f) const {
    const int a = f & 1 ? x.y : x.x, c = f & 1 ? x.w : x.z, e = f & 1 ? y.y : y.x;
    return f < 2 ? a : (f < 4 ? c : e);
  }
  __device__ __forceinline__ int kind(int f) const { return (int)((unsigned)word(f) >> 29); }
  __device__ __forceinline__ int arg(int f) const { return word(f) & 0x1fffffff; }
  __device__ __forceinline__ int phys_code(int f) const { return -arg(f); }
  __device__ __forceinline__ unsigned nonlocal() const { return (unsigned)y.z; }
};
__device__ __forceinline__ FaceTopo load_topo(const LevelView& L, int b) {
  const int4* p = reinterpret_cast<const int4*>(L.topo) + 2 * (long long)b;
  FaceTopo t;
  t.x = p[0];
  t.y = p[1];
  return t;
}

// Bijective blockIdx -> box map giving each XCD one contiguous run of boxes
// (workgroups are dealt round-robin over the 8 XCDs), so Morton-close
// neighbour boxes share an L2.  rev: each XCD walks its run backwards (the
// level's passes alternate, LevelView::rev).  Speed only, never correctness.
__device__ __forceinline__ int xcd_box(int bid, int nb, int rev = 0) {
  const int q = nb >> 3, r = nb & 7, x = bid & 7, pos = bid >> 3;
  return x * q + min(x, r) + (rev ? q + (x < r) - 1 - pos : pos);
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

// Same-GPU ghost pushes of box b: for every face with a LOCAL neighbour, the
// boundary cells of the colours in `colours` go to the neighbour's ghost
// half, two consecutive slots of the half per thread as one 16-B store (the
// half of colour e on the opposite face lists exactly our colour-e boundary
// cells, in the same order).  get(i, j, k) reads our (final) interior value;
// `faces` (bit f = face f+1) limits the push to some faces.
template <int NC, class Get>
__device__ __forceinline__ void face_push_local(const LevelView& L, const FaceTopo& T, int colours, Get get,
                                                unsigned faces = 0x3f) {
  using TL = Tl<NC>;
  constexpr int H = TL::H, PF = TL::FH / 2;   // 16-B pairs per face half
  const int ncol = (colours & 1) + ((colours >> 1) & 1);
  const int c_first = (colours & 1) ? 0 : 1;
  faces &= ~T.nonlocal();
  for (int p = threadIdx.x; p < 6 * PF * ncol; p += blockDim.x) {
    const int f = p / (PF * ncol), rem = p % (PF * ncol);
    const int col = ncol == 2 ? rem / PF : c_first, r = rem % PF;
    if (!(faces >> f & 1)) continue;
    const int nb = f + 1;
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1, x1 = low ? 1 : NC;
    double v[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int hi = 2 * r + s, ah = hi % H, c = hi / H + 1;
      const int a = 2 * ah + 1 + ((col + x1 + 1 + c) & 1);
      if (d == 1) v[s] = get(x1, a, c);
      else if (d == 2) v[s] = get(a, x1, c);
      else v[s] = get(a, c, x1);
    }
    const int nbo = low ? nb + 1 : nb - 1;
    v2d* dst = reinterpret_cast<v2d*>(L.phi + (long long)T.arg(f) * L.stride + 2 * TL::HV +
                                      (nbo - 1) * TL::FS + col * TL::FH) + r;
    // default cache policy even in the streaming kernels: measured 5 % faster
    // per substep than non-temporal stores for these 1-KB face halves
    *dst = v2d{v[0], v[1]};
  }
}

// Ghost fill of phi for box b whose final interior is staged in LDS `sb`
// (Tl<NC> layout): same-GPU faces pushed (colours mask), physical ghosts
// recomputed, remote faces packed.  rb_ghost(arg, nb, a, c, x1, x2):
// refinement-boundary faces (NB_RB) too, from the fine box's own boundary
// cells and the coarse level (sides_rb; arg = the FaceTopo argument); null:
// the level has none.
template <int NC, class RbGhost = std::nullptr_t>
__device__ __forceinline__ void tile_face_fill(const LevelView& L, int b, const FaceTopo& T, const double* sb,
                                               int colours, const GcBC& bc, double* sendbuf,
                                               const RbGhost& rb_ghost = nullptr) {
  using TL = Tl<NC>;
  face_push_local<NC>(L, T, colours, [&](int i, int j, int k) { return sb[TL::oint(i, j, k)]; });
  if (!T.nonlocal()) return;
  double* u = L.phi + (long long)b * L.stride;
  for (int p = threadIdx.x; p < 6 * NC * NC; p += blockDim.x) {
    const int nb = p / (NC * NC) + 1, cell = p % (NC * NC);
    const long long fidx = (long long)b * 6 + nb - 1;
    const int kind = T.kind(nb - 1);
    if (kind == NB_LOCAL) continue;
    const int a = cell % NC + 1, c = cell / NC + 1, arg = T.arg(nb - 1);
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1, x1 = low ? 1 : NC, x2 = low ? 2 : NC - 1;
    int i1, j1, k1;
    if (d == 1) { i1 = x1; j1 = a; k1 = c; }
    else if (d == 2) { i1 = a; j1 = x1; k1 = c; }
    else { i1 = a; j1 = c; k1 = x1; }
    const double v1 = sb[TL::oint(i1, j1, k1)];
    if (kind == NB_REMOTE) {
      sendbuf[(long long)arg * NC * NC + (a - 1) + NC * (c - 1)] = v1;
    } else if (kind == NB_PHYS) {
      const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
      const int gi = TL::ogh(nb, a, c);
      u[gi] = phys_ghost(L, bc, b, fidx, nb, -arg, a, c, gi, v1, sb[TL::oint(i2, j2, k2)]);
    } else if constexpr (!std::is_same<RbGhost, std::nullptr_t>::value) {
      if (kind == NB_RB) {
        const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
        u[TL::ogh(nb, a, c)] = rb_ghost(arg, nb, a, c, v1, sb[TL::oint(i2, j2, k2)]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Face work shared by the ghost fill and the smoother epilogue: everything the
// reference's mg_fill_ghost_cells_lvl does for face nb of box b at (a, c)
// (m_ghost_cells.f90:131-175, 232-285).  `colours`: bit e set = the cells of
// colour e changed since the last fill (same-GPU neighbours receive those).
__device__ __forceinline__ void face_cell_fill(const LevelView& L, int iv, int b, int nb, int a, int c,
                                               int colours, const LevelView& C, const RBRec* rb,
                                               const GcBC& bc, double* sendbuf) {
  const int nc = L.nc;
  const long long f = (long long)b * 6 + nb - 1;
  const int kind = L.nbk[f], arg = L.nba[f];
  const bool low = nb & 1;
  const int x1 = low ? 1 : nc, x2 = low ? 2 : nc - 1;
  double* u = boxp(L, iv, b);
  if (kind == NB_LOCAL) {
    // copy_from_nb, done by the box that owns the data (push)
    if (!((colours >> ((x1 + a + c) & 1)) & 1)) return;
    boxp(L, iv, arg)[off_gh(L, low ? nb + 1 : nb - 1, a, c)] = u[off_face_cell(L, nb, x1, a, c)];
  } else if (kind == NB_REMOTE) {
    // buffer_for_nb (m_ghost_cells.f90:348-383): the whole face travels
    sendbuf[(long long)L.sendpos[f] * nc * nc + (a - 1) + (long long)nc * (c - 1)] =
        u[off_face_cell(L, nb, x1, a, c)];
  } else if (kind == NB_PHYS) {
    // box_set_gc + bc_to_gc (m_ghost_cells.f90:264-283, 665-766)
    const int gi = off_gh(L, nb, a, c);
    double bv;
    int type;
    if (bc.phi_stored && iv == 1) {
      bv = boxp(L, 2, b)[gi];
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
    u[gi] = c0 * bv + c1 * u[off_face_cell(L, nb, x1, a, c)] + c2 * u[off_face_cell(L, nb, x2, a, c)];
  } else if (kind == NB_RB) {
    // refinement boundary: box_gc_for_fine_neighbor + sides_rb
    // (m_ghost_cells.f90:287-328, 500-577, 769-861)
    const RBRec R = rb[arg];
    const double* cu = boxp(C, iv, R.coarse_idx);
    const int d = (nb + 1) >> 1;
    const int t1 = (d == 1) ? 1 : 0, t2 = (d == 3) ? 1 : 2;  // tangential dims (0-based)
    const int clayer = low ? nc : 1;                          // coarse face toward us
    const int i = (a + 1) >> 1, j = (c + 1) >> 1;
    auto T = [&](int p, int q) { return cu[off_face_cell(C, nb, clayer, R.dix[t1] + p, R.dix[t2] + q)]; };
    const double tc = T(i, j);
    const double g1 = 0.125 * (T(i + 1, j) - T(i - 1, j));
    const double g2 = 0.125 * (T(i, j + 1) - T(i, j - 1));
    double gv = ((a - 1) & 1) ? tc + g1 : tc - g1;
    gv = ((c - 1) & 1) ? gv + g2 : gv - g2;
    u[off_gh(L, nb, a, c)] = 0.5 * gv + 0.75 * u[off_face_cell(L, nb, x1, a, c)] -
                             0.25 * u[off_face_cell(L, nb, x2, a, c)];
  }
}

// The ghost fill of a 1^3 box (nc == 1), one thread: face_cell_fill's work in
// the reference's order.  In a box of one cell the second cell behind a face
// (bc_to_gc's x2, m_ghost_cells.f90:682-766) is the opposite face's ghost, and
// set_ghost_cells fills faces 1..6 in turn (m_ghost_cells.f90:232-285): the
// low face of a dimension reads the high ghost as it was before the fill, the
// high face the low ghost it just set.  So the box sets its own ghosts in that
// order, same-GPU faces by reading the neighbour's cell (no thread writes
// another box's ghosts).  A remote neighbour's ghost arrives by the unpack
// after the kernel, as with the other box sizes (a continuous high face behind
// a remote low face then reads the ghost of the fill before: not in any
// configuration here, levels of 1^3 boxes are coarse and on one rank).
__device__ __forceinline__ void box1_fill(const LevelView& L, int iv, int b, const LevelView& C, const RBRec* rb,
                                          const GcBC& bc, double* sendbuf) {
  double* u = boxp(L, iv, b);
  for (int nb = 1; nb <= 6; nb++) {
    const long long f = (long long)b * 6 + nb - 1;
    const int kind = L.nbk[f], arg = L.nba[f];
    if (kind == NB_LOCAL)
      u[off_gh(L, nb, 1, 1)] = boxp(L, iv, arg)[off_int(L, 1, 1, 1)];
    else
      face_cell_fill(L, iv, b, nb, 1, 1, 3, C, rb, bc, sendbuf);
  }
}

}  // namespace omg
