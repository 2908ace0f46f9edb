// omg_gsrb.h — the red-black substep of one 16^3 (or 8, 4, 2) box, as a device
// function of a workgroup: used by k_gsrb_tile (omg_sweep.hip) and by the
// single-workgroup coarse-level program (omg_tiles.hip).
#pragma once

#include "omg_face.h"

namespace omg {

// LDS doubles gsrb_box<NC> needs
template <int NC>
constexpr int gsrb_lds() { return 2 * (NC / 2) * NC * NC + 6 * (NC / 2) * NC; }

// One substep on box b (the workgroup's BS threads), LDS at `lds`.
// PRE: the caller has already put colour 1-e and the colour-(1-e) ghost
// halves into LDS (k_prolong_smooth), only rhs is loaded here.
template <int NC, int BS>
struct GsrbRhs {
  static constexpr int NP2 = ((NC / 2) * NC * NC / 2 + BS - 1) / BS;   // double2 cell pairs per thread
  double2 v[NP2];
};

// colour e of rhs for box b, into registers (issued early by callers that
// have other latency to hide)
template <int NC, int BS, int NT>
__device__ __forceinline__ void gsrb_load_rhs(const LevelView& L, int e, int b, GsrbRhs<NC, BS>& fr) {
  constexpr int HV = (NC / 2) * NC * NC;
  const double* __restrict__ f = L.data + L.vstride + (long long)b * L.stride;
#pragma unroll
  for (int r = 0; r < GsrbRhs<NC, BS>::NP2; r++) {
    const int q2 = threadIdx.x + BS * r;
    if (q2 < HV / 2) {
      const double2* fp = reinterpret_cast<const double2*>(f + e * HV) + q2;
      if (NT) {
        const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(fp));
        fr.v[r] = make_double2(t.x, t.y);
      } else {
        fr.v[r] = *fp;
      }
    }
  }
}

// The coarse side of refinement-boundary faces (fine side of sides_rb):
// the level below and the per-face records; rb == nullptr: none on this level.
// gv / gv_mode: the coarse part of every refinement-boundary ghost of the
// level ([box][face][cell], rb_gv below), which stays fixed while the coarse
// level does: 1 = the smoother computes it and stores it there, 2 = it reads
// it instead of the five coarse operands (0: neither)
struct RbSide {
  LevelView C;
  const RBRec* rb;
  double* gv;
  int gv_mode;
};

// Refinement-boundary ghost (box_gc_for_fine_neighbor + sides_rb,
// m_ghost_cells.f90:287-328, 500-577, 769-861) of face nb at (a, c) from the
// two boundary cells v1 (layer x1) and v2 (layer x2) of the fine box.
// The coarse operands: the coarse cell facing (a, c) and its four in-face
// neighbours.  They stay fixed while the fine level is smoothed (nothing
// writes the coarse level then), so the smoother loads them early.
struct RbCoarse {
  double tc, m1, p1, m2, p2;
};
__device__ __forceinline__ RbCoarse rb_coarse_load(const LevelView& L, const RbSide& R, const RBRec& rec, int nb,
                                                   int a, int c) {
  const double* cu = R.C.phi + (long long)rec.coarse_idx * R.C.stride;
  const int d = (nb + 1) >> 1;
  const int t1 = (d == 1) ? 1 : 0, t2 = (d == 3) ? 1 : 2;
  const int clayer = (nb & 1) ? L.nc : 1;
  const int i = (a + 1) >> 1, j = (c + 1) >> 1;
  auto T = [&](int p, int q) { return cu[off_face_cell(R.C, nb, clayer, rec.dix[t1] + p, rec.dix[t2] + q)]; };
  return RbCoarse{T(i, j), T(i - 1, j), T(i + 1, j), T(i, j - 1), T(i, j + 1)};
}
// the coarse part of the ghost (the interpolated coarse value), then the
// ghost from it and the fine box's two boundary cells
__device__ __forceinline__ double rb_gv(const RbCoarse& t, int a, int c) {
  const double g1 = 0.125 * (t.p1 - t.m1);
  const double g2 = 0.125 * (t.p2 - t.m2);
  double gv = ((a - 1) & 1) ? t.tc + g1 : t.tc - g1;
  return ((c - 1) & 1) ? gv + g2 : gv - g2;
}
__device__ __forceinline__ double rb_ghost_gv(double gv, double v1, double v2) {
  return 0.5 * gv + 0.75 * v1 - 0.25 * v2;
}
__device__ __forceinline__ double rb_ghost_from(const RbCoarse& t, int a, int c, double v1, double v2) {
  return rb_ghost_gv(rb_gv(t, a, c), v1, v2);
}
// the RBRec of an NB_RB face from its FaceTopo argument (coarse index in bits
// 0-24, child offset halves in bits 25-27; pack_topo)
__device__ __forceinline__ RBRec rb_unpack(const LevelView& L, int targ) {
  RBRec r;
  r.coarse_idx = targ & 0x1ffffff;
#pragma unroll
  for (int d = 0; d < 3; d++) r.dix[d] = ((targ >> (25 + d)) & 1) * (L.nc >> 1);
  return r;
}
__device__ __forceinline__ double rb_ghost(const LevelView& L, const RbSide& R, int targ, int nb, int a, int c,
                                           double v1, double v2) {
  return rb_ghost_from(rb_coarse_load(L, R, rb_unpack(L, targ), nb, a, c), a, c, v1, v2);
}

// Variable-coefficient operators read eps (var 5; vars 5..7 for the
// anisotropic one) at the cell and at its six neighbours from HBM / L2, at
// the same slots the stencil reads phi from LDS (same layout, same colour).
template <int OP>
struct EpsPtr {
  const double* v[3];
  __device__ __forceinline__ EpsPtr(const LevelView& L, int b) {
    const long long bo = (long long)b * L.stride;
    v[0] = L.data + 4 * L.vstride + bo;
    v[1] = OP == OP_AHELM ? L.data + 5 * L.vstride + bo : v[0];
    v[2] = OP == OP_AHELM ? L.data + 6 * L.vstride + bo : v[0];
  }
};

// eps of the cell pair (colour e, colour-relative slot q of the first cell)
// and of its neighbours, as load_eps gives them cell by cell; the neighbour
// slots are pair_stencil's, in the eps variables (unused loads fold away)
template <int NC, int OP>
__device__ __forceinline__ void pair_eps(const LevelView& L, int b, int e, int q, AEps& E0, AEps& E1) {
  constexpr int H = NC / 2, HV = H * NC * NC, FH = H * NC, FS = 2 * FH;
  const EpsPtr<OP> EP(L, b);
  const int o = 1 - e;
  Nbr7 n0[3], n1[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    if (d > 0 && OP != OP_AHELM) {
      n0[d] = n0[0];
      n1[d] = n1[0];
      continue;
    }
    pair_stencil<NC>(EP.v[d] + o * HV, EP.v[d] + 2 * HV + o * FH, FS, e, q, n0[d], n1[d]);
    const double2 cv = *reinterpret_cast<const double2*>(EP.v[d] + e * HV + q);
    E0.a0[d] = cv.x;
    E1.a0[d] = cv.y;
  }
  E0.a[0] = n0[0].xm; E0.a[1] = n0[0].xp; E0.a[2] = n0[1].ym; E0.a[3] = n0[1].yp; E0.a[4] = n0[2].zm; E0.a[5] = n0[2].zp;
  E1.a[0] = n1[0].xm; E1.a[1] = n1[0].xp; E1.a[2] = n1[1].ym; E1.a[3] = n1[1].yp; E1.a[4] = n1[2].zm; E1.a[5] = n1[2].zp;
  if (OP != OP_AHELM) {
    E0.a0[1] = E0.a0[2] = E0.a0[0];
    E1.a0[1] = E1.a0[2] = E1.a0[0];
  }
}

// box operator of a same-colour cell pair (box_lpl / box_helmh / box_vlpl /
// box_vhelmh / box_ahelmh): s0, s1 hold phi; the eps pair is read for the
// variable-coefficient operators.  NC == 2 has one cell per row: cell by cell.
template <int NC, int OP>
__device__ __forceinline__ void op_pair(const OpCoef<OP>& K, const LevelView& L, int b, int e, int q,
                                        const Nbr7& s0, const Nbr7& s1, double& v0, double& v1) {
  if constexpr (is_varop(OP)) {
    AEps E0, E1;
    if constexpr ((NC / 2) % 2 == 0) {
      pair_eps<NC, OP>(L, b, e, q, E0, E1);
    } else {
      int i, j, k;
      Tl<NC>::decode(e * Tl<NC>::HV + q, i, j, k);
      E0 = load_eps<OP>(L, b, i, j, k);
      Tl<NC>::decode(e * Tl<NC>::HV + q + 1, i, j, k);
      E1 = load_eps<OP>(L, b, i, j, k);
    }
    v0 = aop_value<OP>(K, s0, E0);
    v1 = aop_value<OP>(K, s1, E1);
  } else {
    v0 = op_value<OP>(K, s0);
    v1 = op_value<OP>(K, s1);
  }
}

// RB: the level has refinement-boundary faces (a separate instantiation keeps
// their interpolation out of the plain kernels)
template <int NC, int OP, int BS, int NT, bool PRE = false, bool RB = false>
__device__ __forceinline__ void gsrb_box(const LevelView& L, double lambda, int e, int colours, const GcBC& bc,
                                         double* __restrict__ sendbuf, const double* __restrict__ shift, int b,
                                         double* lds, const GsrbRhs<NC, BS>* pre_rhs = nullptr,
                                         const RbSide* rbs = nullptr) {
  constexpr int H = NC / 2, HV = H * NC * NC, FH = H * NC, FS = 2 * FH;
  constexpr int NP2 = GsrbRhs<NC, BS>::NP2;
  double* so = lds;                            // colour 1-e of the interior
  double* se = lds + HV;                       // colour e, updated
  double* sg = lds + 2 * HV;                   // colour 1-e halves of the ghost faces
  const int tid = threadIdx.x, o = 1 - e;
  const long long boff = (long long)b * L.stride;
  double* __restrict__ u = L.phi + boff;
  const OpCoef<OP> K(L, lambda);
  // the box's face kinds and targets (scalar loads, complete during the
  // stream-in; the pushes and the ghost fill below read them from registers)
  const FaceTopo T = load_topo(L, b);

  // Refinement-boundary faces: the coarse operands are issued right after
  // the stream-in (below), so the ghost fill after the substep finds them in
  // registers (the face's coarse box and child offset are in T: one level of
  // loads instead of kind -> record -> coarse cells).
  constexpr bool RBP = RB;
  constexpr int NF = 6 * NC * NC, NPF = RBP ? (NF + BS - 1) / BS : 1;
  RbCoarse rt[NPF];

  // ---- stream in: colour 1-e, its ghost halves, colour e of rhs ----------
  if (!PRE) {
    const v2d* src = reinterpret_cast<const v2d*>(u + o * HV);
    v2d* dst = reinterpret_cast<v2d*>(so);
    const double m = shift ? *shift : 0.0;
    for (int q = tid; q < HV / 2; q += BS) {
      v2d x = NT >= 2 ? __builtin_nontemporal_load(src + q) : src[q];
      if (shift) {
        x.x = x.x - m;
        x.y = x.y - m;
      }
      dst[q] = x;
    }
    for (int q = tid; q < 3 * FH; q += BS) {   // 6 faces x FH/2 double2
      const int nb = q / (FH / 2), r = q % (FH / 2);
      const v2d* gp = reinterpret_cast<const v2d*>(u + 2 * HV + nb * FS + o * FH) + r;
      v2d x = NT >= 2 ? __builtin_nontemporal_load(gp) : *gp;
      if (shift) {
        x.x = x.x - m;
        x.y = x.y - m;
      }
      reinterpret_cast<v2d*>(sg + nb * FH)[r] = x;
    }
  }
  GsrbRhs<NC, BS> frs;
  if (pre_rhs)
    frs = *pre_rhs;
  else
    gsrb_load_rhs<NC, BS, NT>(L, e, b, frs);
  const double2* fr = frs.v;
  if constexpr (RBP) {
#pragma unroll
    for (int r = 0; r < NPF; r++) {
      const int p = tid + BS * r;
      if (p >= NF) continue;
      const int f = p / (NC * NC), cell = p % (NC * NC);
      if (T.kind(f) != NB_RB) continue;
      if (rbs->gv_mode == 2)   // the stored coarse part (in tc)
        rt[r].tc = rbs->gv[((long long)b * 6 + f) * (NC * NC) + cell];
      else
        rt[r] = rb_coarse_load(L, *rbs, rb_unpack(L, T.arg(f)), f + 1, cell % NC + 1, cell / NC + 1);
    }
  }
  __syncthreads();

  // ---- colour e update ----------------------------------------------------
  // Each thread updates two neighbouring cells of one row (colour indices ih,
  // ih+1 with ih even; NC >= 4).  Their y/z neighbours are aligned
  // colour-(1-e) pairs and their x neighbours one aligned pair plus one single
  // value: five 16-B and one 8-B LDS read per two cells, the lanes of a wave
  // on consecutive 16-B slots.
#pragma unroll
  for (int r = 0; r < NP2; r++) {
    const int q2 = tid + BS * r;
    if (q2 >= HV / 2) continue;
    double2 nv;
    if constexpr (H % 2 == 0) {
      const int q = 2 * q2, ih = q % H, row = q / H, j = row % NC + 1, k = row / NC + 1;
      const int p = (1 + j + k + e) & 1;   // i = 2*ih + 1 + p for the first cell
      const double2 xc = *reinterpret_cast<const double2*>(so + ih + H * row);
      const int xgi = ((j - 1) >> 1) + H * (k - 1);   // x ghosts of this row
      const double* xs_ptr = p ? (ih + 2 == H ? sg + FH + xgi : so + ih + 2 + H * row)
                               : (ih == 0 ? sg + xgi : so + ih - 1 + H * row);
      const double xs = *xs_ptr;
      const double2 ym = *reinterpret_cast<const double2*>(j > 1 ? so + ih + H * (row - 1)
                                                               : sg + 2 * FH + ih + H * (k - 1));
      const double2 yp = *reinterpret_cast<const double2*>(j < NC ? so + ih + H * (row + 1)
                                                                : sg + 3 * FH + ih + H * (k - 1));
      const double2 zm = *reinterpret_cast<const double2*>(k > 1 ? so + ih + H * (row - NC)
                                                               : sg + 4 * FH + ih + H * (j - 1));
      const double2 zp = *reinterpret_cast<const double2*>(k < NC ? so + ih + H * (row + NC)
                                                                : sg + 5 * FH + ih + H * (j - 1));
      Nbr7 s0, s1;
      s0.xm = p ? xc.x : xs;
      s0.xp = p ? xc.y : xc.x;
      s1.xm = p ? xc.y : xc.x;
      s1.xp = p ? xs : xc.y;
      s0.ym = ym.x; s1.ym = ym.y;
      s0.yp = yp.x; s1.yp = yp.y;
      s0.zm = zm.x; s1.zm = zm.y;
      s0.zp = zp.x; s1.zp = zp.y;
      if constexpr (is_varop(OP)) {
        AEps E0, E1;
        pair_eps<NC, OP>(L, b, e, q, E0, E1);
        nv = make_double2(ags_value<OP>(K, s0, E0, fr[r].x), ags_value<OP>(K, s1, E1, fr[r].y));
      } else {
        nv = make_double2(gs_value<OP>(K, s0, fr[r].x), gs_value<OP>(K, s1, fr[r].y));
      }
    } else {   // NC == 2: one cell per row
      double v[2];
#pragma unroll
      for (int s = 0; s < 2; s++) {
        const int q = 2 * q2 + s;
        const int ih = q % H, row = q / H, j = row % NC + 1, k = row / NC + 1;
        const int i = 2 * ih + 1 + ((1 + j + k + e) & 1);
        const int tj = (i - 1) >> 1;
        Nbr7 st;
        st.xm = i > 1 ? so[((i - 2) >> 1) + H * row] : sg[0 * FH + ((j - 1) >> 1) + H * (k - 1)];
        st.xp = i < NC ? so[(i >> 1) + H * row] : sg[1 * FH + ((j - 1) >> 1) + H * (k - 1)];
        st.ym = j > 1 ? so[tj + H * (row - 1)] : sg[2 * FH + tj + H * (k - 1)];
        st.yp = j < NC ? so[tj + H * (row + 1)] : sg[3 * FH + tj + H * (k - 1)];
        st.zm = k > 1 ? so[tj + H * (row - NC)] : sg[4 * FH + tj + H * (j - 1)];
        st.zp = k < NC ? so[tj + H * (row + NC)] : sg[5 * FH + tj + H * (j - 1)];
        if constexpr (is_varop(OP))
          v[s] = ags_value<OP>(K, st, load_eps<OP>(L, b, i, j, k), s ? fr[r].y : fr[r].x);
        else
          v[s] = gs_value<OP>(K, st, s ? fr[r].y : fr[r].x);
      }
      nv = make_double2(v[0], v[1]);
    }
    reinterpret_cast<double2*>(se)[q2] = nv;
    double2* up = reinterpret_cast<double2*>(u + e * HV) + q2;
    if (NT) {
      v2d t = {nv.x, nv.y};
      __builtin_nontemporal_store(t, reinterpret_cast<v2d*>(up));
    } else
      *up = nv;
  }
  __syncthreads();

  // ---- ghost fill after the substep ---------------------------------------
  auto cellv = [&](int i, int j, int k) {
    const int idx = ((i - 1) >> 1) + H * ((j - 1) + NC * (k - 1));
    return ((i + j + k) & 1) == e ? se[idx] : so[idx];
  };
  face_push_local<NC>(L, T, colours, cellv, 0x3fu);
  if (!T.nonlocal()) return;
  auto fill_cell = [&](int p, const RbCoarse* rc) {
    const int nb = p / (NC * NC) + 1, cell = p % (NC * NC);
    const int kind = T.kind(nb - 1), arg = T.arg(nb - 1);
    if (kind == NB_LOCAL) return;
    const long long fidx = (long long)b * 6 + nb - 1;
    const int a = cell % NC + 1, c = cell / NC + 1;
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1;
    // boundary cell x1 (and x2) of this face
    const int x1 = low ? 1 : NC, x2 = low ? 2 : NC - 1;
    int i1, j1, k1;
    if (d == 1) { i1 = x1; j1 = a; k1 = c; }
    else if (d == 2) { i1 = a; j1 = x1; k1 = c; }
    else { i1 = a; j1 = c; k1 = x1; }
    const double v1 = cellv(i1, j1, k1);
    // colours bit 2: the physical / refinement-boundary ghosts of colour e
    // only (the split fused down-step: other boxes of the level read the
    // colour 1-e halves as they stood before this substep, k_face_gc forms
    // them afterwards)
    const bool keep = (colours & 4) && (((low ? 0 : NC + 1) + a + c) & 1) != e;
    if (kind == NB_REMOTE) {
      sendbuf[(long long)arg * NC * NC + (a - 1) + NC * (c - 1)] = v1;
    } else if (keep) {
      if constexpr (RBP) {   // (the stored coarse part is still wanted)
        if (kind == NB_RB && rbs->gv_mode == 1) rbs->gv[fidx * (NC * NC) + cell] = rb_gv(*rc, a, c);
      }
    } else if (kind == NB_PHYS) {
      const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
      const int gi = off_gh(L, nb, a, c);
      u[gi] = phys_ghost(L, bc, b, fidx, nb, -arg, a, c, gi, v1, cellv(i2, j2, k2));
    } else if (RB && kind == NB_RB) {
      const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
      const double v2 = cellv(i2, j2, k2);
      if constexpr (RBP) {
        const double gv = rbs->gv_mode == 2 ? rc->tc : rb_gv(*rc, a, c);
        if (rbs->gv_mode == 1) rbs->gv[fidx * (NC * NC) + cell] = gv;
        u[off_gh(L, nb, a, c)] = rb_ghost_gv(gv, v1, v2);
      } else {
        u[off_gh(L, nb, a, c)] = rb_ghost(L, *rbs, arg, nb, a, c, v1, v2);
      }
    }   // NB_RBREM: the caller's refinement-boundary exchange (finish_rb)
  };
  if constexpr (RBP) {
#pragma unroll
    for (int r = 0; r < NPF; r++)
      if (tid + BS * r < NF) fill_cell(tid + BS * r, &rt[r]);
  } else {
    for (int p = tid; p < NF; p += BS) fill_cell(p, nullptr);
  }
}

// Lexicographic Gauss-Seidel on one box with the box in LDS (the reference's
// mg_smoother_gs, m_laplacian.f90:67-81): phi with its ghost faces and rhs are
// read once, hyperplanes i+j+k = d run in increasing d on LDS (all updates of
// a plane are independent and see planes < d updated, planes > d old: the
// values the i-fastest loop nest reads), the interior is written back.
template <int NC>
constexpr int gs_lex_lds() { return (NC + 2) * (NC + 2) * (NC + 2) + NC * NC * NC; }

template <int OP, int NC>
__device__ __forceinline__ void gs_lex_box(const LevelView& L, double lambda, int b, double* lds) {
  constexpr int S = NC + 2, S3 = S * S * S, N3 = NC * NC * NC;
  double* P = lds;         // phi(0:nc+1)^3, i fastest (edges and corners unused)
  double* R = lds + S3;    // rhs(1:nc)^3
  const OpCoef<OP> K(L, lambda);
  double* u = boxp(L, 1, b);
  const double* f = boxp(L, 2, b);
  for (int q = threadIdx.x; q < S3; q += blockDim.x) {
    const int i = q % S, j = (q / S) % S, k = q / (S * S);
    const int nbd = (i == 0 || i == S - 1) + (j == 0 || j == S - 1) + (k == 0 || k == S - 1);
    const double* up = u + off_cell(L, i, j, k);
    P[q] = nbd <= 1 ? *up : 0.0;
  }
  for (int q = threadIdx.x; q < N3; q += blockDim.x) {
    const double* fp = f + off_int(L, q % NC + 1, (q / NC) % NC + 1, q / (NC * NC) + 1);
    R[q] = *fp;
  }
  __syncthreads();
  for (int d = 3; d <= 3 * NC; d++) {
    for (int p = threadIdx.x; p < NC * NC; p += blockDim.x) {
      const int j = p % NC + 1, k = p / NC + 1, i = d - j - k;
      if (i < 1 || i > NC) continue;
      const int c = i + S * (j + S * k);
      Nbr7 st;
      st.c = P[c];
      st.xm = P[c - 1];
      st.xp = P[c + 1];
      st.ym = P[c - S];
      st.yp = P[c + S];
      st.zm = P[c - S * S];
      st.zp = P[c + S * S];
      const double fv = R[(i - 1) + NC * ((j - 1) + NC * (k - 1))];
      if constexpr (is_varop(OP))
        P[c] = ags_value<OP>(K, st, load_eps<OP>(L, b, i, j, k), fv);
      else
        P[c] = gs_value<OP>(K, st, fv);
    }
    __syncthreads();
  }
  for (int q = threadIdx.x; q < N3; q += blockDim.x) {
    const int i = q % NC + 1, j = (q / NC) % NC + 1, k = q / (NC * NC) + 1;
    u[off_int(L, i, j, k)] = P[i + S * (j + S * k)];
  }
  __syncthreads();
}

}  // namespace omg
