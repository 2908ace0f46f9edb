// omg_tiles.hip — LDS-tiled fused level kernels around the smoother.
//
//  k_resid_restrict: update_coarse's fine-level part (src/m_multigrid.f90:
//    356-363): residual_box over every box of the level, then mg_restrict_lvl
//    of phi and of the residual onto the parents, in one pass over phi.
//  k_prolong_fill:   correct_children's fine-level part + the ghost fill the
//    V-cycle runs right after it (:216-219): phi += prolong(res_coarse)
//    (mg_prolong_sparse, m_prolong.f90:159-240), then the new boundary values
//    go to the neighbours' ghost faces (both colours) and physical ghosts are
//    recomputed.  Nothing reads fine ghosts during the launch: race-free.
//  k_box_sums3 / k_seq_sum3: get_sum (:278-294) in the reference's exact
//    sequential order, with wide loads and the products off the add chain.
#include "omg_face.h"
#include "omg_gsrb.h"
#include "omg_kernels.h"

namespace omg {

// threads per 16^3 box of k_prolong_smooth; waves per SIMD it is compiled for
constexpr int kPsBS16 = 512, kPsWaves = 8;
// get_sum box sums: leaves per wave (a wave per 64 threads), rows of a box per
// chunk, non-temporal loads (plain sums; the fused rhs subtract loads and
// stores with the default policy)
constexpr int kSumsLPW = 32, kSumsR = 4;
constexpr bool kSumsNT = true, kSubNTLd = false, kSubNTSt = false;

template <int NC, int OP, int BS>
__device__ __forceinline__ void resid_restrict_core(const LevelView& F, const LevelView& Cv, double lambda,
                                                    unsigned long long* maxbits, int restrict_on,
                                                    const int* parent_local, const int* dixp, int b, double* sb,
                                                    const v2d* fr);

template <int NC, int OP, int BS>
__device__ __forceinline__ void resid_restrict_box(const LevelView& F, const LevelView& Cv, double lambda,
                                                   unsigned long long* maxbits, int restrict_on,
                                                   const int* parent_local, const int* dixp, int b, double* sb) {
  using TL = Tl<NC>;
  constexpr int NST = TL::NST, HV = TL::HV, NR = (HV + BS - 1) / BS;
  const int tid = threadIdx.x;
  const long long boff = (long long)b * F.stride;
  const double* __restrict__ u = F.phi + boff;
  const double* __restrict__ f = F.data + F.vstride + boff;
  for (int q = tid; q < NST / 2; q += BS) reinterpret_cast<v2d*>(sb)[q] = ld_nt(u + 2 * q);
  v2d fr[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 < HV) fr[r] = ld_nt(f + 2 * q2);
  }
  __syncthreads();
  resid_restrict_core<NC, OP, BS>(F, Cv, lambda, maxbits, restrict_on, parent_local, dixp, b, sb, fr);
}

// The residual and the restriction of box b from its tile in LDS (phi with
// its ghost faces, Tl<NC> layout) and rhs in registers (pairs q2 = tid + BS*r).
template <int NC, int OP, int BS>
__device__ __forceinline__ void resid_restrict_core(const LevelView& F, const LevelView& Cv, double lambda,
                                                    unsigned long long* maxbits, int restrict_on,
                                                    const int* parent_local, const int* dixp, int b, double* sb,
                                                    const v2d* fr) {
  using TL = Tl<NC>;
  constexpr int HV = TL::HV, FH = TL::FH, FS = TL::FS, NR = (HV + BS - 1) / BS, HN = NC / 2;
  const int tid = threadIdx.x;
  double* __restrict__ res = F.data + 3 * F.vstride + (long long)b * F.stride;

  // residual_box (m_multigrid.f90:426-436) with box_lpl / box_helmh, two
  // same-colour cells per thread and step (pair q2: colour q2 / (HV/2))
  const OpCoef<OP> K(F, lambda);
  double mx = 0.0;
  double2 rv[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 >= HV) continue;
    const int e = q2 >= HV / 2, o = 1 - e;
    Nbr7 s0, s1;
    if constexpr (HN % 2 == 0) {
      pair_stencil<NC>(sb + o * HV, sb + 2 * HV + o * FH, FS, e, 2 * q2 - e * HV, s0, s1);
    } else {   // NC == 2: one cell per row
      int i, j, k;
      TL::decode(2 * q2, i, j, k);
      s0.xm = sb[TL::ocell(i - 1, j, k)]; s0.xp = sb[TL::ocell(i + 1, j, k)];
      s0.ym = sb[TL::ocell(i, j - 1, k)]; s0.yp = sb[TL::ocell(i, j + 1, k)];
      s0.zm = sb[TL::ocell(i, j, k - 1)]; s0.zp = sb[TL::ocell(i, j, k + 1)];
      TL::decode(2 * q2 + 1, i, j, k);
      s1.xm = sb[TL::ocell(i - 1, j, k)]; s1.xp = sb[TL::ocell(i + 1, j, k)];
      s1.ym = sb[TL::ocell(i, j - 1, k)]; s1.yp = sb[TL::ocell(i, j + 1, k)];
      s1.zm = sb[TL::ocell(i, j, k - 1)]; s1.zp = sb[TL::ocell(i, j, k + 1)];
    }
    const double2 cc = reinterpret_cast<const double2*>(sb)[q2];
    s0.c = cc.x;
    s1.c = cc.y;
    double l0, l1;
    op_pair<NC, OP>(K, F, b, e, 2 * q2 - e * HV, s0, s1, l0, l1);
    const double r0 = fr[r].x - l0, r1 = fr[r].y - l1;
    mx = amax(mx, amax(fabs(r0), fabs(r1)));
    rv[r] = make_double2(r0, r1);
    st_nt(res + 2 * q2, r0, r1);
  }
  if (maxbits) launch_max<BS>(maxbits, mx);
  if (!restrict_on || parent_local[b] < 0) return;

  // restrict_onto (m_restrict.f90:165-214): phi, then res, onto the parent's
  // octant at offset dix (sequential column-major 8-cell sum from +0.0)
  const int pb = parent_local[b], dp = dixp[b];
  const int dx = dp & 1023, dy = (dp >> 10) & 1023, dz = dp >> 20;
  const long long poff = (long long)pb * Cv.stride;
  for (int pass = 0; pass < 2; pass++) {
    double* __restrict__ dst = pass == 0 ? Cv.phi + poff : Cv.data + 3 * Cv.vstride + poff;
    for (int q = tid; q < HN * HN * HN; q += BS) {
      const int i = q % HN + 1, j = (q / HN) % HN + 1, k = q / (HN * HN) + 1;
      double acc = 0.0;
#pragma unroll
      for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int jj = 0; jj < 2; jj++)
#pragma unroll
          for (int ii = 0; ii < 2; ii++) acc += sb[TL::oint(2 * i - 1 + ii, 2 * j - 1 + jj, 2 * k - 1 + kk)];
      dst[off_int(Cv, dx + i, dy + j, dz + k)] = 0.125 * acc;
    }
    if (pass == 0) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < NR; r++) {
        const int q2 = tid + BS * r;
        if (q2 < HV) reinterpret_cast<double2*>(sb)[q2] = rv[r];
      }
      __syncthreads();
    }
  }
}

template <int NC, int OP, int BS>
__global__ void __launch_bounds__(BS) k_resid_restrict(LevelView F, LevelView Cv, double lambda,
                                                       unsigned long long* maxbits, int restrict_on,
                                                       const int* parent_local, const int* dixp,
                                                       const int* list) {
  __shared__ double sb[Tl<NC>::NST];
  const int q = xcd_box(blockIdx.x, gridDim.x, F.rev);
  resid_restrict_box<NC, OP, BS>(F, Cv, lambda, maxbits, restrict_on, parent_local, dixp, list ? list[q] : q, sb);
}

// Tile offset of the cell at layer v along axis d and tangential (a, c)
// (the two other axes in increasing order)
template <int NC>
__device__ __forceinline__ int sr_int(int d, int v, int a, int c) {
  return d == 0 ? Tl<NC>::oint(v, a, c) : (d == 1 ? Tl<NC>::oint(a, v, c) : Tl<NC>::oint(a, c, v));
}
// Tile offset of the ghost of the neighbour cell (layer nl along d, (a, c))
// past tangential axis t (0: a's axis, 1: c's axis), on the low side if lo
template <int NC>
__device__ __forceinline__ int sr_edge(int d, int t, bool lo, int nl, int a, int c) {
  const int t1 = d == 0 ? 1 : 0, t2 = d == 2 ? 1 : 2, ax = t == 0 ? t1 : t2;
  const int fn = 2 * ax + (lo ? 1 : 2);
  // (i, j, k) of the cell, then its coordinates on face fn
  const int i = d == 0 ? nl : a, j = d == 1 ? nl : (d == 0 ? a : c), k = d == 2 ? nl : c;
  return ax == 0 ? Tl<NC>::ogh(fn, j, k) : (ax == 1 ? Tl<NC>::ogh(fn, i, k) : Tl<NC>::ogh(fn, i, j));
}

// k_smooth_resid loads colour 1 and rhs with the default policy (non-temporal
// measured 85 us slower at 512^3: the neighbours' loads of the same lines then
// miss L2), and issues the neighbour loads before the bulk loads (10 us
// faster)
__device__ __forceinline__ v2d sr_ld(const double* p) { return *reinterpret_cast<const v2d*>(p); }

// The last down-smoothing substep of a level fused with update_coarse's
// residual + restriction (k_smooth_resid).  The substep updates colour 0
// from colour 1, which it does not change, so the colour-0 ghost values the
// residual needs (the neighbours' new boundary cells) are recomputed here from
// colour-1 data that is final: our boundary layer, the neighbour's second
// layer, the neighbour's rhs and, at face edges, the neighbour's own ghosts.
// Same operands, same gs_value: bit-identical to the neighbour's own update.
// Levels whose faces are all same-GPU boxes, Laplacian / Helmholtz, NC 16/8.
// Round 4: boxes with physical or refinement-boundary faces fuse too (BCK:
// 0 = the level has neither, 1 = physical faces, 2 = refinement-boundary
// faces too; separate instantiations keep the plain kernel's registers).  Their
// ghosts on such faces follow from the box's own final cells (bc_to_gc,
// sides_rb with the coarse face), both colour halves, formed in LDS after the
// update for the residual; only the colour-0 halves go to HBM.  The colour-1
// halves must stay as the substep read them: a same-GPU neighbour's edge
// tap (gedge) reads them in this launch.  The host marks the level's ghosts
// stale; the correction of the up-step forms them again before any read.
template <int NC, int OP, int BS, int BCK = 0>
__global__ void __launch_bounds__(BS) k_smooth_resid(LevelView F, LevelView Cv, double lambda, int restrict_on,
                                                     const int* parent_local, const int* dixp,
                                                     const int* list, GcBC bc, const double* __restrict__ rbgv) {
  using TL = Tl<NC>;
  constexpr int H = NC / 2, HV = TL::HV, FH = TL::FH, FS = TL::FS, NR = (HV + BS - 1) / BS;
  constexpr int NG = (6 * FH + BS - 1) / BS;   // colour-0 ghost cells per thread
  __shared__ double sb[TL::NST];
  const int tid = threadIdx.x, bq = xcd_box(blockIdx.x, gridDim.x, F.rev), b = list ? list[bq] : bq;
  const FaceTopo T = load_topo(F, b);
  const long long boff = (long long)b * F.stride;
  double* __restrict__ u = F.phi + boff;
  const double* __restrict__ f = F.data + F.vstride + boff;
  v2d fr[NR];
  auto bulk_loads = [&]() {
    // colour 1 and the colour-1 halves of the ghost faces
    for (int q = tid; q < HV / 2; q += BS)
      reinterpret_cast<v2d*>(sb + HV)[q] = sr_ld(u + HV + 2 * q);
    for (int q = tid; q < 3 * FH; q += BS) {
      const int nb = q / (FH / 2), r = q % (FH / 2);
      reinterpret_cast<v2d*>(sb + 2 * HV + nb * FS + FH)[r] = sr_ld(u + 2 * HV + nb * FS + FH + 2 * r);
    }
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const int q2 = tid + BS * r;
      if (q2 < HV) fr[r] = sr_ld(f + 2 * q2);
    }
  };
  // the neighbour-side operands of our colour-0 ghost cells: N's cell X at
  // (layer nl, a, c) has neighbours deep (N's second layer), across (our
  // boundary layer, LDS), and tangentially N's boundary cells (our colour-1
  // ghosts, LDS) or, past the face edge, N's ghosts on its side faces
  double gdeep[NG] = {}, grhs[NG] = {}, gedge[NG][2] = {};
#pragma unroll
  for (int g = 0; g < NG; g++) {
    const int p = tid + BS * g;
    if (p >= 6 * FH) continue;
    const int nb = p / FH + 1, hi = p % FH, ah = hi % H, c = hi / H + 1;
    // (physical and refinement-boundary faces have no neighbour box: their
    // argument is a BC code or a coarse box index, not a box of this level)
    if (BCK && T.kind(nb - 1) != NB_LOCAL) continue;
    const bool low = nb & 1;
    const int gl = low ? 0 : NC + 1, a = 2 * ah + 1 + ((gl + 1 + c) & 1);
    const int d = (nb - 1) >> 1, nl = low ? NC : 1;
    const long long noff = (long long)T.arg(nb - 1) * F.stride;
    const double* un = F.phi + noff;
    gdeep[g] = un[sr_int<NC>(d, low ? NC - 1 : 2, a, c)];
    grhs[g] = F.data[F.vstride + noff + sr_int<NC>(d, nl, a, c)];
    // a tangential neighbour outside N's face (edges; two at corners)
    gedge[g][0] = gedge[g][1] = 0.0;
    const bool ea = a == 1 || a == NC, ec = c == 1 || c == NC;
    if (ea) gedge[g][0] = un[sr_edge<NC>(d, 0, a == 1, nl, a, c)];
    if (ec) {
      const double e = un[sr_edge<NC>(d, 1, c == 1, nl, a, c)];
      if (ea) gedge[g][1] = e; else gedge[g][0] = e;
    }
  }
  // the coarse operands of refinement-boundary faces (sides_rb): the coarse
  // boxes across them are leaves, which the restriction below never writes
  constexpr int NF = 6 * NC * NC, NPF = (NF + BS - 1) / BS;
  RbCoarse rt[BCK == 2 ? NPF : 1];
  if constexpr (BCK == 2) {
    if (T.nonlocal()) {
#pragma unroll
      for (int r = 0; r < NPF; r++) {
        const int p = tid + BS * r;
        if (p >= NF) continue;
        const int f = p / (NC * NC), cell = p % (NC * NC);
        if (T.kind(f) != NB_RB) continue;
        if (rbgv)   // the coarse parts the level's substeps stored (RbSide::gv)
          rt[r].tc = rbgv[((long long)b * 6 + f) * (NC * NC) + cell];
        else
          rt[r] = rb_coarse_load(F, RbSide{Cv, nullptr}, rb_unpack(F, T.arg(f)), f + 1, cell % NC + 1, cell / NC + 1);
      }
    }
  }
  bulk_loads();
  __syncthreads();

  const OpCoef<OP> K(F, lambda);
  // ---- colour-0 update (the substep), pairs q2 < HV/2 ----
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 >= HV / 2) continue;
    Nbr7 s0, s1;
    pair_stencil<NC>(sb + HV, sb + 2 * HV + FH, FS, 0, 2 * q2, s0, s1);
    const double v0 = gs_value<OP>(K, s0, fr[r].x), v1 = gs_value<OP>(K, s1, fr[r].y);
    reinterpret_cast<double2*>(sb)[q2] = make_double2(v0, v1);
    st_nt(u + 2 * q2, v0, v1);
  }
  // physical / refinement-boundary faces read our second layer (colour 0,
  // just updated by other threads)
  if (BCK && T.nonlocal()) __syncthreads();
  // ---- the neighbours' new colour-0 boundary cells = our colour-0 ghosts ----
#pragma unroll
  for (int g = 0; g < NG; g++) {
    const int p = tid + BS * g;
    if (p >= 6 * FH) continue;
    const int nb = p / FH + 1, hi = p % FH, ah = hi % H, c = hi / H + 1;
    const bool low = nb & 1;
    const int gl = low ? 0 : NC + 1, a = 2 * ah + 1 + ((gl + 1 + c) & 1);
    const int d = (nb - 1) >> 1;
    if (BCK && T.kind(nb - 1) != NB_LOCAL) continue;   // (the loop below)
    const double across = sb[sr_int<NC>(d, low ? 1 : NC, a, c)];
    const bool ea = a == 1 || a == NC;
    // along the face normal, then the two tangential axes (t1 < t2)
    const double dm = low ? gdeep[g] : across, dp = low ? across : gdeep[g];
    const double am = a == 1 ? gedge[g][0] : sb[TL::ogh(nb, a - 1, c)];
    const double ap = a == NC ? gedge[g][0] : sb[TL::ogh(nb, a + 1, c)];
    const double ce = ea ? gedge[g][1] : gedge[g][0];
    const double cm = c == 1 ? ce : sb[TL::ogh(nb, a, c - 1)];
    const double cp = c == NC ? ce : sb[TL::ogh(nb, a, c + 1)];
    Nbr7 s;
    s.xm = d == 0 ? dm : am;
    s.xp = d == 0 ? dp : ap;
    s.ym = d == 1 ? dm : (d == 0 ? am : cm);
    s.yp = d == 1 ? dp : (d == 0 ? ap : cp);
    s.zm = d == 2 ? dm : cm;
    s.zp = d == 2 ? dp : cp;
    sb[2 * HV + (nb - 1) * FS + hi] = gs_value<OP>(K, s, grhs[g]);
  }
  // physical / refinement-boundary faces: both colours of their ghosts from
  // our final cells (the coarse operands of refinement-boundary cells were
  // loaded with the neighbour operands above)
  if (BCK && T.nonlocal()) {
#pragma unroll
    for (int r = 0; r < NPF; r++) {
      const int p = tid + BS * r;
      if (p >= NF) continue;
      const int f = p / (NC * NC), cell = p % (NC * NC), nb = f + 1, kind = T.kind(f);
      if (kind == NB_LOCAL) continue;
      const int a = cell % NC + 1, c = cell / NC + 1, d = f >> 1;
      const bool low = nb & 1;
      const double x1 = sb[sr_int<NC>(d, low ? 1 : NC, a, c)], x2 = sb[sr_int<NC>(d, low ? 2 : NC - 1, a, c)];
      const int gi = TL::ogh(nb, a, c);
      double gv = 0.0;   // (other kinds: unreachable, the host fuses none)
      if (kind == NB_PHYS)
        gv = phys_ghost(F, bc, b, (long long)b * 6 + f, nb, T.phys_code(f), a, c, gi, x1, x2);
      else if constexpr (BCK == 2)
        if (kind == NB_RB) gv = rb_ghost_gv(rbgv ? rt[r].tc : rb_gv(rt[r], a, c), x1, x2);
      sb[gi] = gv;
      if (gi < 2 * HV + f * FS + FH) u[gi] = gv;   // the colour-0 half to HBM
    }
  }
  __syncthreads();
  // our new colour-0 boundary cells to the neighbours' colour-0 ghost halves
  face_push_local<NC>(F, T, 1, [&](int i, int j, int k) { return sb[TL::oint(i, j, k)]; });
  resid_restrict_core<NC, OP, BS>(F, Cv, lambda, nullptr, restrict_on, parent_local, dixp, b, sb, fr);
}

// SUB: correct_children's `res = phi - old` on the parent (m_multigrid.f90:
// 392-399) is formed here while the parent data is loaded; each child writes
// the res cells of its own octant and of the parent ghost faces next to it
// (every stored cell of the parent exactly once over its 8 children).
template <int NC>
constexpr int prolong_cb() { return ((NC / 2 + 2) * (NC / 2 + 2) * (NC / 2 + 2) + 1) & ~1; }

// The parent's octant + one face layer around it into LDS `cb` (the
// prolongation of the octant never reads edges or corners; EDGES also loads
// the edge cells the parent stores, for the siblings' boundary cells).  Loads
// are all issued before any store: the res stores alias the phi/old loads, so
// an interleaved loop would serialise every load behind the previous store.
template <int NC, int BS, bool SUB, bool EDGES = false>
__device__ __forceinline__ void load_parent_octant(const LevelView& Cv, int iv, int pb, int dx, int dy, int dz,
                                                   double* cb) {
  auto ld = [](const double* p) { return *p; };
  constexpr int CB = NC / 2 + 2, N = CB * CB * CB, NQ = (N + BS - 1) / BS;
  const int tid = threadIdx.x;
  const int n1 = Cv.nc + 1;
  double rv[NQ];
  int off[NQ];
  unsigned store = 0;
#pragma unroll
  for (int r = 0; r < NQ; r++) {
    const int q = tid + BS * r;
    off[r] = -1;
    if (q >= N) continue;
    const int p = q % CB, s = (q / CB) % CB, t = q / (CB * CB);
    const int nbnd = (p == 0 || p == CB - 1) + (s == 0 || s == CB - 1) + (t == 0 || t == CB - 1);
    const int x = dx + p, y = dy + s, z = dz + t;
    const int nghost = (x == 0 || x == n1) + (y == 0 || y == n1) + (z == 0 || z == n1);
    if (EDGES ? (nbnd == 3 || nghost >= 2) : nbnd >= 2) continue;
    const int o = off_cell(Cv, x, y, z);
    off[r] = o;
    if (SUB) {
      rv[r] = ld(boxp(Cv, 1, pb) + o) - ld(boxp(Cv, 3, pb) + o);
      if (nbnd == 0 || (nbnd == 1 && nghost)) store |= 1u << r;
    } else {
      rv[r] = ld(boxp(Cv, iv, pb) + o);
    }
  }
#pragma unroll
  for (int r = 0; r < NQ; r++) {
    if (off[r] < 0) continue;
    cb[tid + BS * r] = rv[r];
    if (SUB && (store >> r & 1)) boxp(Cv, 4, pb)[off[r]] = rv[r];
  }
}

// skip1: a red-black substep of colour 1 follows (the V-cycle's up-smoothing,
// m_multigrid.f90:216-222), which overwrites colour 1 and its ghosts without
// reading them, so boxes whose six faces all have same-GPU neighbours correct
// and push colour 0 only.  Boxes with a physical face (bc_to_gc reads the
// colour-1 boundary cell) or a remote face (whole faces travel) do both.
// save_old: FMG's `old = phi` of this level (m_multigrid.f90:127-129) for the
// interior, from the pre-correction values loaded here anyway (the caller
// copies the ghost faces before the launch; needs !skip1: every pair loaded).
template <int NC, int BS, bool SUB, bool RB = false>
__device__ __forceinline__ void prolong_fill_box(const LevelView& Cv, const LevelView& F, int iv,
                                                 const int* parent_local, const int* dixp, const GcBC& bc,
                                                 double* sendbuf, int b, double* lds, bool skip1,
                                                 bool save_old = false, const RBRec* rb = nullptr) {
  using TL = Tl<NC>;
  constexpr int HV = TL::HV, NR = (HV + BS - 1) / BS, HN = NC / 2, CB = HN + 2;
  double* cb = lds;                     // the parent's octant + one face layer around it
  double* sb = lds + prolong_cb<NC>();  // the corrected fine interior
  const int tid = threadIdx.x;
  const FaceTopo T = load_topo(F, b);
  const int pb = parent_local[b], dp = dixp[b];
  const int dx = dp & 1023, dy = (dp >> 10) & 1023, dz = dp >> 20;
  const bool only0 = skip1 && !T.nonlocal();
  const int npair = only0 ? HV / 2 : HV;
  double* __restrict__ u = F.phi + (long long)b * F.stride;
  v2d old[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 < npair) old[r] = ld_nt(u + 2 * q2);
  }
  load_parent_octant<NC, BS, SUB>(Cv, iv, pb, dx, dy, dz, cb);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 >= npair) continue;
    double nv[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int q = 2 * q2 + s;
      int i, j, k;
      TL::decode(q, i, j, k);
      const int ic = (i + 1) >> 1, jc = (j + 1) >> 1, kc = (k + 1) >> 1;   // 1..HN inside the octant
      const int c0 = ic + CB * (jc + CB * kc);
      const double f0 = 0.25 * cb[c0];
      const double fx = 0.25 * cb[(i & 1) ? c0 - 1 : c0 + 1];
      const double fy = 0.25 * cb[(j & 1) ? c0 - CB : c0 + CB];
      const double fz = 0.25 * cb[(k & 1) ? c0 - CB * CB : c0 + CB * CB];
      const double o = s ? old[r].y : old[r].x;
      nv[s] = o + (f0 + fx + fy + fz);
      sb[q] = nv[s];
    }
    st_nt(u + 2 * q2, nv[0], nv[1]);
    if (save_old) st_nt(F.data + 2 * F.vstride + (long long)b * F.stride + 2 * q2, old[r].x, old[r].y);
  }
  __syncthreads();
  if constexpr (RB) {
    // refinement boundaries: the coarse neighbour lives on Cv, the level the
    // correction came from (fill_refinement_bnd + sides_rb, m_ghost_cells.f90:
    // 287-328, 769-861), now final for this up-step
    const RbSide rbs{Cv, rb};
    tile_face_fill<NC>(F, b, T, sb, only0 ? 1 : 3, bc, sendbuf,
                       [&](int arg, int nb, int a, int c, double v1, double v2) {
                         return rb_ghost(F, rbs, arg, nb, a, c, v1, v2);
                       });
  } else {
    tile_face_fill<NC>(F, b, T, sb, only0 ? 1 : 3, bc, sendbuf);
  }
}

template <int NC, int BS, bool SUB, bool RB = false>
__global__ void __launch_bounds__(BS) k_prolong_fill(LevelView Cv, LevelView F, int iv,
                                                     const int* parent_local, const int* dixp, GcBC bc,
                                                     double* sendbuf, int skip1, const int* list, int save_old,
                                                     const RBRec* rb) {
  __shared__ double lds[prolong_cb<NC>() + Tl<NC>::HV * 2];
  const int t = xcd_box(blockIdx.x, gridDim.x, F.rev);
  prolong_fill_box<NC, BS, SUB, RB>(Cv, F, iv, parent_local, dixp, bc, sendbuf, list ? list[t] : t, lds,
                                    skip1 != 0, save_old != 0, rb);
}

// correct_children + fill + the first up-smoothing substep in one pass
// (m_multigrid.f90:216-222 with smooth_boxes :404-424, substep 1 = colour 1).
// The box adds the prolonged correction to both colours, and forms the ghost
// values the substep reads (colour 0) itself: a neighbour's new boundary value
// is its old one (still in our ghost slot) plus the prolongation at that cell,
// computed from the neighbour's parent exactly as the neighbour computes it.
// Colour-0 ghost halves in HBM are left stale: nothing reads them before the
// next substep has pushed colour 0 again.
template <int NC>
__device__ __forceinline__ double prolong_at(const LevelView& Cv, int pc, const int dix[3], int fi, int fj,
                                             int fk) {
  // mg_prolong_sparse (m_prolong.f90:219-233) of res = phi - old of parent pc
  const int ic = ((fi + 1) >> 1) + dix[0], jc = ((fj + 1) >> 1) + dix[1], kc = ((fk + 1) >> 1) + dix[2];
  const double* ph = boxp(Cv, 1, pc);
  const double* ol = boxp(Cv, 3, pc);
  auto r = [&](int x, int y, int z) {
    const int o = off_cell(Cv, x, y, z);
    return ph[o] - ol[o];
  };
  const double f0 = 0.25 * r(ic, jc, kc);
  const double fx = 0.25 * r((fi & 1) ? ic - 1 : ic + 1, jc, kc);
  const double fy = 0.25 * r(ic, (fj & 1) ? jc - 1 : jc + 1, kc);
  const double fz = 0.25 * r(ic, jc, (fk & 1) ? kc - 1 : kc + 1);
  return f0 + fx + fy + fz;
}

// the parent octant (phase 1-2) shares its space with the ghost halves
// (phase 3 on): 4 workgroups of 16^3 boxes fit one CU
template <int NC>
constexpr int prolong_smooth_lds() {
  return 2 * Tl<NC>::HV + (prolong_cb<NC>() > 6 * Tl<NC>::FH ? prolong_cb<NC>() : 6 * Tl<NC>::FH);
}

// RB (round 4): the level has refinement-boundary faces (one GPU): their
// colour-0 ghosts are formed like the physical ones, from the corrected
// boundary cells and the coarse face (sides_rb; Cv is final by now), and the
// substep's epilogue fills them (gsrb_box's RB form)
template <int NC, int OP, int BS, bool RB = false>
__device__ __forceinline__ void prolong_smooth_box(const LevelView& Cv, const LevelView& F, double lambda,
                                                   const int* parent_local, const int* dixp, const GcBC& bc,
                                                   int one_child, const uint8_t* push0, int b, double* lds,
                                                   double* rbgv = nullptr) {
  using TL = Tl<NC>;
  constexpr int HV = TL::HV, FH = TL::FH, NR = (HV + BS - 1) / BS, HN = NC / 2, CB = HN + 2;
  double* sb = lds;                     // both colours of the corrected interior (so | se of gsrb_box)
  double* sg = lds + 2 * HV;            // colour-0 ghost halves, 6 x FH
  double* cb = sg;                      // parent octant + face layer (res), until phase 3
  const int tid = threadIdx.x;
  const FaceTopo T = load_topo(F, b);
  const int pb = parent_local[b], dp = dixp[b];
  const int dix[3] = {dp & 1023, (dp >> 10) & 1023, dp >> 20};
  // The substep overwrites colour 1 without reading it (gs_value has no
  // centre term), so colour 1's corrected values are dead, except where a
  // physical (refinement-boundary) face's colour-0 ghost takes its boundary
  // cell x1 (bc_to_gc, sides_rb).  Boxes without such a face prolong colour 0
  // only.
  bool phys = false;
#pragma unroll
  for (int nb = 0; nb < 6; nb++) phys |= T.kind(nb) == NB_PHYS || (RB && T.kind(nb) == NB_RB);
  const int npair = phys ? HV : HV / 2;
  // all loads that do not depend on LDS first (colour 0; a physical-face box
  // reads its colour 1 when it corrects it)
  constexpr int NR0 = (HV / 2 + BS - 1) / BS;
  double* __restrict__ u = F.phi + (long long)b * F.stride;
  v2d old[NR0];
#pragma unroll
  for (int r = 0; r < NR0; r++) {
    const int q2 = tid + BS * r;
    if (q2 < HV / 2) old[r] = ld_nt(u + 2 * q2);
  }
  // The old values in our colour-0 ghost halves (og below) go by LDS-DMA into
  // the colour-1 half of the tile, unused until the substep in a box without
  // a physical face: no registers held across the parent's loads.
  const bool og_lds = !phys && 6 * FH <= HV;   // fits the colour-1 half (NC >= 8)
  if (og_lds && tid < 3 * FH) {   // 16-B chunks of the six face halves
    const int q = 2 * tid;
    __builtin_amdgcn_global_load_lds((glb_void*)(u + 2 * HV + (q / FH) * TL::FS + q % FH),
                                     (lds_void*)(sb + HV + 2 * (tid & ~63)), 16, 0, 0);
  }
  // ---- colour-0 ghost values from same-GPU neighbours: the neighbour's
  // old boundary value (still in our ghost slot) + its prolongation
  constexpr int NG = (6 * FH + BS - 1) / BS;
  double gv[NG], rva[NG], rvc[NG];
  unsigned defm = 0, rima = 0, rimc = 0;   // from the tile after it is loaded; rim taps
  unsigned ocm = 0;                        // one_child faces: og added after the barrier
#pragma unroll
  for (int g = 0; g < NG; g++) {
    const int q = tid + BS * g;
    gv[g] = 0.0;
    if (q >= 6 * FH) continue;
    const int nb = q / FH + 1, rr = q % FH;
    // (per-lane loads here: they are issued before any store, and the kernel
    // has no VGPRs to spare for the face words)
    if (F.nbk[(long long)b * 6 + nb - 1] != NB_LOCAL) continue;
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1, gpos = low ? 0 : NC + 1;
    const int c = rr / HN + 1, ah = rr % HN;
    const int a = 2 * ah + 1 + ((1 + gpos + c) & 1);   // the colour-0 ghost cell (a, c)
    // the neighbour's cell: along d at NC (low face) or 1 (high face)
    const int xn = low ? NC : 1;
    int fi, fj, fk;
    if (d == 1) { fi = xn; fj = a; fk = c; }
    else if (d == 2) { fi = a; fj = xn; fk = c; }
    else { fi = a; fj = c; fk = xn; }
    const double og = og_lds ? 0.0 : u[TL::ogh(nb, a, c)];
    if (!one_child) {
      // From the tile once it is loaded: a sibling's cells are the parent's
      // own; a neighbour parent's boundary layer is our parent's ghost layer
      // (same phi and old bits, hence same res), its ghost layer our parent's
      // boundary.  Only where a tangential tap leaves both parents' stored
      // cells (the parent's edge) is the neighbour parent's face ghost read.
      gv[g] = og;
      defm |= 1u << g;
      const bool sib = low ? dix[d - 1] == HN : dix[d - 1] == 0;
      if (sib) continue;
      const int pn = Cv.nba[(long long)pb * 6 + nb - 1];
      const int da = d == 1 ? 1 : 0, dc = d == 3 ? 1 : 2;   // tangential dims of a and c
      const int pa = (a + 1) >> 1, pc = (c + 1) >> 1;
      const int oa_ = da == 0 ? dix[0] : dix[1], oc_ = dc == 1 ? dix[1] : dix[2];   // octant offsets
      const int ta = oa_ + ((a & 1) ? pa - 1 : pa + 1), tc = oc_ + ((c & 1) ? pc - 1 : pc + 1);
      const int n1 = NC + 1, xd = low ? NC : 1;   // the neighbour parent's boundary along d
      const int ba = oa_ + pa, bc_ = oc_ + pc;
      if (ta == 0 || ta == n1) {   // (d, a, c) -> (x, y, z)
        const int o = d == 1 ? off_cell(Cv, xd, ta, bc_) : (d == 2 ? off_cell(Cv, ta, xd, bc_) : off_cell(Cv, ta, bc_, xd));
        rva[g] = boxp(Cv, 1, pn)[o] - boxp(Cv, 3, pn)[o];
        rima |= 1u << g;
      }
      if (tc == 0 || tc == n1) {
        const int o = d == 1 ? off_cell(Cv, xd, ba, tc) : (d == 2 ? off_cell(Cv, ba, xd, tc) : off_cell(Cv, ba, tc, xd));
        rvc[g] = boxp(Cv, 1, pn)[o] - boxp(Cv, 3, pn)[o];
        rimc |= 1u << g;
      }
      continue;
    }
    int nd[3] = {dix[0], dix[1], dix[2]};
    const int pn = Cv.nba[(long long)pb * 6 + nb - 1];
    nd[d - 1] = 0;
    if (og_lds) {
      gv[g] = prolong_at<NC>(Cv, pn, nd, fi, fj, fk);
      ocm |= 1u << g;
    } else {
      gv[g] = og + prolong_at<NC>(Cv, pn, nd, fi, fj, fk);
    }
  }
  // ---- parent's res = phi - old on its octant + face layer (stored by owner)
  load_parent_octant<NC, BS, true, true>(Cv, 4, pb, dix[0], dix[1], dix[2], cb);
  __syncthreads();
  // ---- phi += prolong(res): colour 0 (final here), colour 1 for bc_to_gc
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 >= npair) continue;
    const v2d ov = q2 < HV / 2 ? old[r < NR0 ? r : 0] : ld_nt(u + 2 * q2);
    double nv[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int q = 2 * q2 + s;
      int i, j, k;
      TL::decode(q, i, j, k);
      const int ic = (i + 1) >> 1, jc = (j + 1) >> 1, kc = (k + 1) >> 1;
      const int c0 = ic + CB * (jc + CB * kc);
      const double f0 = 0.25 * cb[c0];
      const double fx = 0.25 * cb[(i & 1) ? c0 - 1 : c0 + 1];
      const double fy = 0.25 * cb[(j & 1) ? c0 - CB : c0 + CB];
      const double fz = 0.25 * cb[(k & 1) ? c0 - CB * CB : c0 + CB * CB];
      const double o = s ? ov.y : ov.x;
      nv[s] = o + (f0 + fx + fy + fz);
      sb[q] = nv[s];
    }
    if (2 * q2 < HV) st_nt(u + 2 * q2, nv[0], nv[1]);   // colour 0 to HBM
  }
  // neighbours' boundary cells from the tile (+ rim taps)
#pragma unroll
  for (int g = 0; g < NG; g++) {
    if (!(defm >> g & 1)) continue;
    const int q = tid + BS * g;
    const int nb = q / FH + 1, rr = q % FH;
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1, gpos = low ? 0 : NC + 1;
    const int c = rr / HN + 1, ah = rr % HN;
    const int a = 2 * ah + 1 + ((1 + gpos + c) & 1);
    const int pd = low ? 0 : CB - 1, pa = (a + 1) >> 1, pc = (c + 1) >> 1;
    // cb strides of the normal and the two tangential directions
    const int sn = d == 1 ? 1 : (d == 2 ? CB : CB * CB);
    const int sa = d == 1 ? CB : 1, sc = d == 3 ? CB : CB * CB;
    const int c0 = pd * sn + pa * sa + pc * sc;
    // parity of the neighbour's fine index: NC (low face, even) or 1 (high, odd)
    const double tn = cb[low ? c0 + sn : c0 - sn];
    const double ta = (rima >> g & 1) ? rva[g] : cb[(a & 1) ? c0 - sa : c0 + sa];
    const double tc = (rimc >> g & 1) ? rvc[g] : cb[(c & 1) ? c0 - sc : c0 + sc];
    const double f0 = 0.25 * cb[c0];
    const double fx = 0.25 * (d == 1 ? tn : ta);
    const double fy = 0.25 * (d == 1 ? ta : (d == 2 ? tn : tc));
    const double fz = 0.25 * (d == 3 ? tn : tc);
    gv[g] = (og_lds ? sb[HV + q] : gv[g]) + (f0 + fx + fy + fz);
  }
#pragma unroll
  for (int g = 0; g < NG; g++)
    if (ocm >> g & 1) gv[g] = sb[HV + tid + BS * g] + gv[g];
  __syncthreads();
  // next to boxes the caller runs unfused (multi-GPU: those with a face on
  // another GPU, push0 = the faces toward them): they read our corrected
  // colour 0 from their ghost halves
  if (push0 && push0[b])
    face_push_local<NC>(F, T, 1, [&](int i, int j, int k) { return sb[TL::oint(i, j, k)]; }, push0[b]);
  // ---- colour-0 ghost values the substep reads (physical faces from the
  // corrected boundary cells: bc_to_gc)
#pragma unroll
  for (int g = 0; g < NG; g++) {
    const int q = tid + BS * g;
    if (q >= 6 * FH) continue;
    const int nb = q / FH + 1, rr = q % FH;
    const long long fidx = (long long)b * 6 + nb - 1;
    const int kind = T.kind(nb - 1);
    if (kind == NB_PHYS || (RB && kind == NB_RB)) {
      const bool low = nb & 1;
      const int d = (nb + 1) >> 1, gpos = low ? 0 : NC + 1;
      const int c = rr / HN + 1, ah = rr % HN;
      const int a = 2 * ah + 1 + ((1 + gpos + c) & 1);
      const int x1 = low ? 1 : NC, x2 = low ? 2 : NC - 1;
      int i1, j1, k1;
      if (d == 1) { i1 = x1; j1 = a; k1 = c; }
      else if (d == 2) { i1 = a; j1 = x1; k1 = c; }
      else { i1 = a; j1 = c; k1 = x1; }
      const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
      const double v1 = sb[TL::oint(i1, j1, k1)], v2 = sb[TL::oint(i2, j2, k2)];
      if (kind == NB_PHYS)
        gv[g] = phys_ghost(F, bc, b, fidx, nb, T.phys_code(nb - 1), a, c, TL::ogh(nb, a, c), v1, v2);
      else
        gv[g] = rb_ghost(F, RbSide{Cv, nullptr}, T.arg(nb - 1), nb, a, c, v1, v2);
    }
    sg[(nb - 1) * FH + rr] = gv[g];
  }
  __syncthreads();
  // ---- substep 1: colour 1 from colour 0, then its ghost fill (push colour 1)
  // (the substep's epilogue stores the level's refinement-boundary coarse
  // parts for the substeps after it, RbSide::gv)
  const RbSide rbs{Cv, nullptr, rbgv, rbgv ? 1 : 0};
  gsrb_box<NC, OP, BS, 2, true, RB>(F, lambda, 1, 2, bc, nullptr, nullptr, b, lds, nullptr, RB ? &rbs : nullptr);
}

template <int NC, int OP, int BS, bool RB = false>
// 8 waves per SIMD (4 workgroups of 16^3 per CU, the LDS limit): VGPRs <= 64;
// the refinement-boundary form holds the coarse operands of its epilogue in
// registers too (4 waves per SIMD)
__global__ void __launch_bounds__(BS, RB ? 4 : kPsWaves) k_prolong_smooth(LevelView Cv, LevelView F, double lambda,
                                                       const int* parent_local, const int* dixp, GcBC bc,
                                                       int one_child, const int* list, const uint8_t* push0,
                                                       double* rbgv) {
  __shared__ double lds[prolong_smooth_lds<NC>()];
  const int t = xcd_box(blockIdx.x, gridDim.x, F.rev);
  prolong_smooth_box<NC, OP, BS, RB>(Cv, F, lambda, parent_local, dixp, bc, one_child, push0, list ? list[t] : t,
                                     lds, rbgv);
}

void launch_prolong_smooth(const LevelView& C, const LevelView& F, int op, double lambda, const int* parent_local,
                           const int* dixp, const GcBC& bc, int one_child, const int* list, int n_list,
                           const uint8_t* push0, hipStream_t st, bool rb, double* rbgv) {
  const int n = list ? n_list : F.n;
  if (n == 0) return;
  const dim3 g(n);
  if (rb) {
    if (F.nc != 16 && F.nc != 8) throw std::runtime_error("launch_prolong_smooth: refinement boundaries need 16^3 / 8^3");
#define OMG_PSR(NC, BS)                                                                                         \
  if (op == OP_HELM)                                                                                            \
    k_prolong_smooth<NC, OP_HELM, BS, true><<<g, BS, 0, st>>>(C, F, lambda, parent_local, dixp, bc, one_child, \
                                                              list, push0, rbgv);                               \
  else                                                                                                          \
    k_prolong_smooth<NC, OP_LPL, BS, true><<<g, BS, 0, st>>>(C, F, lambda, parent_local, dixp, bc, one_child,  \
                                                             list, push0, rbgv);
    if (F.nc == 16) OMG_PSR(16, kPsBS16) else OMG_PSR(8, 256)
#undef OMG_PSR
    return;
  }
#define OMG_PS(NC, BS)                                                                                \
  if (op == OP_HELM)                                                                                  \
    k_prolong_smooth<NC, OP_HELM, BS><<<g, BS, 0, st>>>(C, F, lambda, parent_local, dixp, bc, one_child, \
                                                        list, push0, nullptr);                        \
  else                                                                                                \
    k_prolong_smooth<NC, OP_LPL, BS><<<g, BS, 0, st>>>(C, F, lambda, parent_local, dixp, bc, one_child,  \
                                                       list, push0, nullptr);
  switch (F.nc) {
    case 16: OMG_PS(16, kPsBS16) break;
    case 8: OMG_PS(8, 256) break;
    case 4: OMG_PS(4, 256) break;
    default: OMG_PS(2, 256) break;
  }
#undef OMG_PS
}

// get_sum's per-leaf interior sums (m_multigrid.f90:286-290): one lane per
// leaf, each summing its box sequentially in column-major order from +0.0
// (amdflang -O2 emits a single accumulator).  A wave owns LPW leaves and
// streams them through LDS in chunks of R rows: the loads are whole 256-B
// colour segments shared by 64 lanes (coalesced), the next chunk is in flight
// while the lanes run their add chains out of LDS.
// SUB: subtract_mean fused in front (m_multigrid.f90:268-272, no ghosts): every
// value is replaced by v - mean in HBM and the box sums are those of the new
// values (what the next get_sum of this variable will need).
// NT: non-temporal streams (the level is read once per pass)
template <bool NT>
__device__ __forceinline__ double2 sums_ld(const double* p) {
  if (NT) {
    const v2d t = ld_nt(p);
    return make_double2(t.x, t.y);
  }
  return *reinterpret_cast<const double2*>(p);
}
template <bool NT>
__device__ __forceinline__ void sums_st(double* p, double2 v) {
  if (NT)
    st_nt(p, v.x, v.y);
  else
    *reinterpret_cast<double2*>(p) = v;
}

template <int NC, bool SUB, int LPW = kSumsLPW>
__global__ void __launch_bounds__(64) k_box_sums3(LevelView L, int iv, const int* __restrict__ leaves,
                                                  int n_leaves, double* __restrict__ out,
                                                  const double* __restrict__ mean) {
  constexpr int H = NC / 2, R = kSumsR < NC ? kSumsR : NC, SEG = R * H;   // doubles of one colour in a chunk
  constexpr bool NTL = SUB ? kSubNTLd : kSumsNT;
  constexpr int CH2 = SEG;                        // double2 per box per chunk (2 colours)
  constexpr int PER = LPW * CH2 / 64;             // double2 per lane per chunk
  constexpr int P = 2 * SEG + 1;                  // LDS box stride (odd: no bank conflicts)
  constexpr int NCH = NC * NC / R;
  __shared__ double lds[LPW * P];
  const int lane = threadIdx.x, b0 = (L.rev ? gridDim.x - 1 - blockIdx.x : blockIdx.x) * LPW;
  const long long hv = L.hv;
  double* src[PER];
  int dst[PER];
  bool own[PER];   // lanes past the last leaf load a duplicate and never store
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const int t = lane + 64 * r, bb = t / CH2, w = t % CH2, seg = w / (SEG / 2), off = w % (SEG / 2);
    const int q = min(b0 + bb, n_leaves - 1);
    own[r] = b0 + bb < n_leaves;
    src[r] = boxp(L, iv, leaves[q]) + seg * hv + 2 * off;
    dst[r] = bb * P + seg * SEG + 2 * off;
  }
  const double m = SUB ? *mean : 0.0;
  // two chunks in flight (vmcnt counts loads and stores together, in issue
  // order: with one chunk of lookahead every chunk's loads also waited for the
  // previous chunk's stores)
  double2 va[PER], vb[PER];
  auto chunk_off = [](int c) { return H * (((c % (NC / R)) * R) + NC * (c / (NC / R))); };
#pragma unroll
  for (int r = 0; r < PER; r++) va[r] = sums_ld<NTL>(src[r]);
#pragma unroll
  for (int r = 0; r < PER; r++) vb[r] = sums_ld<NTL>(src[r] + chunk_off(1));
  double acc = 0.0;
  const double* my = lds + lane * P;
  auto process = [&](double2* v, int c) {
    __syncthreads();
    const int rc = chunk_off(c);
#pragma unroll
    for (int r = 0; r < PER; r++) {
      if (SUB) {
        v[r].x = v[r].x - m;
        v[r].y = v[r].y - m;
        if (own[r]) sums_st<kSubNTSt>(src[r] + rc, v[r]);
      }
      lds[dst[r]] = v[r].x;
      lds[dst[r] + 1] = v[r].y;
    }
    __syncthreads();
    if (c + 2 < NCH) {
      const int r2 = chunk_off(c + 2);
#pragma unroll
      for (int r = 0; r < PER; r++) v[r] = sums_ld<NTL>(src[r] + r2);
    }
    const int k = c / (NC / R) + 1, j0 = (c % (NC / R)) * R + 1;
    if (lane < LPW) {
#pragma unroll
      for (int rr = 0; rr < R; rr++) {
        const int ca = (1 + j0 + rr + k) & 1;   // colour of the odd-i cells of row j0+rr
        const double* A = my + ca * SEG + rr * H;
        const double* B = my + (1 - ca) * SEG + rr * H;
#pragma unroll
        for (int q = 0; q < H; q++) {
          acc += A[q];
          acc += B[q];
        }
      }
    }
  };
  static_assert(NCH % 2 == 0, "chunks come in pairs");
  for (int c = 0; c < NCH; c += 2) {
    process(va, c);
    process(vb, c + 1);
  }
  if (lane < LPW && b0 + lane < n_leaves) out[b0 + lane] = acc;
}

// generic box size: one lane per leaf straight from HBM
__global__ void __launch_bounds__(64) k_box_sums_any(LevelView L, int iv, const int* leaves, int n_leaves,
                                                     double* out) {
  const int q = blockIdx.x * 64 + threadIdx.x;
  if (q >= n_leaves) return;
  const double* u = boxp(L, iv, leaves[q]);
  double acc = 0.0;
  for (int k = 1; k <= L.nc; k++)
    for (int j = 1; j <= L.nc; j++)
      for (int i = 1; i <= L.nc; i++) acc += u[off_int(L, i, j, k)];
  out[q] = acc;
}

// acc = acc + w*s_q in leaf order (get_sum's loop, m_multigrid.f90:284-291).
// One wave: the box sums are staged through LDS 1024 at a time (the next
// stage in flight in registers), every lane runs the same add chain reading
// LDS a group ahead, and the products are formed off the chain.
__global__ void __launch_bounds__(64) k_seq_sum3(const double* __restrict__ box_sums, int n, double w,
                                                 double* __restrict__ acc, int init) {
  constexpr int CH = 1024, PL = CH / 128, G = 16;
  __shared__ double st[CH];
  const int lane = threadIdx.x;
  double a = init ? 0.0 : *acc;
  double2 pre[PL];
  auto fetch = [&](int base) {
#pragma unroll
    for (int r = 0; r < PL; r++) {
      const int q = base + 2 * (lane + 64 * r);
      pre[r].x = q < n ? box_sums[q] : 0.0;
      pre[r].y = q + 1 < n ? box_sums[q + 1] : 0.0;
    }
  };
  fetch(0);
  for (int base = 0; base < n; base += CH) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PL; r++) reinterpret_cast<double2*>(st)[lane + 64 * r] = pre[r];
    __syncthreads();
    if (base + CH < n) fetch(base + CH);
    const int m = min(CH, n - base);
    if (m == CH) {
      double cur[G], nxt[G];
#pragma unroll
      for (int t = 0; t < G; t++) cur[t] = st[t];
      for (int g = 0; g < CH / G; g++) {
        const int gn = g + 1 < CH / G ? g + 1 : g;
#pragma unroll
        for (int t = 0; t < G; t++) nxt[t] = st[G * gn + t];
        double p[G];
#pragma unroll
        for (int t = 0; t < G; t++) p[t] = w * cur[t];
#pragma unroll
        for (int t = 0; t < G; t++) a = a + p[t];
#pragma unroll
        for (int t = 0; t < G; t++) cur[t] = nxt[t];
      }
    } else {
      for (int q = 0; q < m; q++) a = a + w * st[q];
    }
  }
  if (lane == 0) *acc = a;
}

// mg_fill_ghost_cells_lvl of phi (m_ghost_cells.f90:131-175) for a level
// without refinement boundaries: the box's interior is read once, whole and
// coalesced, into LDS, then tile_face_fill pushes its boundary cells to the
// same-GPU neighbours as 16-B pairs, packs remote faces and forms physical
// ghosts (k_fill_gc reads and writes every face cell with its own 8-B access).
template <int NC, int BS>
__global__ void __launch_bounds__(BS) k_fill_tile(LevelView L, GcBC bc, double* sendbuf) {
  constexpr int HV = Tl<NC>::HV;
  __shared__ double sb[2 * HV];
  const int b = xcd_box(blockIdx.x, gridDim.x, L.rev);
  const FaceTopo T = load_topo(L, b);
  const double* u = L.phi + (long long)b * L.stride;
  for (int q = threadIdx.x; q < HV; q += BS) reinterpret_cast<v2d*>(sb)[q] = reinterpret_cast<const v2d*>(u)[q];
  __syncthreads();
  tile_face_fill<NC>(L, b, T, sb, 3, bc, sendbuf);
}

// k_fill_tile after a register-ring GS sweep.  tile_face_fill reads only the
// boundary layers of a box whose faces are same-GPU or remote neighbours (the
// second layers only for physical faces), so such a box stages 12 KB instead
// of its 32 KB interior: the k = 1 and k = 16 planes and the j = 1 and j = 16
// rows from phi, the i = 1 and i = 16 layers (strided in the colour-split
// layout) from the sweep's copy xl.  Boxes with a physical face load the
// whole interior as k_fill_tile does.  Same values, same pushes.
template <int NC, int BS>
__global__ void __launch_bounds__(BS) k_fill_tile_xl(LevelView L, GcBC bc, double* sendbuf,
                                                     const double* __restrict__ xl) {
  using TL = Tl<NC>;
  constexpr int HV = TL::HV, H = NC / 2, FH = H * NC;
  __shared__ double sb[2 * HV];
  const int b = xcd_box(blockIdx.x, gridDim.x, L.rev);
  const FaceTopo T = load_topo(L, b);
  const double* u = L.phi + (long long)b * L.stride;
  bool phys = false;
#pragma unroll
  for (int nb = 0; nb < 6; nb++) phys |= T.kind(nb) == NB_PHYS;
  if (phys) {
    for (int q = threadIdx.x; q < HV; q += BS) reinterpret_cast<v2d*>(sb)[q] = reinterpret_cast<const v2d*>(u)[q];
  } else {
    const int t = threadIdx.x;
    // planes k = 1, NC of both colours: 4 x FH doubles
    for (int q = t; q < 2 * FH; q += BS) {   // double pairs
      const int e = q / FH, w = q % FH, pl = w / (FH / 2), r2 = w % (FH / 2);
      const int off = e * HV + (pl ? FH * (NC - 1) : 0) + 2 * r2;
      *reinterpret_cast<v2d*>(sb + off) = *reinterpret_cast<const v2d*>(u + off);
    }
    // rows j = 1, NC of every plane, both colours: 4 x NC rows of H doubles
    for (int q = t; q < 4 * NC * (H / 2); q += BS) {
      const int r2 = q % (H / 2), row = q / (H / 2), k = row % NC, jj = (row / NC) & 1, e = row / (2 * NC);
      const int off = e * HV + H * ((jj ? NC - 1 : 0) + NC * k) + 2 * r2;
      *reinterpret_cast<v2d*>(sb + off) = *reinterpret_cast<const v2d*>(u + off);
    }
    // x layers i = 1, NC from xl
    const double* xb = xl + (long long)b * 512;
    for (int q = t; q < 2 * NC * NC; q += BS) {
      const int f = q / (NC * NC), c = q % (NC * NC), j = c % NC + 1, k = c / NC + 1;
      sb[TL::oint(f ? NC : 1, j, k)] = xb[q];
    }
  }
  __syncthreads();
  tile_face_fill<NC>(L, b, T, sb, 3, bc, sendbuf);
}

void launch_fill_tile_xl(const LevelView& L, const GcBC& bc, double* sendbuf, const double* xl, hipStream_t st) {
  if (L.n == 0) return;
  if (L.nc != 16) throw std::runtime_error("launch_fill_tile_xl: 16^3 boxes only");
  k_fill_tile_xl<16, 512><<<L.n, 512, 0, st>>>(L, bc, sendbuf, xl);
}

bool launch_fill_tile(const LevelView& L, const GcBC& bc, double* sendbuf, hipStream_t st) {
  if (L.n == 0) return true;
  const dim3 g(L.n);
  switch (L.nc) {
    case 16: k_fill_tile<16, 512><<<g, 512, 0, st>>>(L, bc, sendbuf); return true;
    case 8: k_fill_tile<8, 256><<<g, 256, 0, st>>>(L, bc, sendbuf); return true;
    case 4: k_fill_tile<4, 64><<<g, 64, 0, st>>>(L, bc, sendbuf); return true;
    default: return false;
  }
}

bool launch_smooth_resid(const LevelView& F, const LevelView& C, int op, double lambda, int restrict_on,
                         const int* parent_local, const int* dixp, hipStream_t st, const int* list,
                         int n_list, const GcBC& bc, bool has_rb, bool has_phys, const double* rbgv) {
  if (op != OP_LPL && op != OP_HELM) return false;
  if (!has_rb) rbgv = nullptr;
  const int n = list ? n_list : F.n;
  if (n == 0) return true;
  const dim3 g(n);
#define OMG_SR_RB(NC, BS, RB)                                                                                    \
  if (op == OP_LPL)                                                                                              \
    k_smooth_resid<NC, OP_LPL, BS, RB><<<g, BS, 0, st>>>(F, C, lambda, restrict_on, parent_local, dixp, list, bc,   \
                                                         rbgv);                                                   \
  else                                                                                                           \
    k_smooth_resid<NC, OP_HELM, BS, RB><<<g, BS, 0, st>>>(F, C, lambda, restrict_on, parent_local, dixp, list, bc,  \
                                                          rbgv);
#define OMG_SR(NC, BS)           \
  if (has_rb) {                  \
    OMG_SR_RB(NC, BS, 2)         \
  } else if (has_phys) {         \
    OMG_SR_RB(NC, BS, 1)         \
  } else {                       \
    OMG_SR_RB(NC, BS, 0)         \
  }
  switch (F.nc) {
    case 16: OMG_SR(16, 512) return true;
    case 8: OMG_SR(8, 256) return true;
    default: return false;
  }
#undef OMG_SR
#undef OMG_SR_RB
}

bool tiled_nc(int nc) { return nc == 16 || nc == 8 || nc == 4 || nc == 2; }

void launch_resid_restrict(const LevelView& F, const LevelView& C, int op, double lambda,
                           unsigned long long* maxbits, int restrict_on, const int* parent_local,
                           const int* dixp, hipStream_t st, const int* list, int n_list) {
  const int n = list ? n_list : F.n;
  if (n == 0) return;
  const dim3 g(n);
#define OMG_RR_OP(NC, BS, OPV) \
  k_resid_restrict<NC, OPV, BS><<<g, dim3(BS), 0, st>>>(F, C, lambda, maxbits, restrict_on, parent_local, dixp, list);
#define OMG_RR(NC, BS) OMG_FOR_OP(op, OMG_RR_OP, NC, BS)
  switch (F.nc) {
    case 16: OMG_RR(16, 512) break;
    case 8: OMG_RR(8, 256) break;
    case 4: OMG_RR(4, 256) break;
    default: OMG_RR(2, 256) break;
  }
#undef OMG_RR
#undef OMG_RR_OP
}

void launch_prolong_fill(const LevelView& C, const LevelView& F, int iv, const int* parent_local,
                         const int* dixp, const GcBC& bc, double* sendbuf, bool sub, bool skip1,
                         hipStream_t st, const int* list, int n_list, bool save_old, const RBRec* rb) {
  const int n = list ? n_list : F.n;
  if (n == 0) return;
  const dim3 g(n);
  const int so = save_old && !skip1;
#define OMG_PF(NC, BS)                                                                                              \
  if (rb && sub)                                                                                                    \
    k_prolong_fill<NC, BS, true, true><<<g, BS, 0, st>>>(C, F, iv, parent_local, dixp, bc, sendbuf, skip1, list, so, rb); \
  else if (rb)                                                                                                      \
    k_prolong_fill<NC, BS, false, true><<<g, BS, 0, st>>>(C, F, iv, parent_local, dixp, bc, sendbuf, skip1, list, so, rb); \
  else if (sub)                                                                                                     \
    k_prolong_fill<NC, BS, true><<<g, BS, 0, st>>>(C, F, iv, parent_local, dixp, bc, sendbuf, skip1, list, so, rb); \
  else                                                                                                              \
    k_prolong_fill<NC, BS, false><<<g, BS, 0, st>>>(C, F, iv, parent_local, dixp, bc, sendbuf, skip1, list, so, rb);
  switch (F.nc) {
    case 16: OMG_PF(16, 512) break;
    case 8: OMG_PF(8, 256) break;
    case 4: OMG_PF(4, 256) break;
    default: OMG_PF(2, 256) break;
  }
#undef OMG_PF
}

// update_coarse's parent loop (m_multigrid.f90:364-383) for one parent box
// per workgroup: rhs = L(phi) + res over the interior (box_op, then the sum),
// old = phi over the whole stored box.
// NT: non-temporal streams (a whole level per launch; the coarse tail's
// levels are re-read right away and keep the default policy)
template <int NC, int OP, int BS, bool NT = false>
__device__ __forceinline__ void coarse_rhs_box(const LevelView& Cv, double lambda, int b, double* sb) {
  using TL = Tl<NC>;
  constexpr int HV = TL::HV, FH = TL::FH, FS = TL::FS, NR = (HV + BS - 1) / BS, H = NC / 2;
  constexpr int NST = TL::NST;
  const int tid = threadIdx.x;
  const long long boff = (long long)b * Cv.stride;
  const double* __restrict__ u = Cv.phi + boff;
  double* __restrict__ rhs = Cv.data + Cv.vstride + boff;
  double* __restrict__ old = Cv.data + 2 * Cv.vstride + boff;
  const double* __restrict__ res = Cv.data + 3 * Cv.vstride + boff;
  for (int q = tid; q < NST / 2; q += BS) {
    const v2d x = NT ? ld_nt(u + 2 * q) : reinterpret_cast<const v2d*>(u)[q];
    reinterpret_cast<v2d*>(sb)[q] = x;
    if (NT)
      st_nt(old + 2 * q, x.x, x.y);
    else
      reinterpret_cast<v2d*>(old)[q] = x;
  }
  v2d rr[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 < HV) rr[r] = NT ? ld_nt(res + 2 * q2) : reinterpret_cast<const v2d*>(res)[q2];
  }
  __syncthreads();
  const OpCoef<OP> K(Cv, lambda);
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 >= HV) continue;
    const int e = q2 >= HV / 2, o = 1 - e;
    Nbr7 s0, s1;
    if constexpr (H % 2 == 0) {
      pair_stencil<NC>(sb + o * HV, sb + 2 * HV + o * FH, FS, e, 2 * q2 - e * HV, s0, s1);
    } else {
      int i, j, k;
      TL::decode(2 * q2, i, j, k);
      s0.xm = sb[TL::ocell(i - 1, j, k)]; s0.xp = sb[TL::ocell(i + 1, j, k)];
      s0.ym = sb[TL::ocell(i, j - 1, k)]; s0.yp = sb[TL::ocell(i, j + 1, k)];
      s0.zm = sb[TL::ocell(i, j, k - 1)]; s0.zp = sb[TL::ocell(i, j, k + 1)];
      TL::decode(2 * q2 + 1, i, j, k);
      s1.xm = sb[TL::ocell(i - 1, j, k)]; s1.xp = sb[TL::ocell(i + 1, j, k)];
      s1.ym = sb[TL::ocell(i, j - 1, k)]; s1.yp = sb[TL::ocell(i, j + 1, k)];
      s1.zm = sb[TL::ocell(i, j, k - 1)]; s1.zp = sb[TL::ocell(i, j, k + 1)];
    }
    const double2 cc = reinterpret_cast<const double2*>(sb)[q2];
    s0.c = cc.x;
    s1.c = cc.y;
    double l0, l1;
    op_pair<NC, OP>(K, Cv, b, e, 2 * q2 - e * HV, s0, s1, l0, l1);
    v2d out;
    out.x = l0 + rr[r].x;
    out.y = l1 + rr[r].y;
    if (NT)
      st_nt(rhs + 2 * q2, out.x, out.y);
    else
      reinterpret_cast<v2d*>(rhs)[q2] = out;
  }
}

// update_coarse's fill of the coarse level (mg_fill_ghost_cells_lvl,
// m_ghost_cells.f90:131-175) and its parents' rhs = L(phi) + res, old = phi
// (m_multigrid.f90:364-383) in one pass, for a level whose faces are same-GPU
// or physical.  Every box pushes its boundary cells and forms its physical
// ghosts as k_fill_tile does; a parent box also needs its own ghost faces
// for the operator, and rather than wait for its neighbours' pushes it reads
// their boundary cells itself (the same values the pushes carry: phi of this
// level is final once the restriction above has run) and forms its physical
// ghosts in LDS from its own cells (bc_to_gc, as the push side does).  Then
// the tile holds exactly what k_coarse_rhs_tile would load after the fill.
template <int NC, int OP, int BS>
__global__ void __launch_bounds__(BS) k_fill_crhs(LevelView C, double lambda, GcBC bc,
                                                  const uint8_t* __restrict__ parmask) {
  using TL = Tl<NC>;
  constexpr int HV = TL::HV, NST = TL::NST, FH = TL::FH, NR = (HV + BS - 1) / BS, H = NC / 2;
  __shared__ double sb[NST];
  const int tid = threadIdx.x, b = xcd_box(blockIdx.x, gridDim.x, C.rev);
  const FaceTopo T = load_topo(C, b);
  const long long boff = (long long)b * C.stride;
  const double* __restrict__ u = C.phi + boff;
  const bool par = parmask[b] != 0;
  for (int q = tid; q < HV; q += BS) reinterpret_cast<v2d*>(sb)[q] = reinterpret_cast<const v2d*>(u)[q];
  v2d rr[NR];
  if (par) {
    // the neighbours' boundary cells into our ghost faces (both colours)
    for (int p = tid; p < 6 * NC * NC; p += BS) {
      const int f = p / (NC * NC), cell = p % (NC * NC);
      if (T.kind(f) != NB_LOCAL) continue;
      const int nb = f + 1, a = cell % NC + 1, c = cell / NC + 1, d = f >> 1;
      const bool low = nb & 1;
      sb[TL::ogh(nb, a, c)] = C.phi[(long long)T.arg(f) * C.stride + sr_int<NC>(d, low ? NC : 1, a, c)];
    }
    const double* __restrict__ res = C.data + 3 * C.vstride + boff;
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const int q2 = tid + BS * r;
      if (q2 < HV) rr[r] = ld_nt(res + 2 * q2);
    }
  }
  __syncthreads();
  tile_face_fill<NC>(C, b, T, sb, 3, bc, nullptr);
  if (!par) return;
  if (T.nonlocal()) {   // physical ghosts in the tile too
    for (int p = tid; p < 6 * NC * NC; p += BS) {
      const int f = p / (NC * NC), cell = p % (NC * NC);
      if (T.kind(f) != NB_PHYS) continue;
      const int nb = f + 1, a = cell % NC + 1, c = cell / NC + 1, d = f >> 1;
      const bool low = nb & 1;
      const int gi = TL::ogh(nb, a, c);
      sb[gi] = phys_ghost(C, bc, b, (long long)b * 6 + f, nb, T.phys_code(f), a, c, gi,
                          sb[sr_int<NC>(d, low ? 1 : NC, a, c)], sb[sr_int<NC>(d, low ? 2 : NC - 1, a, c)]);
    }
  }
  __syncthreads();
  // old = phi over the stored box, then rhs = L(phi) + res (coarse_rhs_box)
  double* __restrict__ old = C.data + 2 * C.vstride + boff;
  double* __restrict__ rhs = C.data + C.vstride + boff;
  for (int q = tid; q < NST / 2; q += BS) {
    const v2d x = reinterpret_cast<const v2d*>(sb)[q];
    st_nt(old + 2 * q, x.x, x.y);
  }
  const OpCoef<OP> K(C, lambda);
  constexpr int FS = TL::FS;
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int q2 = tid + BS * r;
    if (q2 >= HV) continue;
    const int e = q2 >= HV / 2, o = 1 - e;
    Nbr7 s0, s1;
    if constexpr (H % 2 == 0) {
      pair_stencil<NC>(sb + o * HV, sb + 2 * HV + o * FH, FS, e, 2 * q2 - e * HV, s0, s1);
    } else {
      int i, j, k;
      TL::decode(2 * q2, i, j, k);
      s0.xm = sb[TL::ocell(i - 1, j, k)]; s0.xp = sb[TL::ocell(i + 1, j, k)];
      s0.ym = sb[TL::ocell(i, j - 1, k)]; s0.yp = sb[TL::ocell(i, j + 1, k)];
      s0.zm = sb[TL::ocell(i, j, k - 1)]; s0.zp = sb[TL::ocell(i, j, k + 1)];
      TL::decode(2 * q2 + 1, i, j, k);
      s1.xm = sb[TL::ocell(i - 1, j, k)]; s1.xp = sb[TL::ocell(i + 1, j, k)];
      s1.ym = sb[TL::ocell(i, j - 1, k)]; s1.yp = sb[TL::ocell(i, j + 1, k)];
      s1.zm = sb[TL::ocell(i, j, k - 1)]; s1.zp = sb[TL::ocell(i, j, k + 1)];
    }
    const double2 cc = reinterpret_cast<const double2*>(sb)[q2];
    s0.c = cc.x;
    s1.c = cc.y;
    double l0, l1;
    op_pair<NC, OP>(K, C, b, e, 2 * q2 - e * HV, s0, s1, l0, l1);
    st_nt(rhs + 2 * q2, l0 + rr[r].x, l1 + rr[r].y);
  }
}

void launch_fill_crhs(const LevelView& C, int op, double lambda, const GcBC& bc, const uint8_t* parmask,
                      hipStream_t st) {
  if (C.n == 0) return;
  const dim3 g(C.n);
#define OMG_FC_OP(NC, BS, OPV) k_fill_crhs<NC, OPV, BS><<<g, BS, 0, st>>>(C, lambda, bc, parmask);
#define OMG_FC(NC, BS) OMG_FOR_OP(op, OMG_FC_OP, NC, BS)
  switch (C.nc) {
    case 16: OMG_FC(16, 512) break;
    case 8: OMG_FC(8, 256) break;
    case 4: OMG_FC(4, 64) break;
    default: throw std::runtime_error("launch_fill_crhs: box sizes 16, 8, 4");
  }
#undef OMG_FC
#undef OMG_FC_OP
}

template <int NC, int OP, int BS>
__global__ void __launch_bounds__(BS) k_coarse_rhs_tile(LevelView Cv, double lambda, const int* parents) {
  __shared__ double sb[Tl<NC>::NST];
  coarse_rhs_box<NC, OP, BS, true>(Cv, lambda, parents[xcd_box(blockIdx.x, gridDim.x, Cv.rev)], sb);
}

bool launch_coarse_rhs_tile(const LevelView& C, int op, double lambda, const int* parents, int n_par,
                            hipStream_t st) {
  if (!tiled_nc(C.nc)) return false;
  if (n_par == 0) return true;
  const dim3 g(n_par);
#define OMG_CR_OP(NC, BS, OPV) k_coarse_rhs_tile<NC, OPV, BS><<<g, BS, 0, st>>>(C, lambda, parents);
#define OMG_CR(NC, BS) OMG_FOR_OP(op, OMG_CR_OP, NC, BS)
  switch (C.nc) {
    case 16: OMG_CR(16, 512) break;
    case 8: OMG_CR(8, 256) break;
    case 4: OMG_CR(4, 256) break;
    default: OMG_CR(2, 256) break;
  }
#undef OMG_CR
#undef OMG_CR_OP
  return true;
}

void launch_box_sums(const LevelView& L, int iv, const int* leaves, int n, double* out, hipStream_t st) {
  if (n == 0) return;
  const dim3 g((n + kSumsLPW - 1) / kSumsLPW);
  switch (L.nc) {
    case 16: k_box_sums3<16, false><<<g, 64, 0, st>>>(L, iv, leaves, n, out, nullptr); break;
    case 8: k_box_sums3<8, false><<<g, 64, 0, st>>>(L, iv, leaves, n, out, nullptr); break;
    case 4: k_box_sums3<4, false><<<g, 64, 0, st>>>(L, iv, leaves, n, out, nullptr); break;
    default: k_box_sums_any<<<(n + 63) / 64, 64, 0, st>>>(L, iv, leaves, n, out); break;
  }
}

bool subtract_sums_nc(int nc) { return nc == 16 || nc == 8 || nc == 4; }

void launch_subtract_sums(const LevelView& L, int iv, const int* leaves, int n, const double* mean, double* out,
                          hipStream_t st) {
  if (n == 0) return;
  const dim3 g((n + kSumsLPW - 1) / kSumsLPW);
  switch (L.nc) {
    case 16: k_box_sums3<16, true><<<g, 64, 0, st>>>(L, iv, leaves, n, out, mean); break;
    case 8: k_box_sums3<8, true><<<g, 64, 0, st>>>(L, iv, leaves, n, out, mean); break;
    case 4: k_box_sums3<4, true><<<g, 64, 0, st>>>(L, iv, leaves, n, out, mean); break;
    default: break;
  }
}

// mean = MPI_Allreduce(sum) / volume on the device (subtract_mean,
// m_multigrid.f90:255-262): the per-rank sums combined in MPICH's one-node
// binomial order, ((a0+a1)+(a2+a3))+..., then the division.
__global__ void k_mean(const double* all, int n, double volume, double* mean) {
  __shared__ double t[64];   // (a per-lane array indexed by r would live in scratch)
  if (threadIdx.x || blockIdx.x) return;
  for (int r = 0; r < n; r++) t[r] = all[r];
  for (int w = 1; w < n; w *= 2)
    for (int r = 0; r + w < n; r += 2 * w) t[r] = t[r] + t[r + w];
  *mean = t[0] / volume;
}

void launch_mean(const double* all, int n, double volume, double* mean, hipStream_t st) {
  k_mean<<<1, 64, 0, st>>>(all, n, volume, mean);
}

void launch_seq_sum(const double* box_sums, int n, double w, double* acc, bool init, hipStream_t st) {
  if (n == 0) return;
  k_seq_sum3<<<1, 64, 0, st>>>(box_sums, n, w, acc, init);
}

// ---------------------------------------------------------------------------
// The coarse end of mg_fas_vcycle (m_multigrid.f90:185-229) in one workgroup.
constexpr int kTailBS = 512;
// LDS of the largest box program: 16^3 residual / coarse rhs, and with LEX
// (lexicographic GS) the 16^3 sweep
template <bool LEX>
constexpr int tail_lds() {
  return LEX && gs_lex_lds<16>() > Tl<16>::NST ? gs_lex_lds<16>() : Tl<16>::NST;
}

__device__ void tail_fill(const TailArgs& A, int li);

template <int OP, bool LEX>
__device__ void tail_smooth(const TailArgs& A, int li, int n_cycle, double* lds) {
  const TailLevel& T = A.lv[li];
  if constexpr (LEX) {
    // smooth_boxes with mg_smoother_gs: a sweep of every box, then the fill
    for (int n = 1; n <= n_cycle; n++) {
      for (int b = 0; b < T.L.n; b++) {
        switch (T.L.nc) {
          case 16: gs_lex_box<OP, 16>(T.L, A.lambda, b, lds); break;
          case 8: gs_lex_box<OP, 8>(T.L, A.lambda, b, lds); break;
          case 4: gs_lex_box<OP, 4>(T.L, A.lambda, b, lds); break;
          default: gs_lex_box<OP, 2>(T.L, A.lambda, b, lds); break;
        }
      }
      tail_fill(A, li);
    }
    return;
  }
  for (int n = 1; n <= 2 * n_cycle; n++) {
    const int e = n & 1;
    for (int b = 0; b < T.L.n; b++) {
      switch (T.L.nc) {
        case 16: gsrb_box<16, OP, kTailBS, 0>(T.L, A.lambda, e, 1 << e, T.bc, nullptr, nullptr, b, lds); break;
        case 8: gsrb_box<8, OP, kTailBS, 0>(T.L, A.lambda, e, 1 << e, T.bc, nullptr, nullptr, b, lds); break;
        case 4: gsrb_box<4, OP, kTailBS, 0>(T.L, A.lambda, e, 1 << e, T.bc, nullptr, nullptr, b, lds); break;
        default: gsrb_box<2, OP, kTailBS, 0>(T.L, A.lambda, e, 1 << e, T.bc, nullptr, nullptr, b, lds); break;
      }
      __syncthreads();
    }
  }
}

// residual over level li (+ restriction onto li-1 when restrict_on); with
// maxbits: max |res| returned to every thread
template <int OP>
__device__ double tail_residual(const TailArgs& A, int li, int restrict_on, bool want_max, double* lds) {
  const TailLevel& T = A.lv[li];
  const LevelView C = restrict_on ? A.lv[li - 1].L : T.L;
  unsigned long long* mb = want_max ? A.maxbits : nullptr;
  if (want_max) {
    if (threadIdx.x == 0) *mb = 0ull;
    __syncthreads();
  }
  for (int b = 0; b < T.L.n; b++) {
    switch (T.L.nc) {
      case 16: resid_restrict_box<16, OP, kTailBS>(T.L, C, A.lambda, mb, restrict_on, T.parent_local, T.dixp, b, lds); break;
      case 8: resid_restrict_box<8, OP, kTailBS>(T.L, C, A.lambda, mb, restrict_on, T.parent_local, T.dixp, b, lds); break;
      case 4: resid_restrict_box<4, OP, kTailBS>(T.L, C, A.lambda, mb, restrict_on, T.parent_local, T.dixp, b, lds); break;
      default: resid_restrict_box<2, OP, kTailBS>(T.L, C, A.lambda, mb, restrict_on, T.parent_local, T.dixp, b, lds); break;
    }
    __syncthreads();
  }
  if (!want_max) return 0.0;
  const unsigned long long bits = __hip_atomic_load(mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  return __longlong_as_double((long long)bits);
}

// mg_fill_ghost_cells_lvl of phi on level li (same-GPU faces and physical
// boundaries only, which is all a tail level has)
__device__ void tail_fill(const TailArgs& A, int li) {
  const TailLevel& T = A.lv[li];
  const int nc = T.L.nc, nc2 = nc * nc;
  const LevelView none{};
  if (nc == 1) {   // (the reference's face order, box1_fill)
    for (int b = threadIdx.x; b < T.L.n; b += blockDim.x) box1_fill(T.L, 1, b, none, nullptr, T.bc, nullptr);
  } else {
    for (int t = threadIdx.x; t < T.L.n * 6 * nc2; t += blockDim.x) {
      const int cell = t % nc2, f = t / nc2;
      face_cell_fill(T.L, 1, f / 6, f % 6 + 1, cell % nc + 1, cell / nc + 1, 3, none, nullptr, T.bc, nullptr);
    }
  }
  __syncthreads();
}

template <int OP>
__device__ void tail_coarse_rhs(const TailArgs& A, int li, double* lds) {
  const TailLevel& T = A.lv[li];
  for (int p = 0; p < T.n_par; p++) {
    const int b = T.parents[p];
    switch (T.L.nc) {
      case 16: coarse_rhs_box<16, OP, kTailBS>(T.L, A.lambda, b, lds); break;
      case 8: coarse_rhs_box<8, OP, kTailBS>(T.L, A.lambda, b, lds); break;
      case 4: coarse_rhs_box<4, OP, kTailBS>(T.L, A.lambda, b, lds); break;
      default: coarse_rhs_box<2, OP, kTailBS>(T.L, A.lambda, b, lds); break;
    }
    __syncthreads();
  }
}

// correct_children(li-1) + mg_fill_ghost_cells_lvl(li): every parent's
// children are here, so each child forms its parent's res = phi - old
__device__ void tail_correct(const TailArgs& A, int li, double* lds) {
  const TailLevel& T = A.lv[li];
  const LevelView C = A.lv[li - 1].L;
  for (int b = 0; b < T.L.n; b++) {
    switch (T.L.nc) {
      case 16: prolong_fill_box<16, kTailBS, true>(C, T.L, 4, T.parent_local, T.dixp, T.bc, nullptr, b, lds, false); break;
      case 8: prolong_fill_box<8, kTailBS, true>(C, T.L, 4, T.parent_local, T.dixp, T.bc, nullptr, b, lds, false); break;
      case 4: prolong_fill_box<4, kTailBS, true>(C, T.L, 4, T.parent_local, T.dixp, T.bc, nullptr, b, lds, false); break;
      default: prolong_fill_box<2, kTailBS, true>(C, T.L, 4, T.parent_local, T.dixp, T.bc, nullptr, b, lds, false); break;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// The levels of the tail with boxes of at most 8^3 cells run with their boxes
// resident in LDS: all four variables of each such level (one box each) in a
// plain (nc+2)^3 layout, i fastest (edges and corners unused), loaded once
// and written back once.  Every step keeps the arithmetic of the global-memory
// box programs above (gs_value / op_value on the same operands, the same
// sequential restriction sum, the same prolongation order, the same ghost
// formulas), so the results are bit-identical; only the L2 round trips and
// the per-step LDS staging go away.  The one-box levels of the tail are
// single boxes whose local neighbours are the box itself (periodic faces);
// run_tail (omg_api.cpp) checks that when it sets lds_levels / lds_top.
constexpr int kTailLdsLevels = kTailLdsMaxLevels;
constexpr int kTailLdsDoubles = 4 * (10 * 10 * 10 + 6 * 6 * 6 + 4 * 4 * 4);
// the physical bc values of each face cell of each level, resolved once
// (stored in rhs ghosts / tabulated / constant)
constexpr int kTailLdsBcDoubles = 6 * (8 * 8 + 4 * 4 + 2 * 2);
// A 16^3 top level as well, phi and rhs only (its old is
// not used inside the tail, its res goes straight to HBM)
constexpr int kTailBigS = 18, kTailBigS3 = kTailBigS * kTailBigS * kTailBigS;
constexpr int kTailBigDoubles = 2 * kTailBigS3 + 6 * 16 * 16;

struct TailBox {
  double *P, *F, *O, *R;   // phi, rhs, old, res
  double* B;               // bc value per face cell (6 nc^2)
  int nc, S;
  int ln;                  // log2(nc): the per-cell index math uses shifts and masks
                           // (nc is a power of two; division by a runtime value
                           // costs tens of instructions per cell)
  __device__ __forceinline__ int at(int i, int j, int k) const { return i + S * (j + S * k); }
};

// per LDS level, kept in LDS so the per-cell work never reads the tail's
// argument block in HBM with lane-dependent indices
__device__ __forceinline__ Nbr7 tail_nbr(const TailBox& X, const double* U, int c) {
  Nbr7 s;
  s.c = U[c];
  s.xm = U[c - 1];
  s.xp = U[c + 1];
  s.ym = U[c - X.S];
  s.yp = U[c + X.S];
  s.zm = U[c - X.S * X.S];
  s.zp = U[c + X.S * X.S];
  return s;
}

struct TailLdsLevel {
  int local[6];                // periodic face: the box itself on the other side
  double c0[6], c1[6], c2[6];  // bc_to_gc coefficients of each physical face
};

__device__ __forceinline__ TailBox tail_box(const TailArgs& A, int li, double* tl) {
  TailBox X;
  int base = 0, bbase = kTailLdsDoubles;
  for (int l = 0; l < li; l++) {
    const int s = A.lv[l].L.nc + 2;
    base += 4 * s * s * s;
    bbase += 6 * A.lv[l].L.nc * A.lv[l].L.nc;
  }
  X.nc = A.lv[li].L.nc;
  X.S = X.nc + 2;
  X.ln = 31 - __clz(X.nc);
  const int s3 = X.S * X.S * X.S;
  X.P = tl + base;
  X.F = X.P + s3;
  X.O = X.F + s3;
  X.R = X.O + s3;
  X.B = tl + bbase;
  return X;
}

__device__ __forceinline__ TailBox tail_big_box(double* tl) {
  TailBox X;
  X.nc = 16;
  X.S = kTailBigS;
  X.ln = 4;
  X.P = tl + kTailLdsDoubles + kTailLdsBcDoubles;
  X.F = X.P + kTailBigS3;
  X.O = X.R = nullptr;
  X.B = X.F + kTailBigS3;
  return X;
}

// One box variable set of the LDS-resident tail, HBM <-> LDS: NV variables
// (1 = phi, 2 = rhs, ...) of the single box of level L, interior and face
// ghosts, to / from the plain (NC+2)^3 arrays at dst (consecutive per
// variable).  The stored box is contiguous per variable (omg_device.h), so
// each thread moves whole 16-B pairs: all loads of the box are issued at once
// (one memory latency) and scattered to their plain positions in LDS; the
// edges and corners, which the device does not store, are zeroed in LDS and
// never written back.
template <int NC>
__device__ __forceinline__ int stored_dense(int q) {
  using TL = Tl<NC>;
  constexpr int S = NC + 2, H = TL::H, HV = TL::HV, FS = TL::FS;
  int i, j, k;
  if (q < 2 * HV) {
    TL::decode(q, i, j, k);
  } else {
    const int r0 = q - 2 * HV, nb = r0 / FS + 1, r1 = r0 % FS;
    const int e = r1 >= H * NC, r = r1 - e * H * NC, ah = r % H, c = r / H + 1;
    const int g = (nb & 1) ? 0 : NC + 1;
    const int a = 2 * ah + 1 + ((1 + g + c + e) & 1);
    const int d = (nb + 1) >> 1;
    if (d == 1) { i = g; j = a; k = c; }
    else if (d == 2) { i = a; j = g; k = c; }
    else { i = a; j = c; k = g; }
  }
  return i + S * (j + S * k);
}

template <int NC, int NV, bool LOAD, int V0 = 1>
__device__ void tail_io_stored(const LevelView& L, double* dst) {
  constexpr int S = NC + 2, S3 = S * S * S, NP = Tl<NC>::NST / 2, N = NV * NP;
  constexpr int R = (N + kTailBS - 1) / kTailBS;
  const int tid = threadIdx.x;
  if (LOAD) {
    // edges and corners: 12 edges of NC cells and 8 corners per variable
    constexpr int NE = 12 * NC + 8;
    for (int t = tid; t < NV * NE; t += kTailBS) {
      const int var = t / NE, e = t % NE;
      int x, y, z;
      if (e < 12 * NC) {
        const int ax = e / (4 * NC), w = e % (4 * NC), m = w / NC, a = w % NC + 1;
        const int u = (m & 1) ? S - 1 : 0, v = (m & 2) ? S - 1 : 0;
        if (ax == 0) { x = a; y = u; z = v; }
        else if (ax == 1) { x = u; y = a; z = v; }
        else { x = u; y = v; z = a; }
      } else {
        const int m = e - 12 * NC;
        x = (m & 1) ? S - 1 : 0; y = (m & 2) ? S - 1 : 0; z = (m & 4) ? S - 1 : 0;
      }
      dst[var * S3 + x + S * (y + S * z)] = 0.0;
    }
    v2d v[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int t = tid + kTailBS * r;
      if (t < N) v[r] = reinterpret_cast<const v2d*>(boxp(L, t / NP + V0, 0))[t % NP];
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int t = tid + kTailBS * r;
      if (t >= N) continue;
      const int var = t / NP, p = t % NP;
      dst[var * S3 + stored_dense<NC>(2 * p)] = v[r].x;
      dst[var * S3 + stored_dense<NC>(2 * p + 1)] = v[r].y;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int t = tid + kTailBS * r;
      if (t >= N) continue;
      const int var = t / NP, p = t % NP;
      v2d x;
      x.x = dst[var * S3 + stored_dense<NC>(2 * p)];
      x.y = dst[var * S3 + stored_dense<NC>(2 * p + 1)];
      reinterpret_cast<v2d*>(boxp(L, var + V0, 0))[p] = x;
    }
  }
}

// the same load in two halves, so that the loads of several boxes are all in
// flight before the first one is scattered (one memory latency for the tail's
// whole entry instead of one per box)
template <int NC, int NV>
struct TailIoRegs {
  static constexpr int NP = Tl<NC>::NST / 2, N = NV * NP, R = (N + kTailBS - 1) / kTailBS;
  v2d v[R];
  __device__ __forceinline__ void issue(const LevelView& L) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int t = threadIdx.x + kTailBS * r;
      if (t < N) v[r] = reinterpret_cast<const v2d*>(boxp(L, t / NP + 1, 0))[t % NP];
    }
  }
  __device__ __forceinline__ void commit(double* dst) const {
    constexpr int S = NC + 2, S3 = S * S * S, NE = 12 * NC + 8;
    const int tid = threadIdx.x;
    for (int t = tid; t < NV * NE; t += kTailBS) {   // edges and corners: zero
      const int var = t / NE, e = t % NE;
      int x, y, z;
      if (e < 12 * NC) {
        const int ax = e / (4 * NC), w = e % (4 * NC), m = w / NC, a = w % NC + 1;
        const int u = (m & 1) ? S - 1 : 0, q = (m & 2) ? S - 1 : 0;
        if (ax == 0) { x = a; y = u; z = q; }
        else if (ax == 1) { x = u; y = a; z = q; }
        else { x = u; y = q; z = a; }
      } else {
        const int m = e - 12 * NC;
        x = (m & 1) ? S - 1 : 0; y = (m & 2) ? S - 1 : 0; z = (m & 4) ? S - 1 : 0;
      }
      dst[var * S3 + x + S * (y + S * z)] = 0.0;
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int t = tid + kTailBS * r;
      if (t >= N) continue;
      const int var = t / NP, p = t % NP;
      dst[var * S3 + stored_dense<NC>(2 * p)] = v[r].x;
      dst[var * S3 + stored_dense<NC>(2 * p + 1)] = v[r].y;
    }
  }
};

template <bool LOAD>
__device__ void tail_io_box(const LevelView& L, double* dst) {   // the LDS levels: all four variables
  switch (L.nc) {
    case 8: tail_io_stored<8, 4, LOAD>(L, dst); break;
    case 4: tail_io_stored<4, 4, LOAD>(L, dst); break;
    default: tail_io_stored<2, 4, LOAD>(L, dst); break;
  }
}

// all four variables of the boxes of levels 0..ls (contiguous in LDS)
template <bool LOAD>
__device__ void tail_boxes_io(const TailArgs& A, int ls, double* tl) {
  int base = 0;
  for (int l = 0; l <= ls; l++) {
    const LevelView& L = A.lv[l].L;
    tail_io_box<LOAD>(L, tl + base);
    const int S = L.nc + 2;
    base += 4 * S * S * S;
  }
  __syncthreads();
}

// the fill's per-level data (TailLdsLevel) and the bc value of every
// physical face cell (bc_to_gc's argument: the stored value in the rhs ghost
// when mg_phi_bc_store ran, else the tabulated or constant one); after the
// rhs ghosts are in LDS
__device__ __forceinline__ long long tail_foff(const TailArgs& A, int l, int nb) {
  const int o = A.lv[l].foff[nb - 1];
  return o == -2 ? A.lv[l].bc.face_off[nb - 1] : (long long)o;
}

__device__ __forceinline__ void tail_setup_coef(const TailArgs& A, int l, TailLdsLevel& D, int nb) {
  const LevelView& L = A.lv[l].L;
  const GcBC& bc = A.lv[l].bc;
  const bool low = nb & 1;
  // every read first, then the selection (one round trip, not one per test)
  const int ps = bc.phi_stored, fo = A.lv[l].foff[nb - 1];
  const int nba = L.nba[nb - 1], fty = A.lv[l].ftype[nb - 1], typ = bc.type[nb - 1], kind = L.nbk[nb - 1];
  const double drv = L.dr[(nb - 1) >> 1];
  const int type = ps ? nba : fo == -2 ? bc.face_type[nb - 1] : fo >= 0 ? fty : typ;
  double c0, c1, c2;
  if (type == -10) {
    c0 = 2; c1 = -1; c2 = 0;
  } else if (type == -11) {
    c0 = drv * (low ? -1.0 : 1.0); c1 = 1; c2 = 0;
  } else {
    c0 = 0; c1 = 2; c2 = -1;
  }
  D.local[nb - 1] = kind == NB_LOCAL;
  D.c0[nb - 1] = c0;
  D.c1[nb - 1] = c1;
  D.c2[nb - 1] = c2;
}

// face cell p (6 nc^2 of them) of level l: whether its face is physical, and
// its bc value into bv
__device__ __forceinline__ bool tail_bc_value(const TailArgs& A, int l, const TailBox& X, int p, double& bv) {
  const LevelView& L = A.lv[l].L;
  const GcBC& bc = A.lv[l].bc;
  const int nc = X.nc, nc2 = nc * nc;
  const int nb = p / nc2 + 1, cell = p % nc2, a = cell % nc + 1, c = cell / nc + 1;
  if (L.nbk[nb - 1] != NB_PHYS) return false;
  const int d = (nb + 1) >> 1, g = (nb & 1) ? 0 : nc + 1;
  if (bc.phi_stored)
    bv = X.F[d == 1 ? X.at(g, a, c) : d == 2 ? X.at(a, g, c) : X.at(a, c, g)];
  else if (A.lv[l].foff[nb - 1] != -1)
    bv = bc.face_data[tail_foff(A, l, nb) + (a - 1) + (long long)nc * (c - 1)];
  else
    bv = bc.value[nb - 1];
  return true;
}

__device__ __forceinline__ void tail_lds_setup(const TailArgs& A, int l, const TailBox& X, TailLdsLevel& D) {
  if (threadIdx.x < 6) tail_setup_coef(A, l, D, threadIdx.x + 1);
  for (int p = threadIdx.x; p < 6 * X.nc * X.nc; p += blockDim.x) {
    double bv;
    if (tail_bc_value(A, l, X, p, bv)) X.B[p] = bv;
  }
}

// tail_lds_setup of the usual chain (16^3 top over 8^3, 4^3, 2^3) in two
// halves around the boxes' load: issue() reads every bc value held in HBM
// (tabulated faces) while the boxes' loads are in flight, commit() (after
// they are in LDS) takes the stored ones from the rhs ghosts and writes all
struct TailChainBc {
  static constexpr int O8 = 6 * 256, O4 = O8 + 6 * 64, O2 = O4 + 6 * 16, NT = O2 + 6 * 4;
  static constexpr int R = (NT + kTailBS - 1) / kTailBS;
  double bv[R];
  int dst[R], src[R];   // offsets into the LDS array: the bc slot (-1: not a
                        // physical face), the rhs ghost it is stored in (-1: bv)
  // Every read of the argument block a face cell needs is issued before any
  // of them is tested (each test would wait for its own round trip), and the
  // LDS places of the chain's boxes are compile-time (tail_box's layout).
  __device__ __forceinline__ void issue(const TailArgs& A, int top, const TailBox& XB, double* lds,
                                        TailLdsLevel* tll) {
    if (threadIdx.x < 24) {
      const int k = threadIdx.x / 6, l = k == 0 ? top : 3 - k;
      tail_setup_coef(A, l, tll[l], threadIdx.x % 6 + 1);
    }
    constexpr int P0 = 0, P1 = P0 + 4 * 4 * 4 * 4, P2 = P1 + 4 * 6 * 6 * 6;   // phi of 2^3, 4^3, 8^3
    constexpr int B0 = kTailLdsDoubles, B1 = B0 + 6 * 4, B2 = B1 + 6 * 16;    // their bc slots
    const int bt = (int)(XB.B - lds), ft = (int)(XB.F - lds);
#pragma unroll
    for (int r = 0; r < R; r++) {
      dst[r] = -1;
      src[r] = -1;
      bv[r] = 0.0;
      const int t = threadIdx.x + kTailBS * r;
      if (t >= NT) continue;
      const int q = t < O8 ? 0 : t < O4 ? 1 : t < O2 ? 2 : 3;   // top, 8^3, 4^3, 2^3
      const int l = q == 0 ? top : 3 - q;
      const int p = t - (q == 0 ? 0 : q == 1 ? O8 : q == 2 ? O4 : O2);
      const int ln = 4 - q, nc = 1 << ln, S = nc + 2;
      const int bofs = q == 0 ? bt : q == 1 ? B2 : q == 2 ? B1 : B0;
      const int fofs = q == 0 ? ft : (q == 1 ? P2 : q == 2 ? P1 : P0) + S * S * S;
      const int nb = (p >> (2 * ln)) + 1, cell = p & (nc * nc - 1), a = (cell & (nc - 1)) + 1, c = (cell >> ln) + 1;
      const TailLevel& T = A.lv[l];
      const int kind = T.L.nbk[nb - 1];
      const int ps = T.bc.phi_stored;
      const int fo = T.foff[nb - 1];
      const double val = T.bc.value[nb - 1];
      const double* fd = T.bc.face_data;
      if (kind != NB_PHYS) continue;
      dst[r] = bofs + p;
      const int d = (nb + 1) >> 1, g = (nb & 1) ? 0 : nc + 1;
      if (ps) {
        src[r] = fofs + (d == 1 ? g + S * (a + S * c) : d == 2 ? a + S * (g + S * c) : a + S * (c + S * g));
      } else if (fo != -1) {
        bv[r] = fd[(fo == -2 ? T.bc.face_off[nb - 1] : (long long)fo) + (a - 1) + (long long)nc * (c - 1)];
      } else {
        bv[r] = val;
      }
    }
  }
  __device__ __forceinline__ void commit(double* lds) const {
#pragma unroll
    for (int r = 0; r < R; r++)
      if (dst[r] >= 0) lds[dst[r]] = src[r] >= 0 ? lds[src[r]] : bv[r];
  }
};

// phi and rhs of the 16^3 top level (interior and face ghosts) HBM <-> LDS;
// only phi goes back
template <bool LOAD>
__device__ __forceinline__ void tail_big_io(const LevelView& L, const TailBox& X) {
  if (LOAD)
    tail_io_stored<16, 2, true>(L, X.P);
  else
    tail_io_stored<16, 1, false>(L, X.P);
  __syncthreads();
}

// update_coarse's fine part for the 16^3 top level in LDS: one parent cell
// per thread, its eight children's residuals (res = rhs - L phi, written to
// HBM as residual_box leaves them) summed as restrict_onto sums them, next to
// the sum of their phi
template <int OP>
__device__ __forceinline__ void tail_big_resid_restrict(const TailArgs& A, int li, const TailBox& X, const TailBox& Xc) {
  const LevelView& L = A.lv[li].L;
  const OpCoef<OP> K(L, A.lambda);
  const int dp = A.lv[li].dixp[0];
  const int dx = dp & 1023, dy = (dp >> 10) & 1023, dz = dp >> 20;
  double* res = boxp(L, 4, 0);
  for (int q = threadIdx.x; q < 8 * 8 * 8; q += blockDim.x) {
    const int i = q % 8 + 1, j = (q / 8) % 8 + 1, k = q / 64 + 1;
    double ap = 0.0, ar = 0.0;
    for (int kk = 0; kk < 2; kk++)
      for (int jj = 0; jj < 2; jj++)
        for (int ii = 0; ii < 2; ii++) {
          const int fi = 2 * i - 1 + ii, fj = 2 * j - 1 + jj, fk = 2 * k - 1 + kk, c = X.at(fi, fj, fk);
          const double r = X.F[c] - op_value<OP>(K, tail_nbr(X, X.P, c));
          res[off_int(L, fi, fj, fk)] = r;
          ap += X.P[c];
          ar += r;
        }
    Xc.P[Xc.at(dx + i, dy + j, dz + k)] = 0.125 * ap;
    Xc.R[Xc.at(dx + i, dy + j, dz + k)] = 0.125 * ar;
  }
  __syncthreads();
}

// mg_fill_ghost_cells_lvl of phi for the box in LDS: a periodic face copies
// the opposite boundary layer (what the owner pushes), a physical face is
// bc_to_gc's c0*bc + c1*x1 + c2*x2
template <int NC>
__device__ __forceinline__ void tail_lds_fill_nc(const TailLdsLevel& D, const TailBox& X) {
  constexpr int S = NC + 2, NF = 6 * NC * NC, R = (NF + kTailBS - 1) / kTailBS;
  int gd[R];
  double v[R];
#pragma unroll
  for (int r = 0; r < R; r++) {   // every face cell's reads first, then the ghost writes
    const int p = threadIdx.x + kTailBS * r;
    if (p >= NF) continue;
    const int nb = p / (NC * NC) + 1, cell = p % (NC * NC), a = cell % NC + 1, c = cell / NC + 1;
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1, g = low ? 0 : NC + 1, x1 = low ? 1 : NC, x2 = low ? 2 : NC - 1;
    auto cell_at = [&](int layer) {
      return d == 1 ? layer + S * (a + S * c) : d == 2 ? a + S * (layer + S * c) : a + S * (c + S * layer);
    };
    gd[r] = cell_at(g);
    if (D.local[nb - 1])
      v[r] = X.P[cell_at(low ? NC : 1)];
    else
      v[r] = D.c0[nb - 1] * X.B[p] + D.c1[nb - 1] * X.P[cell_at(x1)] + D.c2[nb - 1] * X.P[cell_at(x2)];
  }
#pragma unroll
  for (int r = 0; r < R; r++)
    if (threadIdx.x + kTailBS * r < NF) X.P[gd[r]] = v[r];
  __syncthreads();
}

__device__ __forceinline__ void tail_lds_fill(const TailLdsLevel& D, const TailBox& X) {
  // ghosts are written only from interior cells, so the reads may precede the writes
  if (X.nc == 16) return tail_lds_fill_nc<16>(D, X);
  const int nc = X.nc, nc2 = nc * nc, ln = X.ln;
  for (int p = threadIdx.x; p < 6 * nc2; p += blockDim.x) {
    const int nb = (p >> (2 * ln)) + 1, cell = p & (nc2 - 1), a = (cell & (nc - 1)) + 1, c = (cell >> ln) + 1;
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1, g = low ? 0 : nc + 1, x1 = low ? 1 : nc, x2 = low ? 2 : nc - 1;
    auto cell_at = [&](int layer) {
      return d == 1 ? X.at(layer, a, c) : d == 2 ? X.at(a, layer, c) : X.at(a, c, layer);
    };
    if (D.local[nb - 1]) {
      X.P[cell_at(g)] = X.P[cell_at(low ? nc : 1)];
      continue;
    }
    X.P[cell_at(g)] = D.c0[nb - 1] * X.B[p] + D.c1[nb - 1] * X.P[cell_at(x1)] + D.c2[nb - 1] * X.P[cell_at(x2)];
  }
  __syncthreads();
}


// update_coarse's parent part for the 16^3 top level (A.top_crhs): the ghost
// fill of phi in LDS, old = phi over the stored box and rhs = L(phi) + res on
// the interior, both to HBM (the level's rhs and old after the cycle, and the
// old its correction of top+1 reads), rhs into LDS for the smoothing; the
// arithmetic of k_fill_crhs / coarse_rhs_box on the same operands
// the top level's residuals, read before the fill (their loads in flight
// with the entry's)
struct TailCrhsRegs {
  static constexpr int N3 = 16 * 16 * 16, R = N3 / kTailBS;
  static_assert(N3 % kTailBS == 0, "whole rounds of interior cells");
  double rv[R];
  __device__ __forceinline__ void issue(const LevelView& L) {
    const double* res = boxp(L, 4, 0);
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int q = threadIdx.x + kTailBS * r;
      rv[r] = res[off_int(L, (q & 15) + 1, ((q >> 4) & 15) + 1, (q >> 8) + 1)];
    }
  }
};

template <int OP>
__device__ __forceinline__ void tail_big_crhs(const TailArgs& A, int li, const TailLdsLevel& D, const TailBox& X,
                                              const TailCrhsRegs& rr) {
  const LevelView& L = A.lv[li].L;
  const OpCoef<OP> K(L, A.lambda);
  constexpr int R = TailCrhsRegs::R;
  double* rhs = boxp(L, 2, 0);
  tail_lds_fill(D, X);
  tail_io_stored<16, 1, false, 3>(L, X.P);
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int q = threadIdx.x + kTailBS * r;
    const int i = (q & 15) + 1, j = ((q >> 4) & 15) + 1, k = (q >> 8) + 1, c = X.at(i, j, k);
    const double v = op_value<OP>(K, tail_nbr(X, X.P, c)) + rr.rv[r];
    X.F[c] = v;
    rhs[off_int(L, i, j, k)] = v;
  }
  __syncthreads();
}

// one red-black substep (colour e) of an NC^3 box in LDS: the cells of colour
// e only, i = 2*ih + 1 + p with (i+j+k) & 1 == e; colour e reads colour 1-e
// only (gs_value has no centre term), so all reads may precede the updates
template <int NC, int OP>
__device__ __forceinline__ void tail_rb_substep(const OpCoef<OP>& K, const TailBox& X, int e) {
  constexpr int S = NC + 2, H = NC / 2, NQ = NC * NC * NC / 2, R = (NQ + kTailBS - 1) / kTailBS;
  int cc[R];
  Nbr7 st[R];
  double f[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int q = threadIdx.x + kTailBS * r;
    if (q >= NQ) continue;
    const int ih = q % H, row = q / H, j = row % NC + 1, k = row / NC + 1;
    cc[r] = 2 * ih + 1 + ((1 + j + k + e) & 1) + S * (j + S * k);
    st[r] = tail_nbr(X, X.P, cc[r]);
    f[r] = X.F[cc[r]];
  }
#pragma unroll
  for (int r = 0; r < R; r++)
    if (threadIdx.x + kTailBS * r < NQ) X.P[cc[r]] = gs_value<OP>(K, st[r], f[r]);
}

// smooth_boxes: red-black substeps (colour e = n & 1 for n = 1 .. 2 n_cycle)
// or lexicographic sweeps (hyperplanes i+j+k = d, as gs_lex_box), each
// followed by the ghost fill
template <int OP, bool LEX>
__device__ __forceinline__ void tail_lds_smooth(const TailArgs& A, int li, const TailLdsLevel& D, const TailBox& X, int n_cycle) {
  const OpCoef<OP> K(A.lv[li].L, A.lambda);
  const int nc = X.nc, n3 = nc * nc * nc;
  if constexpr (LEX) {
    for (int n = 1; n <= n_cycle; n++) {
      for (int d = 3; d <= 3 * nc; d++) {
        for (int p = threadIdx.x; p < nc * nc; p += blockDim.x) {
          const int j = (p & (nc - 1)) + 1, k = (p >> X.ln) + 1, i = d - j - k;
          if (i < 1 || i > nc) continue;
          const int c = X.at(i, j, k);
          X.P[c] = gs_value<OP>(K, tail_nbr(X, X.P, c), X.F[c]);
        }
        __syncthreads();
      }
      tail_lds_fill(D, X);
    }
    return;
  }
  const int h = nc / 2;
  for (int n = 1; n <= 2 * n_cycle; n++) {
    const int e = n & 1;
    if (nc == 16) {   // the box size known at compile time: every read of a
                      // thread's cells issued before its first update
      tail_rb_substep<16, OP>(K, X, e);
      __syncthreads();
      tail_lds_fill(D, X);
      continue;
    }
    // the cells of colour e only: i = 2*ih + 1 + p with (i+j+k) & 1 == e
    for (int q = threadIdx.x; q < n3 / 2; q += blockDim.x) {
      const int ih = q & (h - 1), row = q >> (X.ln - 1), j = (row & (nc - 1)) + 1, k = (row >> X.ln) + 1;
      const int c = X.at(2 * ih + 1 + ((1 + j + k + e) & 1), j, k);
      X.P[c] = gs_value<OP>(K, tail_nbr(X, X.P, c), X.F[c]);
    }
    __syncthreads();
    tail_lds_fill(D, X);
  }
}

// residual_box (res = rhs - L phi) over the box, max |res| when asked, then
// restrict_onto of phi and res into the parent box Xc (sequential 8-cell sum
// from +0.0, i fastest, times 0.125)
template <int OP>
__device__ __forceinline__ double tail_lds_residual(const TailArgs& A, int li, const TailBox& X, const TailBox* Xc,
                                    double* red) {
  const OpCoef<OP> K(A.lv[li].L, A.lambda);
  const int nc = X.nc, n3 = nc * nc * nc;
  double mx = 0.0;
  const int ln = X.ln;
  for (int q = threadIdx.x; q < n3; q += blockDim.x) {
    const int c = X.at((q & (nc - 1)) + 1, ((q >> ln) & (nc - 1)) + 1, (q >> (2 * ln)) + 1);
    const double r = X.F[c] - op_value<OP>(K, tail_nbr(X, X.P, c));
    X.R[c] = r;
    mx = amax(mx, fabs(r));
  }
  if (red) {
    for (int off = 32; off > 0; off >>= 1) mx = amax(mx, __shfl_down(mx, off, 64));
    __syncthreads();   // every thread has read the previous maximum
    if (threadIdx.x == 0) *red = 0.0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned long long*>(red),
                                           (unsigned long long)__double_as_longlong(mx));
  }
  __syncthreads();
  if (Xc) {
    const int dp = A.lv[li].dixp[0];
    const int dx = dp & 1023, dy = (dp >> 10) & 1023, dz = dp >> 20, hn = nc / 2;
    const int lh = ln - 1;   // log2(hn)
    for (int t = threadIdx.x; t < 2 * hn * hn * hn; t += blockDim.x) {
      const int pass = t >> (3 * lh), q = t & (hn * hn * hn - 1);
      const int i = (q & (hn - 1)) + 1, j = ((q >> lh) & (hn - 1)) + 1, k = (q >> (2 * lh)) + 1;
      const double* src = pass ? X.R : X.P;
      double acc = 0.0;
      for (int kk = 0; kk < 2; kk++)
        for (int jj = 0; jj < 2; jj++)
          for (int ii = 0; ii < 2; ii++) acc += src[X.at(2 * i - 1 + ii, 2 * j - 1 + jj, 2 * k - 1 + kk)];
      (pass ? Xc->R : Xc->P)[Xc->at(dx + i, dy + j, dz + k)] = 0.125 * acc;
    }
    __syncthreads();
  }
  return red ? *red : 0.0;
}

// update_coarse's parent part: rhs = L(phi) + res on the interior, old = phi
// on the whole stored box
template <int OP>
__device__ __forceinline__ void tail_lds_coarse_rhs(const TailArgs& A, int li, const TailBox& X) {
  const OpCoef<OP> K(A.lv[li].L, A.lambda);
  const int nc = X.nc, s3 = X.S * X.S * X.S;
  for (int q = threadIdx.x; q < s3; q += blockDim.x) {
    const int i = q % X.S, j = (q / X.S) % X.S, k = q / (X.S * X.S);
    X.O[q] = X.P[q];
    if (i < 1 || i > nc || j < 1 || j > nc || k < 1 || k > nc) continue;
    X.F[q] = op_value<OP>(K, tail_nbr(X, X.P, q)) + X.R[q];
  }
  __syncthreads();
}

// correct_children of the parent Xc (res = phi - old over its stored cells)
// + mg_prolong_sparse onto the box + the ghost fill
template <int NC>
__device__ __forceinline__ void tail_correct_nc(const TailArgs& A, int li, const TailBox& X, const TailBox& Xc) {
  constexpr int S = NC + 2, SC = NC / 2 + 2, SC3 = SC * SC * SC, N3 = NC * NC * NC;
  constexpr int R = (N3 + kTailBS - 1) / kTailBS, RC = (SC3 + kTailBS - 1) / kTailBS;
#pragma unroll
  for (int r = 0; r < RC; r++) {
    const int q = threadIdx.x + kTailBS * r;
    if (q < SC3) Xc.R[q] = Xc.P[q] - Xc.O[q];
  }
  __syncthreads();
  const int dp = A.lv[li].dixp[0];
  const int dx = dp & 1023, dy = (dp >> 10) & 1023, dz = dp >> 20;
  int cc[R];
  double nv[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int q = threadIdx.x + kTailBS * r;
    if (q >= N3) continue;
    const int i = q % NC + 1, j = (q / NC) % NC + 1, k = q / (NC * NC) + 1;
    const int c0 = (((i + 1) >> 1) + dx) + SC * ((((j + 1) >> 1) + dy) + SC * (((k + 1) >> 1) + dz));
    const double f0 = 0.25 * Xc.R[c0];
    const double fx = 0.25 * Xc.R[(i & 1) ? c0 - 1 : c0 + 1];
    const double fy = 0.25 * Xc.R[(j & 1) ? c0 - SC : c0 + SC];
    const double fz = 0.25 * Xc.R[(k & 1) ? c0 - SC * SC : c0 + SC * SC];
    cc[r] = i + S * (j + S * k);
    nv[r] = X.P[cc[r]] + (f0 + fx + fy + fz);
  }
#pragma unroll
  for (int r = 0; r < R; r++)
    if (threadIdx.x + kTailBS * r < N3) X.P[cc[r]] = nv[r];
  __syncthreads();
}

__device__ __forceinline__ void tail_lds_correct(const TailArgs& A, int li, const TailLdsLevel& D, const TailBox& X,
                                 const TailBox& Xc) {
  if (X.nc == 16 && Xc.S == 10) {   // the 16^3 level, a one-box parent of half the size
    tail_correct_nc<16>(A, li, X, Xc);
    tail_lds_fill(D, X);
    return;
  }
  const int sc3 = Xc.S * Xc.S * Xc.S;
  for (int q = threadIdx.x; q < sc3; q += blockDim.x) Xc.R[q] = Xc.P[q] - Xc.O[q];
  __syncthreads();
  const int dp = A.lv[li].dixp[0];
  const int dx = dp & 1023, dy = (dp >> 10) & 1023, dz = dp >> 20, nc = X.nc, n3 = nc * nc * nc;
  const int ln = X.ln;
  for (int q = threadIdx.x; q < n3; q += blockDim.x) {
    const int i = (q & (nc - 1)) + 1, j = ((q >> ln) & (nc - 1)) + 1, k = (q >> (2 * ln)) + 1;
    const int c0 = Xc.at(((i + 1) >> 1) + dx, ((j + 1) >> 1) + dy, ((k + 1) >> 1) + dz);
    const double f0 = 0.25 * Xc.R[c0];
    const double fx = 0.25 * Xc.R[(i & 1) ? c0 - 1 : c0 + 1];
    const double fy = 0.25 * Xc.R[(j & 1) ? c0 - Xc.S : c0 + Xc.S];
    const double fz = 0.25 * Xc.R[(k & 1) ? c0 - Xc.S * Xc.S : c0 + Xc.S * Xc.S];
    const int c = X.at(i, j, k);
    X.P[c] = X.P[c] + (f0 + fx + fy + fz);
  }
  __syncthreads();
  tail_lds_fill(D, X);
}

template <int OP, bool LEX>
__global__ void __launch_bounds__(kTailBS) k_coarse_tail(const TailArgs* __restrict__ dA) {
  // the global-memory box programs' LDS, which also holds the LDS-resident
  // levels while they are in use (the two never overlap in time)
  constexpr int kSmall = kTailLdsDoubles + kTailLdsBcDoubles + kTailBigDoubles;
  __shared__ double lds[tail_lds<LEX>() > kSmall ? tail_lds<LEX>() : kSmall];
  __shared__ double red;
  __shared__ TailLdsLevel tll[kTailLdsLevels + 1];
  const TailArgs& A = *dA;
  const int top = A.n_lvls - 1;
  // levels 0..ls live in LDS, and with big the 16^3 top level above them
  // (phi, rhs); the host decided which (run_tail)
  const int ls = A.lds_levels - 1;
  const bool big = A.lds_top;
  const TailBox XB = tail_big_box(lds);
  int ns = 0;
  auto stamp = [&]() {
    if (A.stamps && threadIdx.x == 0) A.stamps[ns] = (long long)wall_clock64();
    ns++;
  };
  auto enter_lds = [&]() {
    tail_boxes_io<true>(A, ls, lds);
    for (int l = 0; l <= ls; l++) tail_lds_setup(A, l, tail_box(A, l, lds), tll[l]);
    __syncthreads();
  };
  stamp();
  if (ls == top) {
    enter_lds();
    if (A.top_crhs) {
      const TailBox X = tail_box(A, top, lds);
      tail_lds_fill(tll[top], X);
      tail_lds_coarse_rhs<OP>(A, top, X);
    }
  } else if (A.top_crhs && !big) {
    tail_fill(A, top);
    tail_coarse_rhs<OP>(A, top, lds);
  }
  if (big) {
    TailCrhsRegs rr;
    if (A.top_crhs) rr.issue(A.lv[top].L);
    if (ls == 2 && A.lv[0].L.nc == 2 && A.lv[1].L.nc == 4 && A.lv[2].L.nc == 8) {
      // the usual chain (16^3 over 8^3, 4^3, 2^3): every load of the entry
      // in flight at once
      TailIoRegs<16, 2> r16;
      TailIoRegs<8, 4> r8;
      TailIoRegs<4, 4> r4;
      TailIoRegs<2, 4> r2;
      r16.issue(A.lv[top].L);
      r8.issue(A.lv[2].L);
      r4.issue(A.lv[1].L);
      r2.issue(A.lv[0].L);
      TailChainBc cb;
      cb.issue(A, top, XB, lds, tll);
      stamp();
      r16.commit(XB.P);
      r8.commit(tail_box(A, 2, lds).P);
      r4.commit(tail_box(A, 1, lds).P);
      r2.commit(tail_box(A, 0, lds).P);
      __syncthreads();
      stamp();
      cb.commit(lds);
    } else {
      tail_big_io<true>(A.lv[top].L, XB);
      tail_boxes_io<true>(A, ls, lds);
      stamp();
      for (int l = 0; l <= ls; l++) tail_lds_setup(A, l, tail_box(A, l, lds), tll[l]);
      tail_lds_setup(A, top, XB, tll[top]);
    }
    __syncthreads();
    stamp();
    if (A.top_crhs) tail_big_crhs<OP>(A, top, tll[top], XB, rr);
    stamp();
    const TailBox Xc = tail_box(A, ls, lds);
    tail_lds_smooth<OP, LEX>(A, top, tll[top], XB, A.n_down);
    stamp();
    tail_big_resid_restrict<OP>(A, top, XB, Xc);
    stamp();
    tail_lds_fill(tll[ls], Xc);
    stamp();
    tail_lds_coarse_rhs<OP>(A, ls, Xc);
    stamp();
  }
  for (int li = big ? top - 1 : top; li >= 1; li--) {
    if (li <= ls) {
      const TailBox X = tail_box(A, li, lds), Xc = tail_box(A, li - 1, lds);
      tail_lds_smooth<OP, LEX>(A, li, tll[li], X, A.n_down);
      stamp();
      tail_lds_residual<OP>(A, li, X, &Xc, nullptr);
      stamp();
      tail_lds_fill(tll[li - 1], Xc);
      stamp();
      tail_lds_coarse_rhs<OP>(A, li - 1, Xc);
      stamp();
      continue;
    }
    tail_smooth<OP, LEX>(A, li, A.n_down, lds);
    stamp();
    tail_residual<OP>(A, li, 1, false, lds);   // update_coarse: residual + restriction of phi, res
    stamp();
    if (li - 1 == ls) {   // the level below goes to LDS now
      enter_lds();
      const TailBox Xc = tail_box(A, ls, lds);
      tail_lds_fill(tll[ls], Xc);
      stamp();
      tail_lds_coarse_rhs<OP>(A, ls, Xc);
      stamp();
      continue;
    }
    tail_fill(A, li - 1);
    stamp();
    tail_coarse_rhs<OP>(A, li - 1, lds);
    stamp();
  }
  // coarse solve (m_multigrid.f90:197-208)
  int its = 0;
  if (ls >= 0) {
    const TailBox X = tail_box(A, 0, lds);
    const double init_res = tail_lds_residual<OP>(A, 0, X, nullptr, &red);
    for (int i = 1; i <= A.max_coarse; i++) {
      tail_lds_smooth<OP, LEX>(A, 0, tll[0], X, A.n_up + A.n_down);
      its = i;
      const double res = tail_lds_residual<OP>(A, 0, X, nullptr, &red);
      if (res < A.res_rel * init_res || res < A.res_abs) break;
    }
  } else {
    const double init_res = tail_residual<OP>(A, 0, 0, true, lds);
    for (int i = 1; i <= A.max_coarse; i++) {
      tail_smooth<OP, LEX>(A, 0, A.n_up + A.n_down, lds);
      its = i;
      const double res = tail_residual<OP>(A, 0, 0, true, lds);
      if (res < A.res_rel * init_res || res < A.res_abs) break;
    }
  }
  stamp();
  for (int li = 1; li <= top; li++) {
    if (li <= ls || big) {
      const TailBox X = li <= ls ? tail_box(A, li, lds) : XB, Xc = tail_box(A, li - 1, lds);
      tail_lds_correct(A, li, tll[li], X, Xc);
      stamp();
      tail_lds_smooth<OP, LEX>(A, li, tll[li], X, A.n_up);
      stamp();
      continue;
    }
    if (li == ls + 1 && ls >= 0) tail_boxes_io<false>(A, ls, lds);   // the LDS levels back to HBM first
    tail_correct(A, li, lds);
    stamp();
    tail_smooth<OP, LEX>(A, li, A.n_up, lds);
    stamp();
  }
  if (ls == top || big) tail_boxes_io<false>(A, ls, lds);
  if (big) tail_big_io<false>(A.lv[top].L, XB);
  if (threadIdx.x == 0) *A.coarse_its = its;
}

// The tail's arguments into device memory, carried as a kernel argument (a
// captured graph keeps its own copy; a pageable memcpy node would read the host
// buffer when the graph runs).  The parameter itself is copied, word by word
// with vector stores (the compiler stages it wherever it likes: this one-block
// kernel runs only when the arguments change), so no assumption on where the
// by-value struct sits in the kernarg segment is made.
static_assert(sizeof(TailArgs) % 4 == 0, "TailArgs is copied as 32-bit words");
static_assert(sizeof(TailArgs) + sizeof(TailArgs*) <= 4096, "TailArgs must fit the 4 KiB kernel-argument limit");
static_assert(alignof(TailArgs) <= 8, "TailArgs alignment");
__global__ void __launch_bounds__(256) k_store_tail(TailArgs A, TailArgs* d) {
  const unsigned* s = reinterpret_cast<const unsigned*>(&A);
  unsigned* o = reinterpret_cast<unsigned*>(d);
  for (int i = threadIdx.x; i < (int)(sizeof(TailArgs) / 4); i += blockDim.x) o[i] = s[i];
}

void launch_store_tail(const TailArgs& A, TailArgs* d, hipStream_t st) {
  k_store_tail<<<1, 256, 0, st>>>(A, d);
}

void launch_coarse_tail(const TailArgs* dA, int gs_lex, int op, hipStream_t st) {
  if (op == OP_HELM) {
    if (gs_lex)
      k_coarse_tail<OP_HELM, true><<<1, kTailBS, 0, st>>>(dA);
    else
      k_coarse_tail<OP_HELM, false><<<1, kTailBS, 0, st>>>(dA);
  } else {
    if (gs_lex)
      k_coarse_tail<OP_LPL, true><<<1, kTailBS, 0, st>>>(dA);
    else
      k_coarse_tail<OP_LPL, false><<<1, kTailBS, 0, st>>>(dA);
  }
}



}  // namespace omg
