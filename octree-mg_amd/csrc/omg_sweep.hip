// omg_sweep.hip — the LDS-tiled red-black Gauss-Seidel substep (the hot kernel).
//
// One launch = one substep of smooth_boxes over a whole level plus the ghost
// fill the reference runs after it (src/m_multigrid.f90:412-423):
//   for every box: colour e = (substep counter) mod 2 is updated from colour
//   1-e (box_gs_lpl / box_gs_helmh, m_laplacian.f90:52-114,
//   m_helmholtz.f90:49-108), then the box pushes its new colour-e boundary
//   values into the ghost faces of its same-GPU neighbours, recomputes its
//   physical-boundary ghosts (bc_to_gc, m_ghost_cells.f90:665-766) and packs
//   its faces toward other GPUs for the RCCL halo exchange.
//
// Traffic per box of 16^3 (colour-split layout, omg_device.h): colour 1-e of
// phi (16 KB) + its ghost halves (6 KB) + colour e of rhs (16 KB) in, colour e
// of phi (16 KB) + pushed ghost halves (6 KB) out: ~60 KB per substep, all
// contiguous, against the 48 KB the 12 B/cell algorithmic figure counts.
//
// Workgroup = one box; blockIdx is remapped so that each XCD walks one
// contiguous (Morton-ordered) run of boxes and neighbours share its L2.
// Colour e reads only colour 1-e and neighbours receive only colour e, so the
// in-place update and the pushes are race-free across workgroups.
#include "omg_device.h"
#include "omg_face.h"
#include "omg_kernels.h"

namespace omg {

typedef double v2d __attribute__((ext_vector_type(2)));

template <int NC, int OP, int BS, int NT>
__global__ void __launch_bounds__(BS) k_gsrb_tile(LevelView L, double lambda, int e, int colours, GcBC bc,
                                                  double* __restrict__ sendbuf, const double* __restrict__ shift) {
  constexpr int H = NC / 2, HV = H * NC * NC, FH = H * NC, FS = 2 * FH;
  constexpr int NP2 = (HV / 2 + BS - 1) / BS;  // double2 cell pairs per thread
  __shared__ double so[HV];                    // colour 1-e of the interior
  __shared__ double se[HV];                    // colour e, updated
  __shared__ double sg[6 * FH];                // colour 1-e halves of the ghost faces
  const int b = xcd_box(blockIdx.x, gridDim.x), tid = threadIdx.x, o = 1 - e;
  const long long boff = (long long)b * L.stride;
  double* __restrict__ u = L.phi + boff;
  const double* __restrict__ f = L.data + L.vstride + boff;
  const OpCoef<OP> K(L, lambda);

  // ---- stream in: colour 1-e, its ghost halves, colour e of rhs ----------
  {
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
  double2 fr[NP2];
#pragma unroll
  for (int r = 0; r < NP2; r++) {
    const int q2 = tid + BS * r;
    if (q2 < HV / 2) {
      const double2* fp = reinterpret_cast<const double2*>(f + e * HV) + q2;
      if (NT) {
        const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(fp));
        fr[r] = make_double2(t.x, t.y);
      } else {
        fr[r] = *fp;
      }
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
      nv = make_double2(gs_value<OP>(K, s0, fr[r].x), gs_value<OP>(K, s1, fr[r].y));
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
  for (int p = tid; p < 6 * NC * NC; p += BS) {
    const int nb = p / (NC * NC) + 1, cell = p % (NC * NC);
    const int a = cell % NC + 1, c = cell / NC + 1;
    const long long fidx = (long long)b * 6 + nb - 1;
    const int kind = L.nbk[fidx], arg = L.nba[fidx];
    const bool low = nb & 1;
    const int d = (nb + 1) >> 1;
    // boundary cell x1 (and x2) of this face: colour and index
    const int x1 = low ? 1 : NC, x2 = low ? 2 : NC - 1;
    int i1, j1, k1;
    if (d == 1) { i1 = x1; j1 = a; k1 = c; }
    else if (d == 2) { i1 = a; j1 = x1; k1 = c; }
    else { i1 = a; j1 = c; k1 = x1; }
    const int c1 = (i1 + j1 + k1) & 1;
    const int idx1 = ((i1 - 1) >> 1) + H * ((j1 - 1) + NC * (k1 - 1));
    const double v1 = c1 == e ? se[idx1] : so[idx1];
    if (kind == NB_LOCAL) {
      if ((colours >> c1) & 1) {
        double* gp = L.phi + (long long)arg * L.stride + off_gh(L, low ? nb + 1 : nb - 1, a, c);
        if (NT >= 2)
          __builtin_nontemporal_store(v1, gp);
        else
          *gp = v1;
      }
    } else if (kind == NB_REMOTE) {
      sendbuf[(long long)L.sendpos[fidx] * NC * NC + (a - 1) + NC * (c - 1)] = v1;
    } else {  // NB_PHYS (refinement boundaries take the generic kernel)
      const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
      const int idx2 = ((i2 - 1) >> 1) + H * ((j2 - 1) + NC * (k2 - 1));
      const double v2 = c1 == e ? so[idx2] : se[idx2];   // x2 has the other colour
      const int gi = off_gh(L, nb, a, c);
      u[gi] = phys_ghost(L, bc, b, fidx, nb, arg, a, c, gi, v1, v2);
    }
  }
}

void launch_gs_substep(const LevelView& L, int op, double lambda, int e, int colours, const LevelView& C,
                       const RBRec* rb, bool has_rb, const GcBC& bc, double* sendbuf, const double* shift,
                       hipStream_t st) {
  if (L.n == 0) return;
  if (!gs_tiled(L.nc, op, has_rb)) {
    launch_gs_sub(L, op, lambda, e, colours, C, rb, bc, sendbuf, st);
    return;
  }
  GcBC b2 = bc;
  b2.phi_stored = bc.phi_stored;  // iv == 1 here
  // 16^3 boxes: 8 waves per box (4 boxes = 32 waves per CU, the LDS of 4
  // boxes fits); streaming loads/stores are non-temporal: nothing a substep
  // reads or writes is touched again before the next substep has swept the
  // level, far beyond L2 / MALL at the sizes that matter.
  const dim3 g(L.n);
#define OMG_TILE(NC, BS)                                                                   \
  if (op == OP_HELM)                                                                       \
    k_gsrb_tile<NC, OP_HELM, BS, 2><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift); \
  else                                                                                     \
    k_gsrb_tile<NC, OP_LPL, BS, 2><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift);
  switch (L.nc) {
    case 16: OMG_TILE(16, 512) break;
    case 8: OMG_TILE(8, 256) break;
    case 4: OMG_TILE(4, 256) break;
    default: OMG_TILE(2, 256) break;
  }
#undef OMG_TILE
}

}  // namespace omg
