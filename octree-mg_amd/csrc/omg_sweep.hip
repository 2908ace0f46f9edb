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
#include "omg_gsrb.h"
#include "omg_kernels.h"

namespace omg {


template <int NC, int OP, int BS, int NT, bool RB>
__global__ void __launch_bounds__(BS) k_gsrb_tile(LevelView L, double lambda, int e, int colours, GcBC bc,
                                                  double* __restrict__ sendbuf, const double* __restrict__ shift,
                                                  const int* __restrict__ boxes, RbSide rbs) {
  __shared__ double lds[gsrb_lds<NC>()];
  const int q = xcd_box(blockIdx.x, gridDim.x, L.rev);
  gsrb_box<NC, OP, BS, NT, false, RB>(L, lambda, e, colours, bc, sendbuf, shift, boxes ? boxes[q] : q, lds,
                                      nullptr, &rbs);
}

void launch_gs_substep(const LevelView& L, int op, double lambda, int e, int colours, const LevelView& C,
                       const RBRec* rb, bool has_rb, const GcBC& bc, double* sendbuf, const double* shift,
                       hipStream_t st, const int* boxes, int n_boxes, double* rbgv, int rbgv_mode) {
  if (L.n == 0) return;
  if (boxes && !gs_tiled(L.nc, op, has_rb)) return;   // subsets only exist for the tiled kernel
  if (!gs_tiled(L.nc, op, has_rb)) {
    launch_gs_sub(L, op, lambda, e, colours, C, rb, bc, sendbuf, st);
    return;
  }
  GcBC b2 = bc;
  b2.phi_stored = bc.phi_stored;  // iv == 1 here
  // 16^3 boxes: 8 waves per box (4 boxes = 32 waves per CU, the LDS of 4
  // boxes fits); streaming loads/stores are non-temporal on large levels:
  // nothing a substep reads or writes is touched again before the next
  // substep has swept the level, far beyond L2 / MALL.  A level whose phi and
  // rhs fit in about 1.5x the 256 MiB Infinity Cache streams with the default
  // policy, so that the next pass (walking the other way) re-reads what this
  // one touched last from the cache (kGsCachedBytes).
  // Measured -1 to -2 % per cycle at 256^3 (Laplacian, Helmholtz); the
  // operators that also read eps lost 2-8 % and stay non-temporal.
  constexpr long long kGsCachedBytes = 400ll << 20;
  const bool cached = (op == OP_LPL || op == OP_HELM) && 2ll * 8 * L.stride * L.n <= kGsCachedBytes;
  const dim3 g(boxes ? n_boxes : L.n);
  if (g.x == 0) return;
  const RbSide rbs{C, has_rb ? rb : nullptr, rbgv, rbgv ? rbgv_mode : 0};
  // NT 2: non-temporal streams, 0: default policy (the cached levels)
#define OMG_TILE_OP(NC, BS, NT, RB, OPV) \
  k_gsrb_tile<NC, OPV, BS, NT, RB><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift, boxes, rbs)
#define OMG_TILE_RB(NC, BS, NT, RB)                               \
  switch (op) {                                                   \
    case OP_HELM: OMG_TILE_OP(NC, BS, NT, RB, OP_HELM); break;    \
    case OP_VLPL: OMG_TILE_OP(NC, BS, NT, RB, OP_VLPL); break;    \
    case OP_VHELM: OMG_TILE_OP(NC, BS, NT, RB, OP_VHELM); break;  \
    case OP_AHELM: OMG_TILE_OP(NC, BS, NT, RB, OP_AHELM); break;  \
    default: OMG_TILE_OP(NC, BS, NT, RB, OP_LPL);                 \
  }
#define OMG_TILE(NC, BS, NT)          \
  if (has_rb)                         \
    OMG_TILE_RB(NC, BS, NT, true)     \
  else                                \
    OMG_TILE_RB(NC, BS, NT, false)
  switch (L.nc) {
    case 16:
      if (cached) {
        OMG_TILE(16, 512, 0)
      } else {
        OMG_TILE(16, 512, 2)
      }
      break;
    case 8: OMG_TILE(8, 256, 2) break;
    case 4: OMG_TILE(4, 256, 2) break;
    default: OMG_TILE(2, 256, 2) break;
  }
#undef OMG_TILE
#undef OMG_TILE_RB
#undef OMG_TILE_OP
}

// The ghosts of phi on the physical and refinement-boundary faces of the
// listed boxes, formed from their stored (final) boundary cells as the fill
// after a substep forms them (bc_to_gc, m_ghost_cells.f90:665-766; sides_rb
// over box_gc_for_fine_neighbor, :500-577, 769-861).  Runs after a split
// fused down-step (update_coarse): the boundary boxes' plain substep wrote
// only the colour-e halves of those ghosts, because the fused interior
// boxes' edge taps read the other halves as they stood before the substep.
__global__ void __launch_bounds__(256) k_face_gc(LevelView L, LevelView C, GcBC bc, const int* __restrict__ boxes) {
  const int b = boxes[blockIdx.x];
  const FaceTopo T = load_topo(L, b);
  double* u = boxp(L, 1, b);
  const int nc = L.nc, n2 = nc * nc;
  const RbSide R{C, nullptr, nullptr, 0};
  for (int p = threadIdx.x; p < 6 * n2; p += blockDim.x) {
    const int f = p / n2, nb = f + 1, a = p % nc + 1, c = (p % n2) / nc + 1;
    const int kind = T.kind(f);
    if (kind != NB_PHYS && kind != NB_RB) continue;
    const bool low = nb & 1;
    const int x1 = low ? 1 : nc, x2 = low ? 2 : nc - 1, gi = off_gh(L, nb, a, c);
    const double v1 = u[off_face_cell(L, nb, x1, a, c)], v2 = u[off_face_cell(L, nb, x2, a, c)];
    u[gi] = kind == NB_PHYS ? phys_ghost(L, bc, b, (long long)b * 6 + f, nb, T.phys_code(f), a, c, gi, v1, v2)
                            : rb_ghost(L, R, T.arg(f), nb, a, c, v1, v2);
  }
}

void launch_face_gc(const LevelView& L, const LevelView& C, const GcBC& bc, const int* boxes, int n_boxes,
                    hipStream_t st) {
  if (n_boxes > 0) k_face_gc<<<n_boxes, 256, 0, st>>>(L, C, bc, boxes);
}

}  // namespace omg
