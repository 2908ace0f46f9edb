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
  // one touched last from the cache (OMG_GS_NT_BYTES: the bound, bytes).
  // Measured -1 to -2 % per cycle at 256^3 (Laplacian, Helmholtz); the
  // operators that also read eps lost 2-8 % and stay non-temporal.
  static const long long nt_bytes = getenv("OMG_GS_NT_BYTES") ? atoll(getenv("OMG_GS_NT_BYTES")) : 400ll << 20;
  const bool cached = (op == OP_LPL || op == OP_HELM) && 2ll * 8 * L.stride * L.n <= nt_bytes;
  const dim3 g(boxes ? n_boxes : L.n);
  if (g.x == 0) return;
  const RbSide rbs{C, has_rb ? rb : nullptr, rbgv, rbgv ? rbgv_mode : 0};
#ifndef OMG_GS_NT
#define OMG_GS_NT 2
#endif
#define OMG_GS_NT_NOW OMG_GS_NT
#define OMG_TILE_RB(NC, BS, RB)                                                                    \
  switch (op) {                                                                                      \
    case OP_HELM:                                                                                    \
      k_gsrb_tile<NC, OP_HELM, BS, OMG_GS_NT_NOW, RB><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift, boxes, rbs); \
      break;                                                                                         \
    case OP_VLPL:                                                                                    \
      k_gsrb_tile<NC, OP_VLPL, BS, OMG_GS_NT_NOW, RB><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift, boxes, rbs); \
      break;                                                                                         \
    case OP_VHELM:                                                                                   \
      k_gsrb_tile<NC, OP_VHELM, BS, OMG_GS_NT_NOW, RB><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift, boxes, rbs); \
      break;                                                                                         \
    case OP_AHELM:                                                                                   \
      k_gsrb_tile<NC, OP_AHELM, BS, OMG_GS_NT_NOW, RB><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift, boxes, rbs); \
      break;                                                                                         \
    default:                                                                                         \
      k_gsrb_tile<NC, OP_LPL, BS, OMG_GS_NT_NOW, RB><<<g, dim3(BS), 0, st>>>(L, lambda, e, colours, b2, sendbuf, shift, boxes, rbs); \
  }
#define OMG_TILE(NC, BS)          \
  if (has_rb)                     \
    OMG_TILE_RB(NC, BS, true)     \
  else                            \
    OMG_TILE_RB(NC, BS, false)
  switch (L.nc) {
    case 16:
      if (cached) {
#undef OMG_GS_NT_NOW
#define OMG_GS_NT_NOW 0
        OMG_TILE(16, 512)
      } else {
#undef OMG_GS_NT_NOW
#define OMG_GS_NT_NOW OMG_GS_NT
        OMG_TILE(16, 512)
      }
      break;
    case 8: OMG_TILE(8, 256) break;
    case 4: OMG_TILE(4, 256) break;
    default: OMG_TILE(2, 256) break;
  }
#undef OMG_TILE
#undef OMG_TILE_RB
}

}  // namespace omg
