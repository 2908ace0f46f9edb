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
                       hipStream_t st, const int* boxes, int n_boxes) {
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
  const RbSide rbs{C, has_rb ? rb : nullptr};
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

// ---------------------------------------------------------------------------
// Small levels, all substeps of one smooth_boxes call in one launch.  A level
// of at most a few hundred boxes fills the GPU for a few microseconds per
// substep, so each substep launch is mostly latency: start-up, the box's
// first loads, the drain at the end.  Here every workgroup keeps its box (both
// colours and rhs) in LDS for the whole call and the substeps are separated by
// a grid barrier; per substep only the ghost halves the substep reads come
// from memory (where the neighbours pushed them), and the box goes back once
// at the end.  Same cells, operands and gs_value per substep as k_gsrb_tile,
// same pushes and physical / refinement-boundary ghosts: bit-identical.
//
// The barrier: one counter and one generation word (bar[0], bar[1]); the last
// workgroup to arrive resets the counter and advances the generation.  Every
// workgroup of the grid must be resident at once: the grid is at most the
// occupancy bound times the CU count (launch_gsrb_resident), and the wait is
// bounded, so a grid that is not resident sets bar[2] and ends instead of
// hanging (the host turns that into an error, check_grid_barrier).
__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned nblk, int* flag) {
  __threadfence();   // this thread's pushes, visible device-wide before arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    bool ok = true;
    const unsigned g = __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned old = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nblk - 1) {
      __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int spins = 0;
      while (__hip_atomic_load(bar + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 22)) {
          ok = false;
          __hip_atomic_fetch_or(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    *flag = ok;
  }
  __syncthreads();
  return *flag;
}

template <int NC>
constexpr int gsrb_res_lds() { return 4 * Tl<NC>::HV + 6 * Tl<NC>::FH; }

template <int NC, int OP, int BS, bool RB>
__global__ void __launch_bounds__(BS) k_gsrb_resident(LevelView L, double lambda, int n_first, int n_last, GcBC bc,
                                                      RbSide rbs, unsigned* bar) {
  using TL = Tl<NC>;
  constexpr int H = TL::H, HV = TL::HV, FH = TL::FH, FS = TL::FS, NP2 = (HV / 2 + BS - 1) / BS;
  constexpr int NF = 6 * NC * NC, NPF = (NF + BS - 1) / BS;
  static_assert(H % 2 == 0, "paired rows");
  __shared__ double lds[gsrb_res_lds<NC>()];
  __shared__ int flag;
  // lds: the interior (colour 0, colour 1), then rhs in the same layout
  double* rhs = lds + 2 * HV;
  double* sg = lds + 4 * HV;          // the read colour's ghost halves, 6 x FH
  const int tid = threadIdx.x;
  const int b = xcd_box(blockIdx.x, gridDim.x, L.rev);
  double* __restrict__ u = L.phi + (long long)b * L.stride;
  const OpCoef<OP> K(L, lambda);
  // the box and its rhs into LDS
  {
    const v2d* su = reinterpret_cast<const v2d*>(u);
    const v2d* sf = reinterpret_cast<const v2d*>(L.data + L.vstride + (long long)b * L.stride);
    for (int q = tid; q < HV; q += BS) {
      reinterpret_cast<v2d*>(lds)[q] = su[q];
      reinterpret_cast<v2d*>(rhs)[q] = sf[q];
    }
  }
  // face kinds, and the coarse half of every refinement-boundary ghost (the
  // coarse level is not written while this level is smoothed)
  int fkind[NPF], farg[NPF];
#pragma unroll
  for (int r = 0; r < NPF; r++) {
    const int p = tid + BS * r;
    const long long fidx = (long long)b * 6 + (p < NF ? p / (NC * NC) : 0);
    fkind[r] = p < NF ? L.nbk[fidx] : NB_LOCAL;
    farg[r] = p < NF ? L.nba[fidx] : 0;
  }
  RbCoarse rt[RB ? NPF : 1];
  if constexpr (RB) {
#pragma unroll
    for (int r = 0; r < NPF; r++) {
      if (fkind[r] != NB_RB) continue;
      const int p = tid + BS * r, cell = p % (NC * NC);
      rt[r] = rb_coarse_load(L, rbs, rbs.rb[farg[r]], p / (NC * NC) + 1, cell % NC + 1, cell / NC + 1);
    }
  }
  bool go = true;
  for (int n = n_first; n <= n_last && go; n++) {
    const int e = n & 1, o = 1 - e;
    const double* so = lds + o * HV;
    double* se = lds + e * HV;
    // the read colour's ghost halves: pushed by the neighbours during the
    // previous substep (or current on entry), physical / refinement-boundary
    // ones recomputed by this box
    for (int q = tid; q < 3 * FH; q += BS) {
      const int nb = q / (FH / 2), r = q % (FH / 2);
      reinterpret_cast<v2d*>(sg + nb * FH)[r] = reinterpret_cast<const v2d*>(u + 2 * HV + nb * FS + o * FH)[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NP2; r++) {
      const int q2 = tid + BS * r;
      if (q2 >= HV / 2) continue;
      const int q = 2 * q2;
      Nbr7 s0, s1;
      pair_stencil<NC>(so, sg, FH, e, q, s0, s1);
      const double2 f = reinterpret_cast<const double2*>(rhs + e * HV)[q2];
      double2 nv;
      if constexpr (is_varop(OP)) {
        AEps E0, E1;
        pair_eps<NC, OP>(L, b, e, q, E0, E1);
        nv = make_double2(ags_value<OP>(K, s0, E0, f.x), ags_value<OP>(K, s1, E1, f.y));
      } else {
        nv = make_double2(gs_value<OP>(K, s0, f.x), gs_value<OP>(K, s1, f.y));
      }
      reinterpret_cast<double2*>(se)[q2] = nv;
    }
    __syncthreads();
    auto cellv = [&](int i, int j, int k) { return lds[TL::oint(i, j, k)]; };
    face_push_local<NC>(L, b, 1 << e, cellv);
#pragma unroll
    for (int r = 0; r < NPF; r++) {
      const int p = tid + BS * r, kind = fkind[r];
      if (p >= NF || kind == NB_LOCAL) continue;
      const int nb = p / (NC * NC) + 1, cell = p % (NC * NC);
      const long long fidx = (long long)b * 6 + nb - 1;
      const int a = cell % NC + 1, c = cell / NC + 1;
      const bool low = nb & 1;
      const int d = (nb + 1) >> 1, x1 = low ? 1 : NC, x2 = low ? 2 : NC - 1;
      int i1, j1, k1;
      if (d == 1) { i1 = x1; j1 = a; k1 = c; }
      else if (d == 2) { i1 = a; j1 = x1; k1 = c; }
      else { i1 = a; j1 = c; k1 = x1; }
      const int i2 = d == 1 ? x2 : i1, j2 = d == 2 ? x2 : j1, k2 = d == 3 ? x2 : k1;
      const double v1 = cellv(i1, j1, k1), v2 = cellv(i2, j2, k2);
      const int gi = TL::ogh(nb, a, c);
      if (kind == NB_PHYS) {
        u[gi] = phys_ghost(L, bc, b, fidx, nb, farg[r], a, c, gi, v1, v2);
      } else if constexpr (RB) {
        if (kind == NB_RB) u[gi] = rb_ghost_from(rt[r], a, c, v1, v2);
      }
    }
    if (n < n_last) go = grid_barrier(bar, gridDim.x, &flag);
  }
  // the box back: both colours (every call runs at least the two substeps of
  // one cycle, or one, and then only colour e changed: writing both is exact)
  {
    v2d* du = reinterpret_cast<v2d*>(u);
    for (int q = tid; q < HV; q += BS) du[q] = reinterpret_cast<const v2d*>(lds)[q];
  }
}

int gsrb_resident_capacity(int nc, int op, bool has_rb) {
  (void)op;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 0;
  }
  int per_cu = 0;
  if (nc == 16) {
    if (has_rb)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_gsrb_resident<16, OP_LPL, 512, true>, 512, 0);
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_gsrb_resident<16, OP_LPL, 512, false>, 512, 0);
  } else if (nc == 8) {
    if (has_rb)
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_gsrb_resident<8, OP_LPL, 256, true>, 256, 0);
    else
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_gsrb_resident<8, OP_LPL, 256, false>, 256, 0);
  }
  return per_cu * cus;
}

bool launch_gsrb_resident(const LevelView& L, int op, double lambda, int n_first, int n_last, const LevelView& C,
                          const RBRec* rb, bool has_rb, const GcBC& bc, unsigned* bar, hipStream_t st) {
  if (L.n == 0 || n_last < n_first) return true;
  if ((L.nc != 16 && L.nc != 8) || (op != OP_LPL && op != OP_HELM)) return false;
  if (L.n > gsrb_resident_capacity(L.nc, op, has_rb)) return false;
  const RbSide rbs{C, has_rb ? rb : nullptr};
#define OMG_RES(NC, BS, OPV, RBV) \
  k_gsrb_resident<NC, OPV, BS, RBV><<<L.n, BS, 0, st>>>(L, lambda, n_first, n_last, bc, rbs, bar)
#define OMG_RES_OP(NC, BS, RBV)          \
  if (op == OP_HELM)                     \
    OMG_RES(NC, BS, OP_HELM, RBV);       \
  else                                   \
    OMG_RES(NC, BS, OP_LPL, RBV);
  if (L.nc == 16) {
    if (has_rb) { OMG_RES_OP(16, 512, true) } else { OMG_RES_OP(16, 512, false) }
  } else {
    if (has_rb) { OMG_RES_OP(8, 256, true) } else { OMG_RES_OP(8, 256, false) }
  }
#undef OMG_RES_OP
#undef OMG_RES
  return true;
}

}  // namespace omg
