// omg_block.hip — three red-black substeps of a level in one pass (k_gsrb3).
//
// smooth_boxes (m_multigrid.f90:404-424) runs substeps e, 1-e, e with a ghost
// fill after each; every substep of the one-substep kernel (omg_sweep.hip)
// streams half of phi and half of rhs in and half of phi out (12 B per cell
// plus the ghost halves), so three cost 36 B per cell.  Here one workgroup
// streams a column of boxes plane by plane (z) and runs the three substeps as
// a pipeline over the planes (2.5-D temporal blocking): each plane of phi and
// rhs is read once and the final plane written once, 24 B per cell plus the
// pushed ghost faces.
//
// Tile: one box's 16 x 16 columns and three halo columns on each side
// (22 x 22, one thread per column), read from the eight boxes around the box
// in x and y.  At plane iteration t the thread holds the loaded plane t
// (stage 0) and computes stage 1 (substep 1) at plane t-1, stage 2 at t-2 and
// stage 3 at t-3: each stage's z neighbours are the same thread's registers
// (the stage below, one plane lower and the one just computed one plane
// higher), its x / y neighbours the stage below's plane in LDS, written at
// iteration t-1.  Stage s is valid on the columns at distance <= 3-s from the
// box (stage 3 on the box), and the first three planes below and above the
// column only feed the pipeline.  Cells that a substep does not update keep
// the value of the stage below.  The operands of every update are the values
// the reference's substep reads (the neighbours' boundary cells are its ghost
// values after the fill), in the same expression: bit-identical.
//
// In place would race (the halo columns are other workgroups' boxes), so the
// pass reads one phi buffer and writes the level's other one (the host swaps
// Level::d_phi): every interior cell, and every box's six ghost faces, pushed
// by the box that owns the cell.  Levels whose faces are all same-GPU boxes
// (or proxies of other GPUs' boxes, the deep halo) or physical (round 6:
// constant boundary values, B3Phys), 16^3 boxes, Laplacian / Helmholtz, with
// consistent ghosts on entry (same-GPU ones are not read: a neighbour's cells
// are read in its box; physical ones are, by the first substep).
#include <stdexcept>

#include "omg_device.h"
#include "omg_face.h"
#include "omg_kernels.h"

namespace omg {

namespace {

constexpr int B3NC = 16, B3H = 8, B3HV = B3H * B3NC * B3NC, B3FH = B3H * B3NC, B3FS = 2 * B3FH;
constexpr int B3NPX = (kB3TX * B3NC + 8) / 2;   // cell pairs per row: x in [-4, kB3TX*16+3]
constexpr int B3NY = B3NC + 6;                   // rows: y in [-3, 18]
constexpr int B3NT = B3NPX * B3NY;               // compute threads with a pair
constexpr int B3NW = (B3NT + 63) / 64;           // compute waves
constexpr int B3BS = 64 * (B3NW + 1);            // and the store wave
constexpr int B3CP = kB3TX * B3H;                // pairs per row of the tile's boxes
constexpr int B3LP = B3NPX + 2;                  // LDS row pitch (a pad pair on each side)
constexpr int B3PL = B3LP * (B3NY + 2);          // LDS doubles per plane (a pad row on each side)
constexpr int B3XS = kB3TX + 2;                  // record slots per row
// planes of loads in flight (2 / 3 / 4 / 5 / 6 ahead measured: 4 best, C3
// 4.68 ms; more costs a workgroup per CU, profiles/r05/s17)
constexpr int kB3Ahead = 4;
// every thread loads its own cells' rhs (false: only where a substep's result
// is used, tools/b3p_variants.py "rhsall" sets it true for the A/B)
constexpr bool kB3HaloRhs = false;
static_assert(kB3Ahead % 2 == 0, "coarse planes are loaded on the even planes' steps");
// the correction form: the coarse tile of a plane, cx in [-2, kB3TX*8+1] and
// cy in [-2, 9] around the column's coarse cells: the parents and x / y taps
// of the fine cells the pass uses (within 3 cells of the boxes; the pairs'
// outer cells at 4 read a neighbouring tile entry instead, unused), in a
// ring of four coarse planes
static_assert(kB3TX == 2, "a column spans one coarse box in x");
constexpr int B3CO = 2;                                  // tile offset of cx, cy = 0
constexpr int B3CX = kB3TX * B3H + 2 * B3CO, B3CY = B3H + 2 * B3CO, B3CT = B3CX * B3CY;

// ghost slot of face nb (1..6) at tangential (a, c) (omg_device.h off_gh)
__device__ __forceinline__ int b3_gh(int nb, int a, int c) {
  const int g = (nb & 1) ? 0 : B3NC + 1;
  return 2 * B3HV + (nb - 1) * B3FS + ((g + a + c) & 1) * B3FH + ((a - 1) >> 1) + B3H * (c - 1);
}

// an opaque register copy: the loaded value dies here, so the next load can
// land in its register (a plain copy keeps the loaded register alive for as
// long as the copy lives, and the loop then moves in-flight loads around,
// which waits for them)
__device__ __forceinline__ double b3_take(double v) {
  double r;
  asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// A store the compiler does not count.  Only the store wave stores, but the
// compiler's s_waitcnt bookkeeping merges the store wave's path into the
// compute waves' (one kernel), and once stores and loads are both pending it
// treats vmcnt as out of order and waits for vmcnt(0) at every load use,
// which would drain the loads in flight.  Nothing in the kernel reads what
// these write.  base: wave-uniform, off: bytes (< 4 GiB).  Non-temporal:
// nothing re-reads the pass's output before it leaves the L2 (C3 4.49 against
// 4.38 ms per cycle with nt, profiles/r05/s31_block3_ntst_ab.txt).
__device__ __forceinline__ void b3_st(double* base, unsigned off, double v) {
  asm volatile("global_store_dwordx2 %0, %1, %2 nt\n\ts_nop 1" : : "v"(off), "v"(v), "s"(base));
}
// two consecutive doubles, 16-B aligned (the store wave's interior and z-face
// stores: two neighbouring pairs of a row per lane)
__device__ __forceinline__ void b3_st2(double* base, unsigned off, v2d v) {
  asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 1" : : "v"(off), "v"(v), "s"(base));
}
__device__ __forceinline__ double b3_ld(const double* base, unsigned off) {
  return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + off);
}

// The ghost across a physical face, bc_to_gc's c0 * b + c1 * x1 + c2 * x2
// (m_ghost_cells.f90:665-766) in its order, k = c0 * b: x1 the cell next to
// the face, x2 the one behind it
__device__ __forceinline__ double b3_bc(double k, double c1, double c2, double x1, double x2) {
  return (k + c1 * x1) + c2 * x2;
}

// A compute thread's share of a column's physical faces (PHYS passes).
// Where the column has one, nothing lies beyond it: the reference reads the
// ghost layer, filled by bc_to_gc after every substep from the cells next to
// the face.  Substep 1 reads the ghosts as they are on entry (consistent), so
// the thread whose pair is across the face loads its colour-(1-e) ghost
// there instead of a neighbour's cell (the slot across the face names the
// box whose face it is; xyq, kq: the ghost's offset from src and bytes per
// plane).  Later substeps form the ghost where it is read: bx / by = 1 (2)
// when the thread's pair is next to face x- (x+) / y- (y+), whose ghost
// then comes from the cell's own value before the substep and the one behind
// it.  Everything else beyond a physical face is computed and never used.
// (k, c1, c2 of the thread's x and y faces are held in registers and every
// substep forms both ghosts and selects them: in LDS, read in branches taken
// by some lanes, the formation cost C2's 4096-box level 88 us a pass,
// profiles/r06/s15_phys_variants.txt.)
struct B3Face {
  unsigned xyq, kq;
  int bx, by;
  double kx, c1x, c2x, ky, c1y, c2y;
};
__device__ __forceinline__ B3Face b3_face(const B3Phys& P, int fl, int p, int npx, int y, int ih, int j, int e,
                                          unsigned xyb, unsigned pb) {
  B3Face f;
  constexpr int HV = 8 * 16 * 16, FH = 8 * 16, FS = 2 * FH;
  f.xyq = xyb;
  f.kq = pb;
  const int gx = (fl & 1) && p == 1 ? 1 : ((fl & 2) && p == npx - 2 ? 2 : 0);
  const int gy = (fl & 4) && y == -1 ? 1 : ((fl & 8) && y == 16 ? 2 : 0);
  if (gx || gy) {
    // face gx-1 (x) at (j, k), or 1+gy (y) at (i, k): its colour-(1-e) half
    const int o = gx ? 2 * HV + (gx - 1) * FS + (1 - e) * FH + ((j - 1) >> 1)
                     : 2 * HV + (1 + gy) * FS + (1 - e) * FH + ih;
    f.xyq = 8u * (unsigned)(o - (1 - e) * HV);
    f.kq = 8u * 8u;
  }
  f.bx = (fl & 1) && p == 2 ? 1 : ((fl & 2) && p == npx - 3 ? 2 : 0);
  f.by = (fl & 4) && y == 0 ? 1 : ((fl & 8) && y == 15 ? 2 : 0);
  const bool hx = f.bx == 2, hy = f.by == 2;
  f.kx = hx ? P.k[1] : P.k[0]; f.c1x = hx ? P.c1[1] : P.c1[0]; f.c2x = hx ? P.c2[1] : P.c2[0];
  f.ky = hy ? P.k[3] : P.k[2]; f.c1y = hy ? P.c1[3] : P.c1[2]; f.c2y = hy ? P.c2[3] : P.c2[2];
  return f;
}

// the neighbours of a PHYS pass's update at plane ts across the column's
// physical faces (own: the cell's value before the substep); lft: the pair's
// active cell is its left one (n.xm is then the x- neighbour, else x+)
__device__ __forceinline__ void b3_fix(Nbr7& n, const B3Face& f, const B3Phys& P, int fl, bool lft, double own,
                                       int ts, int zend) {
  const double gx = b3_bc(f.kx, f.c1x, f.c2x, own, n.xp);
  const double gy = b3_bc(f.ky, f.c1y, f.c2y, own, f.by == 2 ? n.ym : n.yp);
  n.xm = ((f.bx == 1 && lft) || (f.bx == 2 && !lft)) ? gx : n.xm;
  n.ym = f.by == 1 ? gy : n.ym;
  n.yp = f.by == 2 ? gy : n.yp;
  if ((fl & 16) && ts == 0) n.zm = b3_bc(P.k[4], P.c1[4], P.c2[4], own, n.zp);
  if ((fl & 32) && ts == zend - 1) n.zp = b3_bc(P.k[5], P.c1[5], P.c2[5], own, n.zm);
}

}  // namespace

// Workgroup = B3NW compute waves and one store wave.  A compute thread holds
// one pair of x-neighbour cells (x0, x0+1), x0 even, in one row: one cell of
// each colour in every plane.  Every substep updates exactly one cell of the
// pair, the colour-e cell (stages 1 and 3) or the colour-(1-e) one (stage 2),
// and its six operands are the pair's other cell (register), the neighbour
// pair's cell across (LDS), the same pair in the rows above and below (LDS)
// and the same column one plane down and up (registers).  The three active
// cells of one iteration (planes t-1, t-2, t-3) lie on the same side of the
// pair; the update adds its two x operands in either order (x+ + x- = x- + x+
// exactly), so the side needs no select.  The stage planes in LDS hold one
// value per pair (the colour that stage wrote).  Colour e of phi is not read:
// substep 1 overwrites it without reading it (the operators here have no
// centre term in the update), as the one-substep kernel does.
//
// The compute waves issue no store: a wave's loads and stores share one
// counter (vmcnt), so a wave that stores waits for its stores at every later
// wait for a load, and the loads run kB3Ahead planes ahead only if nothing
// else is pending.  The final plane t-3 goes to LDS; the store wave writes it
// to HBM during the next iteration, with every ghost face it is part of.
// Addresses are 32-bit byte offsets from wave-uniform bases (the host admits
// levels whose phi and rhs each stay under 4 GiB).
//
// PRO (the correct_children form, launch_gsrb3's `coarse`): the pass starts
// from phi before correct_children.  The colour 1-e it reads gets the
// prolonged correction as it is loaded (prolong_at's expression, omg_tiles.hip,
// from the coarse tile in LDS: phi - old of the coarse level, a plane of it
// loaded on every other step, kB3Ahead steps ahead like the fine planes);
// colour e needs none (substep 1 overwrites it).  PRO 1: the tile is formed
// from the coarse phi and old, and the store wave also stores the coarse
// level's res = phi - old, which correct_children leaves there (the column's
// own coarse cells, interior and the faces they are ghosts of); PRO 2: the
// coarse level's last pass stored res already (RES), the tile loads it.
// RES: the pass is the level's last up-smoothing pass and the level above
// takes PRO 2: with the final plane the compute waves form res = phi - old
// (old loaded with the plane kB3Ahead ahead), and the store wave stores it
// with its ghost faces like phi.
template <int OP, int PRO, bool RES, bool PHYS>
__global__ void __launch_bounds__(B3BS) k_gsrb3(LevelView L, double* __restrict__ dst,
                                                          const int* __restrict__ cols, double lambda, int e,
                                                          const double* __restrict__ shift, int push1, LevelView C,
                                                          const int* __restrict__ ccols, B3Phys P) {
  static_assert(!(PHYS && (PRO || RES)), "k_gsrb3: physical faces in the plain form only");
  __shared__ double pl[2][3][B3PL];
  // final plane: [row * B3CP + pair][colour e, 1-e (, their res)]
  // (PHYS: a ring of three, the z ghosts read the plane before)
  __shared__ double fin[PHYS ? 3 : 2][B3NC * B3CP][RES ? 4 : 2];
  auto fsl = [](int z) { return PHYS ? (z + 12) % 3 : z & 1; };
  __shared__ unsigned bo[kB3Rec];             // the record's boxes as byte offsets into a variable
  __shared__ double rc[PRO ? 4 : 1][PRO ? B3CT : 1];   // coarse phi - old, plane c in rc[c & 3]
  __shared__ unsigned cbo[PRO ? kB3CSlots : 1];   // the coarse record, byte offsets
  __shared__ int len_s, cyo_s, fl_s;
  __shared__ double pk[PHYS ? 18 : 1];
  const int tid = threadIdx.x;
  const int cq = xcd_box(blockIdx.x, gridDim.x);
  if (PHYS && tid >= B3BS - 18) pk[tid - (B3BS - 18)] = (&P.k[0])[tid - (B3BS - 18)];
  if (tid < kB3Rec) {
    const int v = cols[(long long)cq * kB3Rec + tid];
    if (tid == 0) {
      len_s = v & kB3LenMask;
      fl_s = v >> 8;
    } else {
      bo[tid - 1] = (unsigned)v * (unsigned)(L.stride * 8);
    }
  }
  if (PRO) {
    const int q = tid - kB3Rec;
    if (q >= 0 && q < 1 + kB3CSlots) {
      const int v = ccols[(long long)cq * kB3CRec + q];
      if (q == 0) cyo_s = v;
      else cbo[q - 1] = (unsigned)v * (unsigned)(C.stride * 8);
    }
    for (int q2 = tid; q2 < 4 * B3CT; q2 += B3BS) (&rc[0][0])[q2] = 0.0;
  }
  for (int q = tid; q < 2 * 3 * B3PL; q += B3BS) (&pl[0][0][0])[q] = 0.0;
  __syncthreads();
  const int len = len_s, zend = B3NC * len;
  const int fl = PHYS ? fl_s : 0;
  constexpr unsigned PB = 8u * B3H * B3NC;   // bytes per plane of one colour
  auto zbox = [&](int t, int& k) {
    const int zs = t < 0 ? 0 : (t >= zend ? len + 1 : (t >> 4) + 1);
    k = t - B3NC * (zs - 1) + 1;
    return zs;
  };
  // ---- PRO: the coarse tile cell this thread loads (cx, cy relative to the
  // column's first coarse cell; threads past the tile load a duplicate)
  const int cyo = PRO ? cyo_s : 0, lenc = len >> 1;
  const double* __restrict__ cold = C.data + 2 * C.vstride;
  const double* __restrict__ cres_in = C.data + 3 * C.vstride;
  const int ct = tid < B3CT ? tid : B3CT - 1;
  const int cxr = ct % B3CX - B3CO, cyy = cyo + ct / B3CX - B3CO;
  const int xsc = cxr < 0 ? 0 : (cxr < B3NC ? 1 : 2), ysc = cyy < 0 ? 0 : (cyy < B3NC ? 1 : 2);
  const int icc = cxr - B3NC * (xsc - 1) + 1, jcc = cyy - B3NC * (ysc - 1) + 1;
  const unsigned cxy = 8u * (((icc - 1) >> 1) + B3H * (jcc - 1));
  auto cload = [&](int c, double& a, double& b) {
    const int zsc = c < 0 ? 0 : (c >= B3NC * lenc ? lenc + 1 : (c >> 4) + 1);
    const int kc = c - B3NC * (zsc - 1) + 1;
    const unsigned o = cbo[9 * zsc + 3 * ysc + xsc] + 8u * B3HV * ((icc + jcc + kc) & 1) + cxy + PB * (kc - 1);
    if (PRO == 2) {
      a = b3_ld(cres_in, o);
      b = 0.0;
    } else {
      a = b3_ld(C.phi, o);
      b = b3_ld(cold, o);
    }
  };
  if (PRO) {
    // coarse planes -2 and -1 (the first fine planes' parents and z taps)
    // before the loop, whose loads reach plane 0 first
    if (tid < B3NW * 64) {
      double a0, b0, a1, b1;
      cload(-2, a0, b0);
      cload(-1, a1, b1);
      if (tid < B3CT) {
        rc[2][tid] = a0 - b0;
        rc[3][tid] = a1 - b1;
      }
    }
    __syncthreads();
  }

  if (tid >= B3NW * 64) {
    // ---- the store wave: plane t-4 (written to fin by iteration t-1) ------
    const int l = tid - B3NW * 64;
    double* __restrict__ dse = dst + e * B3HV;
    double* __restrict__ dso = dst + (1 - e) * B3HV;
    double* __restrict__ rsb = L.data + 3 * L.vstride;   // RES: res, the level's own
    double* __restrict__ rse = rsb + e * B3HV;
    double* __restrict__ rso = rsb + (1 - e) * B3HV;
    auto flush = [&](int t) {
      const int z = t - 4;
      if (z < 0 || z >= zend) return;
      int k;
      const int zsb = zbox(z, k), r0 = kB3S * zsb;
      const auto* F = fin[fsl(z)];
      // colour e is the left cell of the pairs of row jr (0-based) at plane z
      auto leftv = [&](int jr) { return ((jr + z + 1) & 1) == e; };
      // PHYS: a physical z face of this box (no push across it; its ghosts,
      // both colours, once the second cell layer in from it is here)
      const bool zlo = PHYS && (fl & 16) && zsb == 1, zhi = PHYS && (fl & 32) && zsb == len;
      // push1 == 0: only the colour-e cells go to the neighbours' ghosts (the
      // caller's next kernel forms the other colour's ghosts itself)
      // the pairs: interior of both colours, and the z faces of the boxes
      // below / above when the plane is a box's first / last layer
#pragma unroll
      for (int r = 0; r < B3NC * B3CP / 64; r++) {
        const int q = l + 64 * r, jr = q / B3CP, pc = q % B3CP;
        const int xs = 1 + pc / B3H, ih = pc % B3H, j = jr + 1;
        const unsigned o = bo[r0 + xs + B3XS] + 8u * (ih + B3H * (j - 1)) + PB * (k - 1);
        const double ve = F[q][0], vo = F[q][1];
        b3_st(dse, o, ve);
        b3_st(dso, o, vo);
        if (RES) {
          b3_st(rse, o, F[q][2]);
          b3_st(rso, o, F[q][3]);
        }
        const bool lf = leftv(jr);
        const double vl = lf ? ve : vo, vr = lf ? vo : ve;
        const int il = 2 * ih + 1;
        if ((k == 1 && !zlo) || (k == B3NC && !zhi)) {
          const int nb = k == 1 ? 6 : 5;
          const unsigned g = bo[r0 + (k == 1 ? -kB3S : kB3S) + xs + B3XS];
          if (push1 || lf) b3_st(dst, g + 8u * b3_gh(nb, il, j), vl);
          if (push1 || !lf) b3_st(dst, g + 8u * b3_gh(nb, il + 1, j), vr);
          if (RES) {
            b3_st(rsb, g + 8u * b3_gh(nb, il, j), lf ? F[q][2] : F[q][3]);
            b3_st(rsb, g + 8u * b3_gh(nb, il + 1, j), lf ? F[q][3] : F[q][2]);
          }
        }
      }
      if (PHYS && ((zlo && k == 2) || (zhi && k == B3NC))) {
        // the ghosts of face 5 (6) from planes 1, 2 (16, 15): this plane and
        // the one before, in which the pair's colours are swapped
        const int f = k == 2 ? 4 : 5;
        const auto* F0 = fin[fsl(z - 1)];
#pragma unroll 1
        for (int r = 0; r < B3NC * B3CP / 64; r++) {
          const int q = l + 64 * r, jr = q / B3CP, pc = q % B3CP;
          const int xs = 1 + pc / B3H, ih = pc % B3H, j = jr + 1, il = 2 * ih + 1;
          const bool lf = leftv(jr);
          const double vl = F[q][lf ? 0 : 1], vr = F[q][lf ? 1 : 0];
          const double pl0 = F0[q][lf ? 1 : 0], pr0 = F0[q][lf ? 0 : 1];
          const double gl = k == 2 ? b3_bc(pk[f], pk[6 + f], pk[12 + f], pl0, vl)
                                   : b3_bc(pk[f], pk[6 + f], pk[12 + f], vl, pl0);
          const double gr = k == 2 ? b3_bc(pk[f], pk[6 + f], pk[12 + f], pr0, vr)
                                   : b3_bc(pk[f], pk[6 + f], pk[12 + f], vr, pr0);
          const unsigned g = bo[r0 + xs + B3XS];
          b3_st(dst, g + 8u * b3_gh(f + 1, il, j), gl);
          b3_st(dst, g + 8u * b3_gh(f + 1, il + 1, j), gr);
        }
      }
      // x faces: per row the cells x = 0, 15, 16, 31 (lane: row l/4, which l%4)
      {
        const int jr = l >> 2, w = l & 3, j = jr + 1;
        const int pc = w == 0 ? 0 : (w == 1 ? B3H - 1 : (w == 2 ? B3H : 2 * B3H - 1));
        const int xs = 1 + pc / B3H;
        const bool lf = leftv(jr), wantl = (w & 1) == 0;   // x = 0, 16: a left cell; 15, 31: right
        const int s = (wantl == lf) ? 0 : 1;
        const double v = fin[fsl(z)][jr * B3CP + pc][s];
        if (PHYS && ((w == 0 && (fl & 1)) || (w == 3 && (fl & 2)))) {
          // x = 0 / 31 next to a physical face: its ghost, from it and x = 1 / 30
          const int f = w == 0 ? 0 : 1;
          const double v2 = fin[fsl(z)][jr * B3CP + pc][1 - s];
          b3_st(dst, bo[r0 + xs + B3XS] + 8u * b3_gh(f + 1, j, k), b3_bc(pk[f], pk[6 + f], pk[12 + f], v, v2));
        } else {
          const int nxs = wantl ? xs - 1 : xs + 1, nb = wantl ? 2 : 1;
          if (push1 || wantl == lf) b3_st(dst, bo[r0 + nxs + B3XS] + 8u * b3_gh(nb, j, k), v);
          if (RES) b3_st(rsb, bo[r0 + nxs + B3XS] + 8u * b3_gh(nb, j, k), fin[fsl(z)][jr * B3CP + pc][2 + s]);
        }
      }
      // y faces: the cells of rows j = 1 (lanes 0..31) and j = 16 (32..63)
      {
        const int jr = l < 32 ? 0 : B3NC - 1, x = l & 31;
        const int pc = x >> 1, xs = 1 + pc / B3H, i = x - B3NC * (xs - 1) + 1;
        const bool lf = leftv(jr), isl = (x & 1) == 0;
        const int s = (isl == lf) ? 0 : 1;
        const double v = fin[fsl(z)][jr * B3CP + pc][s];
        if (PHYS && ((jr == 0 && (fl & 4)) || (jr == B3NC - 1 && (fl & 8)))) {
          // rows 1 / 16 next to a physical face: the ghost from the row and the
          // one behind it (the same x, the other colour)
          const int f = jr == 0 ? 2 : 3, jr2 = jr == 0 ? 1 : B3NC - 2;
          const double v2 = fin[fsl(z)][jr2 * B3CP + pc][1 - s];
          b3_st(dst, bo[r0 + xs + B3XS] + 8u * b3_gh(f + 1, i, k), b3_bc(pk[f], pk[6 + f], pk[12 + f], v, v2));
        } else {
          const int nys = jr == 0 ? 0 : 2, nb = jr == 0 ? 4 : 3;
          if (push1 || isl == lf) b3_st(dst, bo[r0 + xs + B3XS * nys] + 8u * b3_gh(nb, i, k), v);
          if (RES) b3_st(rsb, bo[r0 + xs + B3XS * nys] + 8u * b3_gh(nb, i, k), fin[fsl(z)][jr * B3CP + pc][2 + s]);
        }
      }
    };
    // PRO: res of the column's own coarse cells, plane cs in steps 2cs (rows
    // 0-3) and 2cs+1 (rows 4-7); rc holds it from step 2cs-1 to 2cs+3
    double* __restrict__ cres = C.data + 3 * C.vstride;
    auto cflush = [&](int t) {
      if (t < 0 || t >= zend) return;
      const int cs = t >> 1, q = l + 64 * (t & 1), cxq = q & 15, cyq = q >> 4;
      const double v = rc[cs & 3][(cxq + B3CO) + B3CX * (cyq + B3CO)];
      const int ic = cxq + 1, jc = cyo + cyq + 1, zsc = (cs >> 4) + 1, kc = (cs & 15) + 1;
      const unsigned* cb = cbo + 9 * zsc;
      const unsigned o = 8u * (((ic + jc + kc) & 1) * B3HV + ((ic - 1) >> 1) + B3H * (jc - 1) + B3FH * (kc - 1));
      b3_st(cres, cb[4] + o, v);
      if (ic == 1) b3_st(cres, cb[3] + 8u * b3_gh(2, jc, kc), v);
      if (ic == B3NC) b3_st(cres, cb[5] + 8u * b3_gh(1, jc, kc), v);
      if (jc == 1) b3_st(cres, cb[1] + 8u * b3_gh(4, ic, kc), v);
      if (jc == B3NC) b3_st(cres, cb[7] + 8u * b3_gh(3, ic, kc), v);
      if (kc == 1) b3_st(cres, cb[4 - 9] + 8u * b3_gh(6, ic, jc), v);
      if (kc == B3NC) b3_st(cres, cb[4 + 9] + 8u * b3_gh(5, ic, jc), v);
    };
    for (int t = -3 - kB3Ahead; t <= zend + 3; t += kB3Ahead) {
#pragma unroll
      for (int u = 0; u < kB3Ahead; u++) {
        flush(t + u);
        if (PRO == 1) cflush(t + u);
        __syncthreads();
      }
    }
    return;
  }

  // ---- the compute waves ---------------------------------------------------
  const bool act = tid < B3NT;
  const int p = tid % B3NPX, y = tid / B3NPX - 3;     // (threads past B3NT: a row inside the tile's y+ box)
  const int x0 = 2 * p - 4;
  const int xs = x0 < 0 ? 0 : (x0 < kB3TX * B3NC ? 1 + x0 / B3NC : kB3TX + 1);
  const int ys = y < 0 ? 0 : (y < B3NC ? 1 : 2);
  const int ih = (x0 - B3NC * (xs - 1)) >> 1, j = y - B3NC * (ys - 1) + 1;
  const int slot = xs + B3XS * ys;
  const unsigned xyb = 8u * (ih + B3H * (j - 1));
  const int li = act ? (p + 1) + B3LP * (y + 4) : B3LP + 1;
  const bool ctr = act && xs >= 1 && xs <= kB3TX && ys == 1;
  const int fi = ctr ? (j - 1) * B3CP + (xs - 1) * B3H + ih : 0;
  const double m = shift ? *shift : 0.0;
  const OpCoef<OP> K(L, lambda);
  // colour 1-e of phi; rhs of colour e / 1-e
  const double* __restrict__ src = L.phi + (1 - e) * B3HV;
  const double* __restrict__ rhe = L.data + L.vstride + e * B3HV;
  const double* __restrict__ rho = L.data + L.vstride + (1 - e) * B3HV;
  const double* __restrict__ ole = L.data + 2 * L.vstride + e * B3HV;   // RES: old
  // (only the box columns' old is used: the halo threads all load one cell of
  // the tile's first box, a single line per plane)
  const int slot3 = ctr ? slot : 1 + B3XS;
  const unsigned xyb3 = ctr ? xyb : 0u;
  const double* __restrict__ olo = L.data + 2 * L.vstride + (1 - e) * B3HV;

  // rhs is used where a substep's result is: colour e (substeps 1 and 3) on
  // the pairs within 2 cells of the tile's boxes, colour 1-e (substep 2)
  // within 1; elsewhere the thread loads one shared line of the first box
  // (what its substeps compute there is not used, as for the outermost halo)
  const bool nde = kB3HaloRhs || (act && p >= 1 && p <= B3NPX - 2 && y >= -2 && y <= B3NC + 1);
  const bool ndo = kB3HaloRhs || (nde && y >= -1 && y <= B3NC);
  const int sle = nde ? slot : 1 + B3XS, slo = ndo ? slot : 1 + B3XS;
  const unsigned xye = nde ? xyb : 0u, xyo = ndo ? xyb : 0u;
  // plane t: colour 1-e of phi, both colours of rhs (no branch: the waits
  // for these loads are counted; planes past the end reload the last one);
  // RES: both colours of old at plane t-3 (final kB3Ahead steps later)
  // PHYS: the thread's physical faces; planes -1 and zend across a physical z
  // face load the ghost of face 5 / 6 of the column's first / last box
  B3Face fc{};
  if (PHYS) fc = b3_face(P, fl, p, B3NPX, y, ih, j, e, xyb, PB);
  const unsigned zql = 8u * (2 * B3HV + 4 * B3FS + (1 - e) * B3FH - (1 - e) * B3HV), zqh = zql + 8u * B3FS;
  auto load = [&](int t, double& q, double& fe, double& fo, double& he, double& ho) {
    int k;
    const int zs = zbox(min(t, zend + 2), k);
    const unsigned po = PB * (k - 1);
    if (!PHYS) q = b3_ld(src, bo[kB3S * zs + slot] + xyb + po);
    else if ((fl & 16) && t == -1) q = b3_ld(src, bo[kB3S + slot] + zql + xyb);
    else if ((fl & 32) && t == zend) q = b3_ld(src, bo[kB3S * len + slot] + zqh + xyb);
    else q = b3_ld(src, bo[kB3S * zs + slot] + fc.xyq + fc.kq * (k - 1));
    fe = b3_ld(rhe, bo[kB3S * zs + sle] + xye + po);
    fo = b3_ld(rho, bo[kB3S * zs + slo] + xyo + po);
    if (RES) {
      int k3;
      const int zs3 = zbox(min(t - 3, zend + 2), k3);
      const unsigned o3 = bo[kB3S * zs3 + slot3] + xyb3 + PB * (k3 - 1);
      he = b3_ld(ole, o3);
      ho = b3_ld(olo, o3);
    }
  };

  // V0: colour 1-e as loaded, planes t-2, t-1; V1: colour e after substep 1,
  // planes t-3, t-2; V2: colour 1-e after substep 2, planes t-4, t-3; rhs of
  // colour e at planes t-1, t-2, t-3 and of colour 1-e at t-1, t-2
  double oa = 0.0, ob = 0.0, ea = 0.0, eb = 0.0, wa = 0.0, wb = 0.0;
  double re1 = 0.0, re2 = 0.0, re3 = 0.0, ro1 = 0.0, ro2 = 0.0;
  // PRO: this thread's coarse cell (the parent of its pair) in the tile
  // (p - 2 is the pair's cx; the outer cells of pairs 0 and B3NPX-1 tap one
  // entry past the tile's edge, in the ring's bounds: their values are unused)
  const int ci = act ? (p - 2 + B3CO) + B3CX * ((y >> 1) + B3CO) : B3CX + 1;
  // cl (PRO): an even plane's step, which takes coarse plane t/2+1 to the
  // ring and loads plane (t+kB3Ahead)/2+1
  auto step = [&](int t, double& q, double& fe, double& fo, double& he, double& ho, double& ca, double& cb,
                  bool cl) {
    double ot = shift ? b3_take(q) - m : b3_take(q);
    const double ret = b3_take(fe), rot = b3_take(fo);
    double cr = 0.0, hte = 0.0, hto = 0.0;
    if (PRO == 1 && cl) cr = b3_take(ca) - b3_take(cb);
    if (PRO == 2 && cl) cr = b3_take(ca);
    if (RES) {
      hte = b3_take(he);
      hto = b3_take(ho);
    }
    load(t + kB3Ahead, q, fe, fo, he, ho);
    if (PRO && cl) cload(min((t + kB3Ahead) / 2 + 1, B3NC * lenc + 2), ca, cb);
    if (PRO) {
      // phi += prolong(phi - old) on the colour-(1-e) cell (prolong_at): the
      // parent, its x tap on the cell's side, its y / z taps by the parity of
      // the cell's row / plane (the column starts at even x, y and z)
      const int cz0 = t >> 1;
      const double* R0 = rc[cz0 & 3];
      const double* Rz = rc[((t & 1) ? cz0 + 1 : cz0 - 1) & 3];
      const bool lft = ((y + t) & 1) == e;
      const double f0 = 0.25 * R0[ci];
      const double fx = 0.25 * R0[lft ? ci - 1 : ci + 1];
      const double fy = 0.25 * R0[(y & 1) ? ci + B3CX : ci - B3CX];
      const double fz = 0.25 * Rz[ci];
      ot = ot + (f0 + fx + fy + fz);
      if (cl) {
        const int c = t / 2 + 1;
        if (c >= 0 && tid < B3CT) rc[c & 3][tid] = cr;
      }
    }
    const double* P0 = pl[t & 1][0];
    const double* P1 = pl[t & 1][1];
    const double* P2 = pl[t & 1][2];
    // the active cells are the pair's left ones (x0) when colour e is there
    // at plane t-1; the neighbour pair across is on that side
    const bool lft = ((y + t) & 1) == e;
    const int far = lft ? li - 1 : li + 1;
    Nbr7 n;
    n.c = 0.0;
    // substep 1 (colour e) at plane t-1
    n.xm = P0[far]; n.xp = ob;
    n.ym = P0[li - B3LP]; n.yp = P0[li + B3LP]; n.zm = oa; n.zp = ot;
    const double s1 = gs_value<OP>(K, n, re1);
    // substep 2 (colour 1-e) at plane t-2 (PHYS: the ghosts across physical
    // faces from the cell's value before it, stage 0's, as in k_gsrb4)
    n.xm = P1[far]; n.xp = eb;
    n.ym = P1[li - B3LP]; n.yp = P1[li + B3LP]; n.zm = ea; n.zp = s1;
    if (PHYS) b3_fix(n, fc, P, fl, lft, oa, t - 2, zend);
    const double s2 = gs_value<OP>(K, n, ro2);
    // substep 3 (colour e) at plane t-3
    n.xm = P2[far]; n.xp = wb;
    n.ym = P2[li - B3LP]; n.yp = P2[li + B3LP]; n.zm = wa; n.zp = s2;
    if (PHYS) b3_fix(n, fc, P, fl, lft, ea, t - 3, zend);
    const double s3 = gs_value<OP>(K, n, re3);
    // plane t-3 is final (colour e = s3, colour 1-e = wb): to the store wave
    if (ctr) {
      double* F = fin[fsl(t - 3)][fi];
      F[0] = s3;
      F[1] = wb;
      if (RES) {
        F[2] = s3 - hte;
        F[3] = wb - hto;
      }
    }
    if (act) {
      double* W = pl[(t + 1) & 1][0];
      W[li] = ot;
      W[B3PL + li] = s1;
      W[2 * B3PL + li] = s2;
    }
    __syncthreads();
    oa = ob; ob = ot;
    ea = eb; eb = s1;
    wa = wb; wb = s2;
    re3 = re2; re2 = re1; re1 = ret;
    ro2 = ro1; ro1 = rot;
  };
  // kB3Ahead planes in flight.  The loop issues every load, planes -3 .. in
  // kB3Ahead extra leading steps that compute nothing used: loads issued
  // before the loop land in other registers than the loop's, and its first
  // wait would drain them all.  Trailing steps past the column compute
  // nothing used either (their loads reload the last plane); the store wave
  // writes plane zend-1 in iteration zend+3.
  double qs[kB3Ahead], fes[kB3Ahead], fos[kB3Ahead], hes[kB3Ahead], hos[kB3Ahead];
  double cas[kB3Ahead / 2], cbs[kB3Ahead / 2];
#pragma unroll
  for (int u = 0; u < kB3Ahead; u++) qs[u] = fes[u] = fos[u] = hes[u] = hos[u] = 0.0;
#pragma unroll
  for (int u = 0; u < kB3Ahead / 2; u++) cas[u] = cbs[u] = 0.0;
  // (t + u is even for odd u: t starts at -3 - kB3Ahead, odd)
  for (int t = -3 - kB3Ahead; t <= zend + 3; t += kB3Ahead) {
#pragma unroll
    for (int u = 0; u < kB3Ahead; u++)
      step(t + u, qs[u], fes[u], fos[u], hes[u], hos[u], cas[u >> 1], cbs[u >> 1], (u & 1) == 1);
  }
}

// Four red-black substeps (colours e, 1-e, e, 1-e) in one pass (k_gsrb4): the
// plain form of k_gsrb3 with a fourth stage at plane t-4 and a 4-row y halo
// (rows -4 .. 19; the x tile already reaches 4 cells), for the down-smoothing
// of a level whose residual + restriction then runs as k_resid_restrict (the
// alternative to k_gsrb3 + k_smooth_resid, the default; OMG_NO_BLOCK4).  Every
// ghost face of both colours is pushed.
// PRO 2 (round 6): the up-smoothing's correct_children form with all four
// substeps (k_gsrb3's PRO 2 reaches three, the fourth was a one-substep
// launch): the colour 1-e it reads gets the prolonged correction from the
// coarse res the coarse level's last pass stored, as in k_gsrb3.  The cells
// used now reach 4 from the boxes (stage 1 at distance 3 reads them), so the
// coarse tile has a 3-cell rim (cx in [-3, 18], cy in [-3, 10]) and the ring
// starts at coarse plane -3.  The compute waves of k_gsrb4 are at 94 VGPRs,
// two workgroups per CU allow 96, so in this form a wave of its own loads the
// coarse planes into the ring (a wave's VGPR count is the most its own path
// needs: 10 waves, two workgroups per CU at 5 waves per SIMD), and the
// compute waves keep 2 planes of loads in flight instead of 4, which makes
// room for the correction: 86 VGPRs.  On C3's level 1 it takes 881 us
// against 819 + 307 for k_gsrb3's form and the last substep
// (profiles/r06/s5_block4p_ab.txt; 4 ahead with rhs of colour 1-e in an LDS
// ring and 2 VGPRs spilled took 1027 us, the correction formed by the loader
// wave alone 1451 us: one wave's issue share of its SIMD).
constexpr int B4NY = B3NC + 8, B4NT = B3NPX * B4NY, B4NW = (B4NT + 63) / 64, B4BS = 64 * (B4NW + 1);
constexpr int B4PL = B3LP * (B4NY + 2);
constexpr int B4CO = 3;
constexpr int B4CX = kB3TX * B3H + 2 * B4CO, B4CY = B3H + 2 * B4CO, B4CT = B4CX * B4CY;
constexpr int B4CL = (B4CT + 63) / 64;   // coarse cells per lane of the loader wave
constexpr int b4_threads(int pro) { return pro ? B4BS + 64 : B4BS; }

template <int OP, int PRO, bool PHYS>
__global__ void __launch_bounds__(b4_threads(PRO)) k_gsrb4(LevelView L, double* __restrict__ dst,
                                               const int* __restrict__ cols, double lambda, int e,
                                               const double* __restrict__ shift, LevelView C,
                                               const int* __restrict__ ccols, double fac, B3Phys P, int push) {
  static_assert(PRO == 0 || PRO == 2, "k_gsrb4: plain or the correction from a stored coarse res");
  static_assert(!(PRO && PHYS), "k_gsrb4: physical faces in the plain form only");
  __shared__ double pl[2][4][B4PL];
  // final plane: [row * B3CP + pair][colour e, 1-e] (PHYS: a ring of three, the
  // z ghosts read the plane before)
  __shared__ double fin[PHYS ? 3 : 2][B3NC * B3CP][2];
  auto fsl = [](int z) { return PHYS ? (z + 12) % 3 : z & 1; };
  __shared__ unsigned bo[kB3Rec];
  __shared__ double rc[PRO ? 4 : 1][PRO ? B4CT : 1];   // coarse res, plane c in rc[c & 3]
  __shared__ unsigned cbo[PRO ? kB3CSlots : 1];        // the coarse record, byte offsets
  __shared__ int len_s, cyo_s, fl_s;
  __shared__ double pk[PHYS ? 18 : 1];
  const int tid = threadIdx.x;
  const int cq = xcd_box(blockIdx.x, gridDim.x);
  constexpr int BS = b4_threads(PRO);
  if (PHYS && tid >= BS - 18) pk[tid - (BS - 18)] = (&P.k[0])[tid - (BS - 18)];
  // planes of loads in flight: the correction form 2 (its registers)
  constexpr int AH = PRO ? 2 : kB3Ahead;
  // steps of every wave's loop: planes -4-AH .. zend+4 in blocks of AH
  const int t0 = -4 - AH;
  for (int q = tid; q < kB3Rec; q += BS) {
    const int v = cols[(long long)cq * kB3Rec + q];
    if (q == 0) {
      len_s = v & kB3LenMask;
      fl_s = v >> 8;
    } else {
      bo[q - 1] = (unsigned)v * (unsigned)(L.stride * 8);
    }
  }
  if (PRO) {
    for (int q = tid; q < 1 + kB3CSlots; q += BS) {
      const int v = ccols[(long long)cq * kB3CRec + q];
      if (q == 0) cyo_s = v;
      else cbo[q - 1] = (unsigned)v * (unsigned)(C.stride * 8);
    }
    for (int q2 = tid; q2 < 4 * B4CT; q2 += BS) (&rc[0][0])[q2] = 0.0;
  }
  for (int q = tid; q < 2 * 4 * B4PL; q += BS) (&pl[0][0][0])[q] = 0.0;
  __syncthreads();
  const int len = len_s, zend = B3NC * len;
  const int fl = PHYS ? fl_s : 0;
  constexpr unsigned PB = 8u * B3H * B3NC;
  auto zbox = [&](int t, int& k) {
    const int zs = t < 0 ? 0 : (t >= zend ? len + 1 : (t >> 4) + 1);
    k = t - B3NC * (zs - 1) + 1;
    return zs;
  };
  if (PRO && tid >= B4BS) {
    // ---- the coarse loader wave: at the even step t it writes coarse plane
    // t/2+1 to the ring (loaded 4 steps before) and loads plane t/2+3, the
    // cells of the tile, B4CL per lane.  The compute threads read plane p at
    // steps 2p-1 .. 2p+2 (the parent of planes 2p, 2p+1, the z tap of 2p-1
    // and 2p+2); it is written at step 2p-2 and its slot next at 2p+6.
    const int l = tid - B4BS, cyo = cyo_s, lenc = len >> 1;
    const double* __restrict__ cres_in = C.data + 3 * C.vstride;
    auto cload = [&](int c, double* v) {
      const int zsc = c < 0 ? 0 : (c >= B3NC * lenc ? lenc + 1 : (c >> 4) + 1);
      const int kc = c - B3NC * (zsc - 1) + 1;
#pragma unroll
      for (int r = 0; r < B4CL; r++) {
        const int ct = min(l + 64 * r, B4CT - 1);
        const int cxr = ct % B4CX - B4CO, cyy = cyo + ct / B4CX - B4CO;
        const int xsc = cxr < 0 ? 0 : (cxr < B3NC ? 1 : 2), ysc = cyy < 0 ? 0 : (cyy < B3NC ? 1 : 2);
        const int icc = cxr - B3NC * (xsc - 1) + 1, jcc = cyy - B3NC * (ysc - 1) + 1;
        v[r] = b3_ld(cres_in, cbo[9 * zsc + 3 * ysc + xsc] + 8u * B3HV * ((icc + jcc + kc) & 1) +
                                  8u * (((icc - 1) >> 1) + B3H * (jcc - 1)) + PB * (kc - 1));
      }
    };
    double va[B4CL], vb[B4CL];
    const int cmax = B3NC * lenc + 2;
    auto cput = [&](int c, double* v) {
#pragma unroll
      for (int r = 0; r < B4CL; r++)
        if (l + 64 * r < B4CT) rc[c & 3][l + 64 * r] = b3_take(v[r]);
    };
    auto cstep = [&](int t, double* v) {
      const int c = t / 2 + 1;
      cput(c, v);
      cload(min(c + 2, cmax), v);
    };
    // the first step is t0 = -6 (even): planes -2 and -1 come from the loop,
    // plane -3 (read from step -4 on) is written before it
    static_assert(!PRO || AH == 2, "the loader's steps start at plane -6");
    cload(-3, va);
    cput(-3, va);
    cload(-2, va);
    cload(-1, vb);
    // (the steps of the compute loop: AH * ceil((zend + 5 - t0) / AH), a multiple of 4)
    const int n_steps = AH * ((zend + 5 - t0 + AH - 1) / AH);
    for (int t = t0; t < t0 + n_steps; t += 4) {
      cstep(t, va);
      __syncthreads();
      __syncthreads();
      cstep(t + 2, vb);
      __syncthreads();
      __syncthreads();
    }
    return;
  }

  if (tid >= B4NW * 64) {
    // ---- the store wave: plane t-5 (written to fin by iteration t-1) ------
    const int l = tid - B4NW * 64;
    double* __restrict__ dse = dst + e * B3HV;
    double* __restrict__ dso = dst + (1 - e) * B3HV;
    auto flush = [&](int t) {
      const int z = t - 5;
      if (z < 0 || z >= zend) return;
      int k;
      const int zsb = zbox(z, k), r0 = kB3S * zsb;
      const auto* F = fin[fsl(z)];
      auto leftv = [&](int jr) { return ((jr + z + 1) & 1) == e; };
      // PHYS: a physical z face of this box (no push across it; its ghosts
      // once the second cell layer in from it is here)
      const bool zlo = PHYS && (fl & 16) && zsb == 1, zhi = PHYS && (fl & 32) && zsb == len;
      // (a lane stores pairs q, q+1 of a row, ih even: 16-B stores, of each
      // colour and, on a box's first / last plane, of each parity half of the
      // z face's ghosts next door; 8-B stores per pair were the round-5 form)
#pragma unroll
      for (int r = 0; r < B3NC * B3CP / 128; r++) {
        const int q = 2 * (l + 64 * r), jr = q / B3CP, pc = q % B3CP;
        const int xs = 1 + pc / B3H, ih = pc % B3H, j = jr + 1;
        const unsigned o = bo[r0 + xs + B3XS] + 8u * (ih + B3H * (j - 1)) + PB * (k - 1);
        const v2d ve = {F[q][0], F[q + 1][0]}, vo = {F[q][1], F[q + 1][1]};
        b3_st2(dse, o, ve);
        b3_st2(dso, o, vo);
        if (push && ((k == 1 && !zlo) || (k == B3NC && !zhi))) {
          const bool lf = leftv(jr);
          const int il = 2 * ih + 1, nb = k == 1 ? 6 : 5;
          const unsigned g = bo[r0 + (k == 1 ? -kB3S : kB3S) + xs + B3XS];
          b3_st2(dst, g + 8u * b3_gh(nb, il, j), lf ? ve : vo);
          b3_st2(dst, g + 8u * b3_gh(nb, il + 1, j), lf ? vo : ve);
        }
      }
      if (PHYS && ((zlo && k == 2) || (zhi && k == B3NC))) {
        // the ghosts of face 5 (6) from planes 1, 2 (16, 15): this plane and
        // the one before, in which the pair's colours are swapped
        const int f = k == 2 ? 4 : 5;
        const auto* F0 = fin[fsl(z - 1)];
#pragma unroll 1
        for (int r = 0; r < B3NC * B3CP / 64; r++) {
          const int q = l + 64 * r, jr = q / B3CP, pc = q % B3CP;
          const int xs = 1 + pc / B3H, ih = pc % B3H, j = jr + 1, il = 2 * ih + 1;
          const bool lf = leftv(jr);
          const double vl = F[q][lf ? 0 : 1], vr = F[q][lf ? 1 : 0];
          const double pl0 = F0[q][lf ? 1 : 0], pr0 = F0[q][lf ? 0 : 1];
          const double gl = k == 2 ? b3_bc(pk[f], pk[6 + f], pk[12 + f], pl0, vl)
                                   : b3_bc(pk[f], pk[6 + f], pk[12 + f], vl, pl0);
          const double gr = k == 2 ? b3_bc(pk[f], pk[6 + f], pk[12 + f], pr0, vr)
                                   : b3_bc(pk[f], pk[6 + f], pk[12 + f], vr, pr0);
          const unsigned g = bo[r0 + xs + B3XS];
          b3_st(dst, g + 8u * b3_gh(f + 1, il, j), gl);
          b3_st(dst, g + 8u * b3_gh(f + 1, il + 1, j), gr);
        }
      }
      // push 0: the interior only (the cycle's last pass on a level whose next
      // reader is a pass that reads no ghosts; correct_block3's defer_gc)
      if (!push) return;
      {
        const int jr = l >> 2, w = l & 3, j = jr + 1;
        const int pc = w == 0 ? 0 : (w == 1 ? B3H - 1 : (w == 2 ? B3H : 2 * B3H - 1));
        const int xs = 1 + pc / B3H;
        const bool lf = leftv(jr), wantl = (w & 1) == 0;
        const int s = (wantl == lf) ? 0 : 1;
        const double v = fin[fsl(z)][jr * B3CP + pc][s];
        if (PHYS && ((w == 0 && (fl & 1)) || (w == 3 && (fl & 2)))) {
          // x = 0 / 31 next to a physical face: its ghost, from it and x = 1 / 30
          const int f = w == 0 ? 0 : 1;
          const double v2 = fin[fsl(z)][jr * B3CP + pc][1 - s];
          b3_st(dst, bo[r0 + xs + B3XS] + 8u * b3_gh(f + 1, j, k), b3_bc(pk[f], pk[6 + f], pk[12 + f], v, v2));
        } else {
          const int nxs = wantl ? xs - 1 : xs + 1, nb = wantl ? 2 : 1;
          b3_st(dst, bo[r0 + nxs + B3XS] + 8u * b3_gh(nb, j, k), v);
        }
      }
      {
        const int jr = l < 32 ? 0 : B3NC - 1, x = l & 31;
        const int pc = x >> 1, xs = 1 + pc / B3H, i = x - B3NC * (xs - 1) + 1;
        const bool lf = leftv(jr), isl = (x & 1) == 0;
        const int s = (isl == lf) ? 0 : 1;
        const double v = fin[fsl(z)][jr * B3CP + pc][s];
        if (PHYS && ((jr == 0 && (fl & 4)) || (jr == B3NC - 1 && (fl & 8)))) {
          // rows 1 / 16 next to a physical face: the ghost from the row and the
          // one behind it (the same x, the other colour)
          const int f = jr == 0 ? 2 : 3, jr2 = jr == 0 ? 1 : B3NC - 2;
          const double v2 = fin[fsl(z)][jr2 * B3CP + pc][1 - s];
          b3_st(dst, bo[r0 + xs + B3XS] + 8u * b3_gh(f + 1, i, k), b3_bc(pk[f], pk[6 + f], pk[12 + f], v, v2));
        } else {
          const int nys = jr == 0 ? 0 : 2, nb = jr == 0 ? 4 : 3;
          b3_st(dst, bo[r0 + xs + B3XS * nys] + 8u * b3_gh(nb, i, k), v);
        }
      }
    };
    for (int t = t0; t <= zend + 4; t += AH) {
#pragma unroll
      for (int u = 0; u < AH; u++) {
        flush(t + u);
        __syncthreads();
      }
    }
    return;
  }

  // ---- the compute waves ---------------------------------------------------
  const bool act = tid < B4NT;
  const int p = tid % B3NPX, y = tid / B3NPX - 4;
  const int x0 = 2 * p - 4;
  const int xs = x0 < 0 ? 0 : (x0 < kB3TX * B3NC ? 1 + x0 / B3NC : kB3TX + 1);
  const int ys = y < 0 ? 0 : (y < B3NC ? 1 : 2);
  const int ih = (x0 - B3NC * (xs - 1)) >> 1, j = y - B3NC * (ys - 1) + 1;
  const int slot = xs + B3XS * ys;
  const unsigned xyb = 8u * (ih + B3H * (j - 1));
  const int li = act ? (p + 1) + B3LP * (y + 5) : B3LP + 1;
  const bool ctr = act && xs >= 1 && xs <= kB3TX && ys == 1;
  const int fi = ctr ? (j - 1) * B3CP + (xs - 1) * B3H + ih : 0;
  const double m = (!PRO && shift) ? *shift : 0.0;
  // fac from the host (op_fac: the same expression, so the same bits): the
  // division on the device would hold it in VGPRs
  OpCoef<OP> K(L, lambda);
  K.fac = fac;
  const double* __restrict__ src = L.phi + (1 - e) * B3HV;
  const double* __restrict__ rhe = L.data + L.vstride + e * B3HV;
  const double* __restrict__ rho = L.data + L.vstride + (1 - e) * B3HV;
  // rhs where a substep's result is used: colour e (substeps 1, 3) within 3
  // cells of the boxes, colour 1-e (substeps 2, 4) within 2
  const bool nde = act && y >= -3 && y <= B3NC + 2;
  const bool ndo = act && p >= 1 && p <= B3NPX - 2 && y >= -2 && y <= B3NC + 1;
  const int sle = nde ? slot : 1 + B3XS, slo = ndo ? slot : 1 + B3XS;
  const unsigned xye = nde ? xyb : 0u, xyo = ndo ? xyb : 0u;
  // PHYS: the thread's physical faces; planes -1 and zend across a physical z
  // face load the ghost of face 5 / 6 of the column's first / last box
  B3Face fc{};
  if (PHYS) fc = b3_face(P, fl, p, B3NPX, y, ih, j, e, xyb, PB);
  const unsigned zql = 8u * (2 * B3HV + 4 * B3FS + (1 - e) * B3FH - (1 - e) * B3HV), zqh = zql + 8u * B3FS;
  auto load = [&](int t, double& q, double& fe, double& fo) {
    int k;
    const int zs = zbox(min(t, zend + 3), k);
    const unsigned po = PB * (k - 1);
    if (!PHYS) q = b3_ld(src, bo[kB3S * zs + slot] + xyb + po);
    else if ((fl & 16) && t == -1) q = b3_ld(src, bo[kB3S + slot] + zql + xyb);
    else if ((fl & 32) && t == zend) q = b3_ld(src, bo[kB3S * len + slot] + zqh + xyb);
    else q = b3_ld(src, bo[kB3S * zs + slot] + fc.xyq + fc.kq * (k - 1));
    fe = b3_ld(rhe, bo[kB3S * zs + sle] + xye + po);
    fo = b3_ld(rho, bo[kB3S * zs + slo] + xyo + po);
  };
  // V0 stage 0 (planes t-2, t-1), V1 stage 1 (t-3, t-2), V2 stage 2 (t-4,
  // t-3), V3 stage 3 (t-5, t-4); rhs colour e at t-1 .. t-3, 1-e at t-1 .. t-4
  double oa = 0.0, ob = 0.0, ea = 0.0, eb = 0.0, wa = 0.0, wb = 0.0, xa = 0.0, xb = 0.0;
  double re1 = 0.0, re2 = 0.0, re3 = 0.0, ro1 = 0.0, ro2 = 0.0, ro3 = 0.0, ro4 = 0.0;
  // PRO: this thread's coarse cell (the parent of its pair) in the tile
  const int ci = act ? (p - 2 + B4CO) + B4CX * ((y >> 1) + B4CO) : B4CX + 1;
  auto step = [&](int t, double& q, double& fe, double& fo) {
    double ot = (!PRO && shift) ? b3_take(q) - m : b3_take(q);
    const double ret = b3_take(fe), rot = b3_take(fo);
    load(t + AH, q, fe, fo);
    if (PRO) {
      // phi += prolong(res) on the colour-(1-e) cell (prolong_at, as k_gsrb3)
      const int cz0 = t >> 1;
      const double* R0 = rc[cz0 & 3];
      const double* Rz = rc[((t & 1) ? cz0 + 1 : cz0 - 1) & 3];
      const bool lft = ((y + t) & 1) == e;
      const double f0 = 0.25 * R0[ci];
      const double fx = 0.25 * R0[lft ? ci - 1 : ci + 1];
      const double fy = 0.25 * R0[(y & 1) ? ci + B4CX : ci - B4CX];
      const double fz = 0.25 * Rz[ci];
      ot = ot + (f0 + fx + fy + fz);
    }
    const double* P0 = pl[t & 1][0];
    const double* P1 = pl[t & 1][1];
    const double* P2 = pl[t & 1][2];
    const double* P3 = pl[t & 1][3];
    const bool lft = ((y + t) & 1) == e;
    const int far = lft ? li - 1 : li + 1;
    Nbr7 n;
    n.c = 0.0;
    n.xm = P0[far]; n.xp = ob;
    n.ym = P0[li - B3LP]; n.yp = P0[li + B3LP]; n.zm = oa; n.zp = ot;
    const double s1 = gs_value<OP>(K, n, re1);
    // (PHYS: substeps 2-4 form the ghosts across physical faces; the cell's
    // value before substep s is stage s-2's)
    n.xm = P1[far]; n.xp = eb;
    n.ym = P1[li - B3LP]; n.yp = P1[li + B3LP]; n.zm = ea; n.zp = s1;
    if (PHYS) b3_fix(n, fc, P, fl, lft, oa, t - 2, zend);
    const double s2 = gs_value<OP>(K, n, ro2);
    n.xm = P2[far]; n.xp = wb;
    n.ym = P2[li - B3LP]; n.yp = P2[li + B3LP]; n.zm = wa; n.zp = s2;
    if (PHYS) b3_fix(n, fc, P, fl, lft, ea, t - 3, zend);
    const double s3 = gs_value<OP>(K, n, re3);
    n.xm = P3[far]; n.xp = xb;
    n.ym = P3[li - B3LP]; n.yp = P3[li + B3LP]; n.zm = xa; n.zp = s3;
    if (PHYS) b3_fix(n, fc, P, fl, lft, wa, t - 4, zend);
    const double s4 = gs_value<OP>(K, n, ro4);
    // plane t-4 is final (colour e = stage 3 of the last iteration, 1-e = s4)
    if (ctr) {
      double* F = fin[fsl(t - 4)][fi];
      F[0] = xb;
      F[1] = s4;
    }
    if (act) {
      double* W = pl[(t + 1) & 1][0];
      W[li] = ot;
      W[B4PL + li] = s1;
      W[2 * B4PL + li] = s2;
      W[3 * B4PL + li] = s3;
    }
    __syncthreads();
    oa = ob; ob = ot;
    ea = eb; eb = s1;
    wa = wb; wb = s2;
    xa = xb; xb = s3;
    re3 = re2; re2 = re1; re1 = ret;
    ro4 = ro3; ro3 = ro2; ro2 = ro1; ro1 = rot;
  };
  double qs[AH], fes[AH], fos[AH];
#pragma unroll
  for (int u = 0; u < AH; u++) qs[u] = fes[u] = fos[u] = 0.0;
  for (int t = t0; t <= zend + 4; t += AH) {
#pragma unroll
    for (int u = 0; u < AH; u++) step(t + u, qs[u], fes[u], fos[u]);
  }
}

// OpCoef's fac on the host: box_gs_lpl's 0.5/sum(idr2) (m_laplacian.f90:64-65),
// box_gs_helmh's 1/(2*sum(idr2)+lambda) (m_helmholtz.f90:58-59), the same
// operations in the same order as the device's (IEEE division both sides)
static double op_fac(const LevelView& L, int op, double lambda) {
  const double ix = L.idr2[0], iy = L.idr2[1], iz = L.idr2[2];
  return op == OP_HELM ? 1.0 / (2 * ((ix + iy) + iz) + lambda) : 0.5 / ((ix + iy) + iz);
}

void launch_gsrb4(const LevelView& L, double* dst, const int* cols, int n_cols, int op, double lambda, int e,
                  const double* shift, hipStream_t st, const LevelView* coarse, const int* ccols,
                  const B3Phys* phys, bool push) {
  const double fac = op_fac(L, op, lambda);
  if (n_cols <= 0) return;
  if (L.nc != B3NC) throw std::runtime_error("launch_gsrb4: box size must be 16");
  if (coarse && (coarse->nc != B3NC || !ccols || shift))
    throw std::runtime_error("launch_gsrb4: the correction form needs a 16^3 coarse level, its records, no shift");
  if (phys && (coarse || shift))
    throw std::runtime_error("launch_gsrb4: physical faces in the plain form without a shift only");
  if (!push && phys) throw std::runtime_error("launch_gsrb4: physical faces need their ghosts written");
  const LevelView& C = coarse ? *coarse : L;
  const B3Phys P = phys ? *phys : B3Phys{};
#define OMG_B4(OPV, PMV, PHV, BS) \
  k_gsrb4<OPV, PMV, PHV><<<n_cols, BS, 0, st>>>(L, dst, cols, lambda, e, shift, C, ccols, fac, P, push ? 1 : 0)
  if (op == OP_HELM) {
    if (coarse) OMG_B4(OP_HELM, 2, false, b4_threads(2));
    else if (phys) OMG_B4(OP_HELM, 0, true, B4BS);
    else OMG_B4(OP_HELM, 0, false, B4BS);
  } else {
    if (coarse) OMG_B4(OP_LPL, 2, false, b4_threads(2));
    else if (phys) OMG_B4(OP_LPL, 0, true, B4BS);
    else OMG_B4(OP_LPL, 0, false, B4BS);
  }
#undef OMG_B4
}

bool gsrb3_op_ok(int op) { return op == OP_LPL || op == OP_HELM; }

void launch_gsrb3(const LevelView& L, double* dst, const int* cols, int n_cols, int op, double lambda, int e,
                  const double* shift, hipStream_t st, bool push1, const LevelView* coarse, const int* ccols,
                  int coarse_mode, bool res, const B3Phys* phys) {
  if (n_cols <= 0) return;
  if (L.nc != B3NC) throw std::runtime_error("launch_gsrb3: box size must be 16");
  const int p1 = push1 ? 1 : 0;
  const int pm = coarse ? coarse_mode : 0;
  if (coarse && (coarse->nc != B3NC || !ccols || shift || (pm != 1 && pm != 2)))
    throw std::runtime_error("launch_gsrb3: the correction form needs a 16^3 coarse level, its records, no shift");
  if (res && (pm || !push1))
    throw std::runtime_error("launch_gsrb3: res = phi - old only on a plain pass that pushes both colours");
  if (phys && (pm || res || shift))
    throw std::runtime_error("launch_gsrb3: physical faces in the plain form without a shift only");
  const LevelView& C = coarse ? *coarse : L;
  const B3Phys P = phys ? *phys : B3Phys{};
#define OMG_B3(OPV, PMV, RV, PHV) \
  k_gsrb3<OPV, PMV, RV, PHV><<<n_cols, B3BS, 0, st>>>(L, dst, cols, lambda, e, shift, p1, C, ccols, P)
  const bool helm = op == OP_HELM;
  if (pm == 1) {
    if (helm) OMG_B3(OP_HELM, 1, false, false); else OMG_B3(OP_LPL, 1, false, false);
  } else if (pm == 2) {
    if (helm) OMG_B3(OP_HELM, 2, false, false); else OMG_B3(OP_LPL, 2, false, false);
  } else if (res) {
    if (helm) OMG_B3(OP_HELM, 0, true, false); else OMG_B3(OP_LPL, 0, true, false);
  } else if (phys) {
    if (helm) OMG_B3(OP_HELM, 0, false, true); else OMG_B3(OP_LPL, 0, false, true);
  } else {
    if (helm) OMG_B3(OP_HELM, 0, false, false); else OMG_B3(OP_LPL, 0, false, false);
  }
#undef OMG_B3
}

}  // namespace omg
