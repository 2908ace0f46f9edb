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
// by the box that owns the cell.  Levels whose faces are all same-GPU boxes,
// 16^3 boxes, Laplacian / Helmholtz, with consistent ghosts on entry (they
// are not read: a neighbour's cells are read in its box).
#include <stdexcept>

#ifndef B3_AHEAD
#define B3_AHEAD 4
#endif
#ifndef B3_WAVES
#define B3_WAVES 1
#endif
#ifndef B4_AHEAD
#define B4_AHEAD 2
#endif
#ifndef B4_STAGE_FENCE
#define B4_STAGE_FENCE __builtin_amdgcn_sched_barrier(0)
#endif
#ifndef B4_WAVES
#define B4_WAVES 1
#endif

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
constexpr int kB3Ahead = B3_AHEAD;               // planes of loads in flight

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

// A store the compiler does not count: its s_waitcnt bookkeeping treats
// vmcnt as out of order once stores and loads are both pending and then waits
// for vmcnt(0) at every load use, which would drain the loads in flight two
// planes ahead.  Loads return in order among themselves, so the counted waits
// it computes from the loads alone stay correct with these stores pending
// (they only make the hardware wait longer); nothing in the kernel reads what
// they write.  base: wave-uniform, off: bytes (< 4 GiB).
__device__ __forceinline__ void b3_st(double* base, unsigned off, double v) {
  asm volatile("global_store_dwordx2 %0, %1, %2\n\ts_nop 1" : : "v"(off), "v"(v), "s"(base));
}
__device__ __forceinline__ double b3_ld(const double* base, unsigned off) {
  return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + off);
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
template <int OP>
__global__ void __launch_bounds__(B3BS, B3_WAVES) k_gsrb3(LevelView L, double* __restrict__ dst,
                                                          const int* __restrict__ cols, double lambda, int e,
                                                          const double* __restrict__ shift) {
  __shared__ double pl[2][3][B3PL];
  __shared__ double fin[2][B3NC * B3CP][2];   // final plane: [row * B3CP + pair][colour e, 1-e]
  __shared__ unsigned bo[kB3Rec];             // the record's boxes as byte offsets into a variable
  __shared__ int len_s;
  const int tid = threadIdx.x;
  const int cq = xcd_box(blockIdx.x, gridDim.x);
  if (tid < kB3Rec) {
    const int v = cols[(long long)cq * kB3Rec + tid];
    if (tid == 0) len_s = v;
    else bo[tid - 1] = (unsigned)v * (unsigned)(L.stride * 8);
  }
  for (int q = tid; q < 2 * 3 * B3PL; q += B3BS) (&pl[0][0][0])[q] = 0.0;
  __syncthreads();
  const int len = len_s, zend = B3NC * len;
  constexpr unsigned PB = 8u * B3H * B3NC;   // bytes per plane of one colour
  auto zbox = [&](int t, int& k) {
    const int zs = t < 0 ? 0 : (t >= zend ? len + 1 : (t >> 4) + 1);
    k = t - B3NC * (zs - 1) + 1;
    return zs;
  };

  if (tid >= B3NW * 64) {
    // ---- the store wave: plane t-4 (written to fin by iteration t-1) ------
    const int l = tid - B3NW * 64;
    double* __restrict__ dse = dst + e * B3HV;
    double* __restrict__ dso = dst + (1 - e) * B3HV;
    auto flush = [&](int t) {
      const int z = t - 4;
      if (z < 0 || z >= zend) return;
      int k;
      const int r0 = kB3S * zbox(z, k);
      const double(*F)[2] = fin[z & 1];
      // colour e is on the left of the pairs of row j at plane z when
      // (j - 1 + z) is even... (the compute side's test at plane z: y + z + 1)
      auto leftv = [&](int jr) { return ((jr + z + 1) & 1) == e; };
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
        if (k == 1 || k == B3NC) {
          const bool lf = leftv(jr);
          const double vl = lf ? ve : vo, vr = lf ? vo : ve;
          const int il = 2 * ih + 1, nb = k == 1 ? 6 : 5;
          const unsigned g = bo[r0 + (k == 1 ? -kB3S : kB3S) + xs + B3XS];
          b3_st(dst, g + 8u * b3_gh(nb, il, j), vl);
          b3_st(dst, g + 8u * b3_gh(nb, il + 1, j), vr);
        }
      }
      // x faces: per row the cells x = 0, 15, 16, 31 (lane: row l/4, which l%4)
      {
        const int jr = l >> 2, w = l & 3, j = jr + 1;
        const int pc = w == 0 ? 0 : (w == 1 ? B3H - 1 : (w == 2 ? B3H : 2 * B3H - 1));
        const int xs = 1 + pc / B3H;
        const bool lf = leftv(jr), wantl = (w & 1) == 0;   // x = 0, 16: a left cell; 15, 31: right
        const double v = (wantl == lf) ? fin[z & 1][jr * B3CP + pc][0] : fin[z & 1][jr * B3CP + pc][1];
        const int nxs = wantl ? xs - 1 : xs + 1, nb = wantl ? 2 : 1;
        b3_st(dst, bo[r0 + nxs + B3XS] + 8u * b3_gh(nb, j, k), v);
      }
      // y faces: the cells of rows j = 1 (lanes 0..31) and j = 16 (32..63)
      {
        const int jr = l < 32 ? 0 : B3NC - 1, x = l & 31;
        const int pc = x >> 1, xs = 1 + pc / B3H, i = x - B3NC * (xs - 1) + 1;
        const bool lf = leftv(jr), isl = (x & 1) == 0;
        const double v = (isl == lf) ? fin[z & 1][jr * B3CP + pc][0] : fin[z & 1][jr * B3CP + pc][1];
        const int nys = jr == 0 ? 0 : 2, nb = jr == 0 ? 4 : 3;
        b3_st(dst, bo[r0 + xs + B3XS * nys] + 8u * b3_gh(nb, i, k), v);
      }
    };
    for (int t = -3 - kB3Ahead; t <= zend + 3; t += kB3Ahead) {
#pragma unroll
      for (int u = 0; u < kB3Ahead; u++) {
        flush(t + u);
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

  // plane t: colour 1-e of phi, both colours of rhs (no branch: the waits
  // for these loads are counted; planes past the end reload the last one)
  auto load = [&](int t, double& q, double& fe, double& fo) {
    int k;
    const int zs = zbox(min(t, zend + 2), k);
    const unsigned o = bo[kB3S * zs + slot] + xyb + PB * (k - 1);
    q = b3_ld(src, o);
    fe = b3_ld(rhe, o);
    fo = b3_ld(rho, o);
  };

  // Stage values live in LDS, not registers: stage plane s of buffer t & 1
  // holds V_s at plane t-1-s (the x / y operands and the pair's own other
  // cell), that of buffer (t+1) & 1 still V_s at t-2-s (the plane below: each
  // thread reads its own slot there before it overwrites it).  Registers: rhs
  // of colour e at t-1, t-2, t-3 and of colour 1-e at t-1, t-2.
  double re1 = 0.0, re2 = 0.0, re3 = 0.0, ro1 = 0.0, ro2 = 0.0;
  auto step = [&](int t, double& q, double& fe, double& fo) {
    const double ot = shift ? b3_take(q) - m : b3_take(q);
    const double ret = b3_take(fe), rot = b3_take(fo);
    load(t + kB3Ahead, q, fe, fo);
    const double* P0 = pl[t & 1][0];
    const double* P1 = pl[t & 1][1];
    const double* P2 = pl[t & 1][2];
    double* Q = pl[(t + 1) & 1][0];   // (stage s at s * B3PL)
    // the active cells are the pair's left ones (x0) when colour e is there
    // at plane t-1; the neighbour pair across is on that side
    const int far = ((y + t) & 1) == e ? li - 1 : li + 1;
    Nbr7 n;
    n.c = 0.0;
    // substep 1 (colour e) at plane t-1
    n.xm = P0[far]; n.xp = P0[li]; n.ym = P0[li - B3LP]; n.yp = P0[li + B3LP]; n.zm = Q[li]; n.zp = ot;
    const double s1 = gs_value<OP>(K, n, re1);
    // substep 2 (colour 1-e) at plane t-2
    n.xm = P1[far]; n.xp = P1[li]; n.ym = P1[li - B3LP]; n.yp = P1[li + B3LP]; n.zm = Q[B3PL + li]; n.zp = s1;
    const double s2 = gs_value<OP>(K, n, ro2);
    // substep 3 (colour e) at plane t-3
    const double wb = P2[li];   // colour 1-e at t-3, final
    n.xm = P2[far]; n.xp = wb; n.ym = P2[li - B3LP]; n.yp = P2[li + B3LP]; n.zm = Q[2 * B3PL + li]; n.zp = s2;
    const double s3 = gs_value<OP>(K, n, re3);
    // plane t-3 is final (colour e = s3, colour 1-e = wb): to the store wave
    if (ctr) {
      double* F = fin[(t - 3) & 1][fi];
      F[0] = s3;
      F[1] = wb;
    }
    if (act) {
      Q[li] = ot;
      Q[B3PL + li] = s1;
      Q[2 * B3PL + li] = s2;
    }
    __syncthreads();
    re3 = re2; re2 = re1; re1 = ret;
    ro2 = ro1; ro1 = rot;
  };
  // kB3Ahead planes in flight.  The loop issues every load, planes -3 .. in
  // kB3Ahead extra leading steps that compute nothing used: loads issued
  // before the loop land in other registers than the loop's, and its first
  // wait would drain them all.  Trailing steps past the column compute
  // nothing used either (their loads reload the last plane); the store wave
  // writes plane zend-1 in iteration zend+3.
  double qs[kB3Ahead], fes[kB3Ahead], fos[kB3Ahead];
#pragma unroll
  for (int u = 0; u < kB3Ahead; u++) qs[u] = fes[u] = fos[u] = 0.0;
  for (int t = -3 - kB3Ahead; t <= zend + 3; t += kB3Ahead) {
#pragma unroll
    for (int u = 0; u < kB3Ahead; u++) step(t + u, qs[u], fes[u], fos[u]);
  }
}

namespace {

// k_gsrb4r's tile: the column's boxes and five cells around them (four
// substeps, then the residual one cell out): pairs x0 = 2p - 6, rows y - 5
constexpr int B4NPX = (kB3TX * B3NC + 12) / 2;   // pairs per row: x in [-6, kB3TX*16+5]
constexpr int B4NY = B3NC + 10;                   // rows: y in [-5, 20]
constexpr int B4NT = B4NPX * B4NY;                // compute threads with a pair
constexpr int B4NW = (B4NT + 63) / 64;            // compute waves
constexpr int B4BS = 64 * (B4NW + 1);             // and the store wave
constexpr int B4LP = B4NPX + 2;                   // LDS row pitch of a stage plane
constexpr int B4PL = B4LP * (B4NY + 2);           // LDS doubles per stage plane
// the final phi plane for the residual: the pairs with a cell at distance
// <= 1 from the boxes (x0 in [-2, 32]) and rows y in [-1, 16]
constexpr int B4FP = kB3TX * B3H + 2, B4FN = B4FP * (B3NC + 2);
constexpr int kB4Ahead = B4_AHEAD;               // planes of loads in flight

}  // namespace

// The last four down-substeps of a level, update_coarse's residual and the
// restriction of phi and res (m_multigrid.f90:347-384, 404-436;
// m_restrict.f90:165-214) in one pass: k_gsrb3's pipeline with a fourth
// stage and a halo of five cells, then at plane t-5 the residual of both
// cells of the pair (box_lpl / box_helmh on the final phi: the pair's other
// cell and the planes above and below from registers, the cells across in x
// and y from an LDS plane of final phi), and the 2x2x2 sums of phi (plane
// t-5) and res (plane t-6, one iteration later: the row above's residual
// comes through LDS) in the reference's order: a thread of an even row adds
// its pair (x), then the pair of the row above, and carries the partial sum
// to the next plane.  The store wave writes phi (plane t-5) with its ghost
// faces, res (plane t-6) and the finished coarse cells.
template <int OP>
__global__ void __launch_bounds__(B4BS, B4_WAVES) k_gsrb4r(LevelView L, LevelView C, double* __restrict__ dst,
                                                 const int* __restrict__ cols, double lambda, int e,
                                                 const double* __restrict__ shift) {
  __shared__ double pl[2][4][B4PL];
  __shared__ double fpl[2][B4FN][2];            // final phi at plane t-4 (read at t+1): [pair][left, right]
  __shared__ double rpl[2][B3NC * B3CP][2];     // res at plane t-5 (read at t+1), the boxes' pairs
  __shared__ double cph[B3NC / 2][B3CP];        // coarse phi / res cells finished this iteration:
  __shared__ double crs[B3NC / 2][B3CP];        //   [coarse row][coarse x across the tile]
  __shared__ unsigned bo[kB3Rec];
  __shared__ unsigned cpo[kB3MaxZ * kB3TX];
  __shared__ int cdx[kB3MaxZ * kB3TX];
  __shared__ int len_s;
  const int tid = threadIdx.x;
  const int cq = xcd_box(blockIdx.x, gridDim.x);
  if (tid < kB3Rec) {
    const int v = cols[(long long)cq * kB3Rec + tid];
    if (tid == 0) len_s = v;
    else if (tid < kB3Par) bo[tid - 1] = (unsigned)v * (unsigned)(L.stride * 8);
    else if (tid < kB3Par + 2 * kB3MaxZ * kB3TX) {
      const int m = (tid - kB3Par) >> 1;
      if ((tid - kB3Par) & 1) cdx[m] = v;
      else cpo[m] = v < 0 ? 0xffffffffu : (unsigned)v * (unsigned)(C.stride * 8);
    }
  }
  for (int q = tid; q < 2 * 4 * B4PL; q += B4BS) (&pl[0][0][0])[q] = 0.0;
  for (int q = tid; q < 2 * B4FN * 2; q += B4BS) (&fpl[0][0][0])[q] = 0.0;
  __syncthreads();
  const int len = len_s, zend = B3NC * len;
  constexpr unsigned PB = 8u * B3H * B3NC;
  auto zbox = [&](int t, int& k) {
    const int zs = t < 0 ? 0 : (t >= zend ? len + 1 : (t >> 4) + 1);
    k = t - B3NC * (zs - 1) + 1;
    return zs;
  };
  // colour e is the left cell of the pairs of row y (0-based) at plane z
  auto lefte = [&](int yy, int z) { return ((yy + z + 1) & 1) == e; };
  // planes -5 .. zend+4 are loaded; the store wave writes the last coarse res
  // cells in iteration zend+6
  const int t_end = zend + 6;

  if (tid >= B4NW * 64) {
    // ---- the store wave ----------------------------------------------------
    const int l = tid - B4NW * 64;
    double* __restrict__ rsv = L.data + 3 * L.vstride;
    double* __restrict__ cres = C.data + 3 * C.vstride;
    auto flush = [&](int t) {
      // phi of plane t-5 (fpl[t & 1], the plane the residual reads in this
      // iteration) and the ghost faces it is part of
      const int z = t - 5;
      if (z >= 0 && z < zend) {
        int k;
        const int r0 = kB3S * zbox(z, k);
#pragma unroll
        for (int r = 0; r < B3NC * B3CP / 64; r++) {
          const int q = l + 64 * r, jr = q / B3CP, pc = q % B3CP;
          const int xs = 1 + pc / B3H, ih = pc % B3H, j = jr + 1;
          const double* F = fpl[t & 1][(pc + 1) + B4FP * (jr + 1)];
          const double vl = F[0], vr = F[1];
          const bool le = lefte(jr, z);
          const unsigned o = bo[r0 + xs + B3XS] + 8u * (ih + B3H * (j - 1)) + PB * (k - 1);
          b3_st(dst + e * B3HV, o, le ? vl : vr);
          b3_st(dst + (1 - e) * B3HV, o, le ? vr : vl);
          if (k == 1 || k == B3NC) {
            const int il = 2 * ih + 1, nb = k == 1 ? 6 : 5;
            const unsigned g = bo[r0 + (k == 1 ? -kB3S : kB3S) + xs + B3XS];
            b3_st(dst, g + 8u * b3_gh(nb, il, j), vl);
            b3_st(dst, g + 8u * b3_gh(nb, il + 1, j), vr);
          }
        }
        {   // x faces: per row the cells x = 0, 15, 16, 31
          const int jr = l >> 2, w = l & 3, j = jr + 1;
          const int pc = w == 0 ? 0 : (w == 1 ? B3H - 1 : (w == 2 ? B3H : 2 * B3H - 1));
          const int xs = 1 + pc / B3H;
          const bool wantl = (w & 1) == 0;
          const double v = fpl[t & 1][(pc + 1) + B4FP * (jr + 1)][wantl ? 0 : 1];
          b3_st(dst, bo[r0 + (wantl ? xs - 1 : xs + 1) + B3XS] + 8u * b3_gh(wantl ? 2 : 1, j, k), v);
        }
        {   // y faces: rows j = 1 (lanes 0..31) and j = 16 (32..63)
          const int jr = l < 32 ? 0 : B3NC - 1, x = l & 31;
          const int pc = x >> 1, xs = 1 + pc / B3H, i = x - B3NC * (xs - 1) + 1;
          const double v = fpl[t & 1][(pc + 1) + B4FP * (jr + 1)][x & 1];
          b3_st(dst, bo[r0 + xs + B3XS * (jr == 0 ? 0 : 2)] + 8u * b3_gh(jr == 0 ? 4 : 3, i, k), v);
        }
      }
      // res of plane t-6 (rpl[t & 1])
      const int zr = t - 6;
      if (zr >= 0 && zr < zend) {
        int k;
        const int r0 = kB3S * zbox(zr, k);
#pragma unroll
        for (int r = 0; r < B3NC * B3CP / 64; r++) {
          const int q = l + 64 * r, jr = q / B3CP, pc = q % B3CP;
          const int xs = 1 + pc / B3H, ih = pc % B3H;
          const double vl = rpl[t & 1][q][0], vr = rpl[t & 1][q][1];
          const bool le = lefte(jr, zr);
          const unsigned o = bo[r0 + xs + B3XS] + 8u * (ih + B3H * jr) + PB * (k - 1);
          b3_st(rsv + e * B3HV, o, le ? vl : vr);
          b3_st(rsv + (1 - e) * B3HV, o, le ? vr : vl);
        }
      }
      // the coarse cells the previous iteration finished: phi of the plane
      // pair ending at t-6, res of the pair ending at t-7
#pragma unroll
      for (int w = 0; w < 2; w++) {
        const int zc = t - 6 - w;
        if (zc < 0 || zc >= zend || !(zc & 1)) continue;
        int k;
        const int zs = zbox(zc, k);
        const int kc = k >> 1;   // k = 2 kc
#pragma unroll
        for (int r = 0; r < (B3NC / 2) * B3CP / 64; r++) {
          const int q = l + 64 * r, jc = q / B3CP + 1, xc = q % B3CP;
          const int m = (zs - 1) * kB3TX + xc / B3H, ic = xc % B3H + 1;
          const unsigned base = cpo[m];
          if (base == 0xffffffffu) continue;   // parent on another rank (restrict_remote)
          const int dp = cdx[m], dx = dp & 1023, dy = (dp >> 10) & 1023, dz = dp >> 20;
          const int I = dx + ic, J = dy + jc, Kc = dz + kc;
          const unsigned o =
              base + 8u * (((I + J + Kc) & 1) * B3HV + ((I - 1) >> 1) + B3H * ((J - 1) + B3NC * (Kc - 1)));
          b3_st(w == 0 ? C.phi : cres, o, w == 0 ? cph[jc - 1][xc] : crs[jc - 1][xc]);
        }
      }
    };
    for (int t = -5 - kB4Ahead; t <= t_end; t += kB4Ahead) {
#pragma unroll
      for (int u = 0; u < kB4Ahead; u++) {
        flush(t + u);
        __syncthreads();
      }
    }
    return;
  }

  // ---- the compute waves ---------------------------------------------------
  const bool act = tid < B4NT;
  const int p = tid % B4NPX, y = tid / B4NPX - 5;
  const int x0 = 2 * p - 6;
  const int xs = x0 < 0 ? 0 : (x0 < kB3TX * B3NC ? 1 + x0 / B3NC : kB3TX + 1);
  const int ys = y < 0 ? 0 : (y < B3NC ? 1 : 2);
  const int ih = (x0 - B3NC * (xs - 1)) >> 1, j = y - B3NC * (ys - 1) + 1;
  const int slot = xs + B3XS * ys;
  const unsigned xyb = 8u * (ih + B3H * (j - 1));
  const int li = act ? (p + 1) + B4LP * (y + 6) : B4LP + 1;
  const bool ctr = act && xs >= 1 && xs <= kB3TX && ys == 1;
  // the residual region (pairs with a cell at distance <= 1 from the boxes):
  // its fpl index; the boxes' pairs: rpl index and coarse x (p - 3)
  const bool rreg = act && x0 >= -2 && x0 <= kB3TX * B3NC && y >= -1 && y <= B3NC;
  const int fq = rreg ? (p - 2) + B4FP * (y + 1) : 0;
  const int rq = ctr ? y * B3CP + (p - 3) : 0;
  const bool rsum = ctr && !(y & 1);   // adds the 2x2 block of its row pair
  const double m = shift ? *shift : 0.0;
  const OpCoef<OP> K(L, lambda);
  const double* __restrict__ src = L.phi + (1 - e) * B3HV;
  const double* __restrict__ rhe = L.data + L.vstride + e * B3HV;
  const double* __restrict__ rho = L.data + L.vstride + (1 - e) * B3HV;

  auto load = [&](int t, double& q, double& fe, double& fo) {
    int k;
    const int zs = zbox(min(t, zend + 4), k);
    const unsigned o = bo[kB3S * zs + slot] + xyb + PB * (k - 1);
    q = b3_ld(src, o);
    fe = b3_ld(rhe, o);
    fo = b3_ld(rho, o);
  };

  // Stage values live in LDS, not registers: stage plane s of buffer t & 1
  // holds V_s at plane t-1-s (the x / y operands and the pair's own other
  // cell), that of buffer (t+1) & 1 still V_s at t-2-s (the plane below: each
  // thread reads its own slot there before it overwrites it).  fpl likewise
  // holds the final phi at t-5 / t-6, rpl the res at t-6.  Registers: rhs of
  // both colours at t-1 .. t-5 and the partial 2x2x2 sums.
  double re1 = 0.0, re2 = 0.0, re3 = 0.0, re4 = 0.0, re5 = 0.0;
  double ro1 = 0.0, ro2 = 0.0, ro3 = 0.0, ro4 = 0.0, ro5 = 0.0;
  double aph = 0.0, ars = 0.0;
  auto step = [&](int t, double& q, double& fe, double& fo) {
    const double ot = shift ? b3_take(q) - m : b3_take(q);
    const double ret = b3_take(fe), rot = b3_take(fo);
    load(t + kB4Ahead, q, fe, fo);
    const double* P0 = pl[t & 1][0];
    const double* P1 = pl[t & 1][1];
    const double* P2 = pl[t & 1][2];
    const double* P3 = pl[t & 1][3];
    double* Q = pl[(t + 1) & 1][0];   // (stage s at s * B4PL)
    // colour e is the left cell at t-1 (and t-3, t-5): then the four active
    // cells (e at t-1, 1-e at t-2, e at t-3, 1-e at t-4) are all left ones
    const bool left = lefte(y, t - 1);
    const int far = left ? li - 1 : li + 1;
    Nbr7 n;
    n.c = 0.0;
    n.xm = P0[far]; n.xp = P0[li]; n.ym = P0[li - B4LP]; n.yp = P0[li + B4LP]; n.zm = Q[li]; n.zp = ot;
    const double s1 = gs_value<OP>(K, n, re1);
    B4_STAGE_FENCE;
    n.xm = P1[far]; n.xp = P1[li]; n.ym = P1[li - B4LP]; n.yp = P1[li + B4LP]; n.zm = Q[B4PL + li]; n.zp = s1;
    const double s2 = gs_value<OP>(K, n, ro2);
    B4_STAGE_FENCE;
    n.xm = P2[far]; n.xp = P2[li]; n.ym = P2[li - B4LP]; n.yp = P2[li + B4LP]; n.zm = Q[2 * B4PL + li]; n.zp = s2;
    const double s3 = gs_value<OP>(K, n, re3);
    B4_STAGE_FENCE;
    const double v3 = P3[li];   // V3 at t-4
    n.xm = P3[far]; n.xp = v3; n.ym = P3[li - B4LP]; n.yp = P3[li + B4LP]; n.zm = Q[3 * B4PL + li]; n.zp = s3;
    const double s4 = gs_value<OP>(K, n, ro4);
    B4_STAGE_FENCE;
    // final phi of the pair at t-4 (left, right): colour e = V3, colour 1-e =
    // V4; colour e is the left cell at t-4 iff not `left`
    const double f4l = left ? s4 : v3, f4r = left ? v3 : s4;
    if (ctr) {
      // residual at t-5, both cells (rhs of colour e / 1-e by side); the pair
      // itself at t-5 and t-6 from fpl
      const double(*FP)[2] = fpl[t & 1];
      const double f5l = FP[fq][0], f5r = FP[fq][1];
      const double f6l = fpl[(t + 1) & 1][fq][0], f6r = fpl[(t + 1) & 1][fq][1];
      Nbr7 a;
      a.c = f5l; a.xm = FP[fq - 1][1]; a.xp = f5r; a.ym = FP[fq - B4FP][0]; a.yp = FP[fq + B4FP][0];
      a.zm = f6l; a.zp = f4l;
      const double r5l = (left ? re5 : ro5) - op_value<OP>(K, a);
      a.c = f5r; a.xm = f5l; a.xp = FP[fq + 1][0]; a.ym = FP[fq - B4FP][1]; a.yp = FP[fq + B4FP][1];
      a.zm = f6r; a.zp = f4r;
      const double r5r = (left ? ro5 : re5) - op_value<OP>(K, a);
      if (rsum) {
        const int z5 = t - 5, z6 = t - 6;
        if (z5 >= 0 && z5 < zend) {   // phi at t-5: this row's pair, then the row above's
          const double s = (((((z5 & 1) ? aph : 0.0) + f5l) + f5r) + FP[fq + B4FP][0]) + FP[fq + B4FP][1];
          if (z5 & 1) cph[y >> 1][p - 3] = 0.125 * s;
          aph = s;
        }
        if (z6 >= 0 && z6 < zend) {   // res at t-6 (rpl: this row's and the row above's)
          const double(*RP)[2] = rpl[t & 1];
          const double s = (((((z6 & 1) ? ars : 0.0) + RP[rq][0]) + RP[rq][1]) + RP[rq + B3CP][0]) + RP[rq + B3CP][1];
          if (z6 & 1) crs[y >> 1][p - 3] = 0.125 * s;
          ars = s;
        }
      }
      rpl[(t + 1) & 1][rq][0] = r5l;
      rpl[(t + 1) & 1][rq][1] = r5r;
    }
    if (rreg) {
      fpl[(t + 1) & 1][fq][0] = f4l;
      fpl[(t + 1) & 1][fq][1] = f4r;
    }
    if (act) {
      Q[li] = ot;
      Q[B4PL + li] = s1;
      Q[2 * B4PL + li] = s2;
      Q[3 * B4PL + li] = s3;
    }
    __syncthreads();
    re5 = re4; re4 = re3; re3 = re2; re2 = re1; re1 = ret;
    ro5 = ro4; ro4 = ro3; ro3 = ro2; ro2 = ro1; ro1 = rot;
  };
  double qs[kB4Ahead], fes[kB4Ahead], fos[kB4Ahead];
#pragma unroll
  for (int u = 0; u < kB4Ahead; u++) qs[u] = fes[u] = fos[u] = 0.0;
  for (int t = -5 - kB4Ahead; t <= t_end; t += kB4Ahead) {
#pragma unroll
    for (int u = 0; u < kB4Ahead; u++) step(t + u, qs[u], fes[u], fos[u]);
  }
}

bool gsrb3_op_ok(int op) { return op == OP_LPL || op == OP_HELM; }

void launch_gsrb3(const LevelView& L, double* dst, const int* cols, int n_cols, int op, double lambda, int e,
                  const double* shift, hipStream_t st) {
  if (n_cols <= 0) return;
  if (L.nc != B3NC) throw std::runtime_error("launch_gsrb3: box size must be 16");
  if (op == OP_HELM)
    k_gsrb3<OP_HELM><<<n_cols, B3BS, 0, st>>>(L, dst, cols, lambda, e, shift);
  else
    k_gsrb3<OP_LPL><<<n_cols, B3BS, 0, st>>>(L, dst, cols, lambda, e, shift);
}

void launch_gsrb4r(const LevelView& L, const LevelView& C, double* dst, const int* cols, int n_cols, int op,
                   double lambda, int e, const double* shift, hipStream_t st) {
  if (n_cols <= 0) return;
  if (L.nc != B3NC || C.nc != B3NC) throw std::runtime_error("launch_gsrb4r: box sizes must be 16");
  if (op == OP_HELM)
    k_gsrb4r<OP_HELM><<<n_cols, B4BS, 0, st>>>(L, C, dst, cols, lambda, e, shift);
  else
    k_gsrb4r<OP_LPL><<<n_cols, B4BS, 0, st>>>(L, C, dst, cols, lambda, e, shift);
}

}  // namespace omg
