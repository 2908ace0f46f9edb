// omg_small.hip — three red-black substeps of a small level in one launch
// (k_gsrb_small).
//
// On levels of a few hundred boxes or fewer every launch is latency-bound:
// the one-substep kernel takes 5-9 us whether the level has 8 or 512 boxes
// (DESIGN §12.9), and smooth_boxes (m_multigrid.f90:404-424) runs one per
// substep.  The column passes of omg_block.hip stream a column's planes in
// sequence and measured slower there.  Here one workgroup takes
// one box and a 3-cell halo of its neighbours' cells (a 22^3 tile of phi and
// a 20^3 tile of rhs in LDS) and runs the three substeps on shrinking regions
// of the tile: substep s updates the cells within 3-s (in the sum of the
// per-axis distances) of the box, the cells the later substeps read.  After
// the start and after every substep the ghost layer across the level's
// physical faces is formed from the cells inside (bc_to_gc,
// m_ghost_cells.f90:665-766, as the reference's fill after each substep), for
// the box's own faces and for its neighbours' that the tile reaches.  Every
// update reads the operands the reference's substep reads, in the same
// expression: bit-identical.
//
// The neighbours' cells are read from phi while they update their own boxes,
// so the pass writes the level's other phi buffer (the host swaps
// Level::d_phi, as for the column passes): the box's interior, its boundary
// cells into its same-GPU neighbours' ghost faces and its physical ghosts,
// both colours.  Levels of 16^3 boxes whose faces are same-GPU boxes or
// physical (no refinement boundaries, no faces on other GPUs), Laplacian /
// Helmholtz, consistent ghosts on entry.
#include <stdexcept>

#include "omg_device.h"
#include "omg_face.h"
#include "omg_kernels.h"

namespace omg {

namespace {

constexpr int SNC = 16;                  // box size
constexpr int SD = 3;                    // halo depth = substeps per launch
constexpr int ST = SNC + 2 * SD;         // phi tile: i in [1-SD, SNC+SD]
constexpr int SR = SNC + 2 * (SD - 1);   // rhs tile: the cells substep 1 updates
constexpr int SBS = 1024;                // threads per workgroup

__device__ __forceinline__ int s_pt(int i, int j, int k) {   // phi tile slot of box coordinates (1-based)
  return (i + SD - 1) + ST * ((j + SD - 1) + ST * (k + SD - 1));
}
__device__ __forceinline__ int s_rt(int i, int j, int k) {   // rhs tile slot
  return (i + SD - 2) + SR * ((j + SD - 2) + SR * (k + SD - 2));
}
// distance of a coordinate from the box's range, and its region (0 below, 1
// in, 2 above)
__device__ __forceinline__ int s_ex(int i) { return i < 1 ? 1 - i : (i > SNC ? i - SNC : 0); }
__device__ __forceinline__ int s_rg(int i) { return i < 1 ? 0 : (i > SNC ? 2 : 1); }

}  // namespace

template <int OP>
__global__ void __launch_bounds__(SBS) k_gsrb_small(LevelView L, double* __restrict__ dst, double lambda, int e,
                                                    const double* __restrict__ shift, GcBC bc) {
  __shared__ double P[ST * ST * ST];
  __shared__ double R[SR * SR * SR];
  __shared__ int nbr[27];   // the box of region (rx, ry, rz) around ours, -1 across a physical face
  const int tid = threadIdx.x;
  const int b = xcd_box(blockIdx.x, gridDim.x);
  if (tid < 27) {
    // walk x, then y, then z from our box (uniform levels: any order meets the
    // same box)
    const int r[3] = {tid % 3, (tid / 3) % 3, tid / 9};
    int x = b;
    for (int d = 0; d < 3 && x >= 0; d++) {
      if (r[d] == 1) continue;
      const long long f = (long long)x * 6 + 2 * d + (r[d] == 2 ? 1 : 0);
      x = L.nbk[f] == NB_LOCAL ? L.nba[f] : -1;
    }
    nbr[tid] = x;
  }
  __syncthreads();
  const double m = shift ? *shift : 0.0;
  // the start state: phi within 3 of the box, rhs within 2 (unused slots 0).
  // Every load is issued before any lands in LDS: one round trip, not one per
  // slot a thread fills
  constexpr int NP = ST * ST * ST, NR = SR * SR * SR, NPT = (NP + SBS - 1) / SBS, NRT = (NR + SBS - 1) / SBS;
  const double* __restrict__ rhs = L.data + L.vstride;
  double vp[NPT], vr[NRT];
#pragma unroll
  for (int r = 0; r < NPT; r++) {
    const int q = tid + SBS * r;
    vp[r] = 0.0;
    if (q >= NP) continue;
    const int i = q % ST + 1 - SD, j = (q / ST) % ST + 1 - SD, k = q / (ST * ST) + 1 - SD;
    if (s_ex(i) + s_ex(j) + s_ex(k) > SD) continue;
    const int rx = s_rg(i), ry = s_rg(j), rz = s_rg(k);
    const int sb = nbr[rx + 3 * ry + 9 * rz];
    if (sb >= 0)
      vp[r] = L.phi[(long long)sb * L.stride + off_int(L, i - SNC * (rx - 1), j - SNC * (ry - 1), k - SNC * (rz - 1))];
  }
#pragma unroll
  for (int r = 0; r < NRT; r++) {
    const int q = tid + SBS * r;
    vr[r] = 0.0;
    if (q >= NR) continue;
    const int i = q % SR + 2 - SD, j = (q / SR) % SR + 2 - SD, k = q / (SR * SR) + 2 - SD;
    if (s_ex(i) + s_ex(j) + s_ex(k) > SD - 1) continue;
    const int rx = s_rg(i), ry = s_rg(j), rz = s_rg(k);
    const int sb = nbr[rx + 3 * ry + 9 * rz];
    if (sb >= 0)
      vr[r] = rhs[(long long)sb * L.stride + off_int(L, i - SNC * (rx - 1), j - SNC * (ry - 1), k - SNC * (rz - 1))];
  }
  // the ghost layer across physical faces: the slots one cell past the box
  // range in exactly one coordinate whose box (in range in that coordinate)
  // exists and has no neighbour there, i.e. its face cell (a, c) of that box.
  // Each thread's slots and their bc_to_gc terms (phys_ghost's: c0 * b, c1,
  // c2, the boundary value from the table it names) are found once here
  constexpr int NFS = 6 * ST * ST, NFT = (NFS + SBS - 1) / SBS;
  int gpos[NFT], gx1[NFT], gx2[NFT];
  double gk[NFT], gc1[NFT], gc2[NFT];
#pragma unroll
  for (int r = 0; r < NFT; r++) {
    gpos[r] = -1;
    gx1[r] = gx2[r] = 0;
    gk[r] = gc1[r] = gc2[r] = 0.0;
    const int p = tid + SBS * r;
    if (p >= NFS) continue;
    const int fc = p / (ST * ST), t = p % (ST * ST);
    const int d = fc >> 1, hi = fc & 1;
    const int u = t % ST + 1 - SD, w = t / ST + 1 - SD;   // tangential coordinates, ascending axes
    if (s_ex(u) + s_ex(w) > SD - 1) continue;               // (no substep reads it)
    int c3[3];
    const int t1 = d == 0 ? 1 : 0, t2 = d == 2 ? 1 : 2;
    c3[d] = hi ? SNC + 1 : 0;
    c3[t1] = u;
    c3[t2] = w;
    int rr[3] = {s_rg(c3[0]), s_rg(c3[1]), s_rg(c3[2])};
    rr[d] = 1;
    const int ob = nbr[rr[0] + 3 * rr[1] + 9 * rr[2]];
    rr[d] = hi ? 2 : 0;
    if (ob < 0 || nbr[rr[0] + 3 * rr[1] + 9 * rr[2]] >= 0) continue;
    const int nb = 2 * d + hi + 1;
    const int a = u - SNC * (s_rg(u) - 1), cc = w - SNC * (s_rg(w) - 1);
    int x1[3] = {c3[0], c3[1], c3[2]}, x2[3] = {c3[0], c3[1], c3[2]};
    x1[d] = hi ? SNC : 1;
    x2[d] = hi ? SNC - 1 : 2;
    gpos[r] = s_pt(c3[0], c3[1], c3[2]);
    gx1[r] = s_pt(x1[0], x1[1], x1[2]);
    gx2[r] = s_pt(x2[0], x2[1], x2[2]);
    // (phys_ghost, omg_face.h, with the product c0 * b formed once)
    const long long f = (long long)ob * 6 + nb - 1;
    double bv;
    int type;
    if (bc.phi_stored) {
      bv = L.data[L.vstride + (long long)ob * L.stride + off_gh(L, nb, a, cc)];
      type = L.nba[f];   // (the boundary code the reference's neighbour slot holds, as face_cell_fill)
    } else if (bc.face_off && bc.face_off[f] >= 0) {
      bv = bc.face_data[bc.face_off[f] + (a - 1) + (long long)SNC * (cc - 1)];
      type = bc.face_type[f];
    } else {
      bv = bc.value[nb - 1];
      type = bc.type[nb - 1];
    }
    double c0;
    if (type == -10) {
      c0 = 2; gc1[r] = -1; gc2[r] = 0;
    } else if (type == -11) {
      c0 = L.dr[(nb - 1) >> 1] * ((nb & 1) ? -1.0 : 1.0); gc1[r] = 1; gc2[r] = 0;
    } else {
      c0 = 0; gc1[r] = 2; gc2[r] = -1;
    }
    gk[r] = c0 * bv;
  }
#pragma unroll
  for (int r = 0; r < NPT; r++)
    if (tid + SBS * r < NP) P[tid + SBS * r] = vp[r] - m;
#pragma unroll
  for (int r = 0; r < NRT; r++)
    if (tid + SBS * r < NR) R[tid + SBS * r] = vr[r];
  __syncthreads();
  auto fill = [&]() {
#pragma unroll
    for (int r = 0; r < NFT; r++)
      if (gpos[r] >= 0) P[gpos[r]] = (gk[r] + gc1[r] * P[gx1[r]]) + gc2[r] * P[gx2[r]];
  };
  fill();
  __syncthreads();

  const OpCoef<OP> K(L, lambda);
#pragma unroll
  for (int s = 1; s <= SD; s++) {
    // (unrolled: the region's extent W is a constant of each substep)
    const int c = (s & 1) ? e : 1 - e, dd = SD - s, W = SNC + 2 * dd, lo = 1 - dd;
    // the colour-c cells of the region, pairs of x positions per thread step
    for (int q = tid; q < (W / 2) * W * W; q += SBS) {
      const int ih = q % (W / 2), j = (q / (W / 2)) % W + lo, k = q / ((W / 2) * W) + lo;
      const int i0 = lo + 2 * ih, i = i0 + (((i0 + j + k) & 1) != c ? 1 : 0);
      if (s_ex(i) + s_ex(j) + s_ex(k) > dd) continue;
      if (nbr[s_rg(i) + 3 * s_rg(j) + 9 * s_rg(k)] < 0) continue;   // (across a physical face)
      const int o = s_pt(i, j, k);
      Nbr7 n;
      n.c = 0.0;
      n.xm = P[o - 1]; n.xp = P[o + 1];
      n.ym = P[o - ST]; n.yp = P[o + ST];
      n.zm = P[o - ST * ST]; n.zp = P[o + ST * ST];
      P[o] = gs_value<OP>(K, n, R[s_rt(i, j, k)]);
    }
    __syncthreads();
    fill();
    __syncthreads();
  }

  // the box to the other buffer: interior (in storage order), the boundary
  // cells into same-GPU neighbours' ghost faces, the physical ghosts
  double* __restrict__ ub = dst + (long long)b * L.stride;
  constexpr int SH = SNC / 2, SHV = SH * SNC * SNC;
  for (int q = tid; q < 2 * SHV; q += SBS) {
    const int col = q >= SHV, r = q - col * SHV;
    const int ih = r % SH, row = r / SH, j = row % SNC + 1, k = row / SNC + 1;
    const int i = 2 * ih + 1 + ((1 + j + k + col) & 1);
    ub[q] = P[s_pt(i, j, k)];
  }
  for (int p = tid; p < 6 * SNC * SNC; p += SBS) {
    const int fc = p / (SNC * SNC), cell = p % (SNC * SNC), a = cell % SNC + 1, cc = cell / SNC + 1;
    const int nb = fc + 1, d = fc >> 1, hi = fc & 1;
    const long long f = (long long)b * 6 + fc;
    int c3[3];
    const int t1 = d == 0 ? 1 : 0, t2 = d == 2 ? 1 : 2;
    c3[t1] = a;
    c3[t2] = cc;
    if (L.nbk[f] == NB_LOCAL) {
      c3[d] = hi ? SNC : 1;
      dst[(long long)L.nba[f] * L.stride + off_gh(L, hi ? nb - 1 : nb + 1, a, cc)] = P[s_pt(c3[0], c3[1], c3[2])];
    } else {
      c3[d] = hi ? SNC + 1 : 0;
      ub[off_gh(L, nb, a, cc)] = P[s_pt(c3[0], c3[1], c3[2])];
    }
  }
}

bool gsrb_small_ok(int nc, int op) { return nc == SNC && (op == OP_LPL || op == OP_HELM); }

void launch_gsrb_small(const LevelView& L, double* dst, int op, double lambda, int e, const double* shift,
                       const GcBC& bc, hipStream_t st) {
  if (L.n <= 0) return;
  if (!gsrb_small_ok(L.nc, op)) throw std::runtime_error("launch_gsrb_small: 16^3 boxes, Laplacian / Helmholtz");
  if (op == OP_HELM)
    k_gsrb_small<OP_HELM><<<L.n, SBS, 0, st>>>(L, dst, lambda, e, shift, bc);
  else
    k_gsrb_small<OP_LPL><<<L.n, SBS, 0, st>>>(L, dst, lambda, e, shift, bc);
}

}  // namespace omg
