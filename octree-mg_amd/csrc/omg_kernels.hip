// omg_kernels.hip — gfx950 kernels of the octree-mg V-cycle hot path.
//
// Every kernel covers one whole octree level (all boxes this rank owns there)
// in one launch, over the colour-split box layout of omg_device.h.
// Arithmetic is fp64 and keeps the reference's association order term by
// term (compiled with -ffp-contract=off, so no FMA contraction), which makes
// every result bit-identical to the reference CPU solver.  Reference routines
// are cited as path:line of FermiQ/octree-mg.
#include "omg_device.h"
#include "omg_face.h"
#include "omg_gsrb.h"
#include "omg_kernels.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace omg {

static inline unsigned grid_for(long long work, int block = 256) {
  long long g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 2048 * 8) g = 2048 * 8;
  return (unsigned)g;
}

#define GRID_STRIDE(t, total)                                                       \
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < (total); \
       t += (long long)gridDim.x * blockDim.x)

// Ghost fill of a level: one thread per (box, face, face cell).
__global__ void __launch_bounds__(256) k_fill_gc(LevelView L, int iv, int colours, LevelView C,
                                                 const RBRec* rb, GcBC bc, double* sendbuf) {
  const int nc = L.nc, nc2 = nc * nc;
  if (nc == 1) {   // (the reference's face order, box1_fill)
    GRID_STRIDE(b, (long long)L.n) box1_fill(L, iv, (int)b, C, rb, bc, sendbuf);
    return;
  }
  GRID_STRIDE(t, (long long)L.n * 6 * nc2) {
    const int cell = (int)(t % nc2), f = (int)(t / nc2);
    face_cell_fill(L, iv, f / 6, f % 6 + 1, cell % nc + 1, cell / nc + 1, colours, C, rb, bc, sendbuf);
  }
}

// fill_buffered_nb (m_ghost_cells.f90:424-454): received faces -> ghosts.
// colours: bit e set = write the ghosts of colour e (the sender packs whole
// faces; a caller that knows only colour e changed writes that half only).
__global__ void __launch_bounds__(256) k_unpack_faces(LevelView L, int iv, const int* items, int n_items,
                                                      const double* recv, int colours) {
  const int nc = L.nc, nc2 = nc * nc;
  GRID_STRIDE(t, (long long)n_items * nc2) {
    const int q = (int)(t / nc2), cell = (int)(t % nc2);
    const int it = items[q], b = it / 6, nb = it % 6 + 1;
    const int a = cell % nc + 1, c = cell / nc + 1, g = (nb & 1) ? 0 : nc + 1;
    if (!((colours >> ((g + a + c) & 1)) & 1)) continue;
    boxp(L, iv, b)[off_gh(L, nb, a, c)] = recv[t];
  }
}

// Deep halo of a level split over GPUs (k_gsrb3 / k_gsrb4 on split levels,
// omg_api.cpp plan_deep): a remote box that some column here reads is held
// as a proxy box after this rank's boxes in every variable, and the cells the
// columns read (4 layers toward this rank's boxes, whole across) travel as
// 4 x 4 x 4 bricks, brick = bx + 4 by + 16 bz.  per = 32: one colour c of
// the brick; 64: both colours.  A brick row of 4 cells is two consecutive
// slots of each colour (omg_device.h off_int), so a brick of one colour is 16
// slot pairs: slot 2 bx + w of row (4 by + jj, 4 bz + kk).  items: (box, brick)
// pairs, box = a local box (pack) or n + proxy (unpack); the same order on
// both sides (sort_and_transfer_buffers' keys, m_communication.f90:37-66).
__global__ void __launch_bounds__(256) k_deep_copy(LevelView L, int iv, int c, int per, const int* items,
                                                   int n_items, double* buf, int unpack) {
  GRID_STRIDE(t, (long long)n_items * per) {
    const int q = (int)(t / per);
    int r = (int)(t % per);
    const int cc = per == 64 ? r >> 5 : c;
    r &= 31;
    const int b = items[2 * q], br = items[2 * q + 1];
    const int w = r & 1, jj = (r >> 1) & 3, kk = r >> 3;
    const int bx = br & 3, by = (br >> 2) & 3, bz = br >> 4;
    double* p = boxp(L, iv, b) + cc * L.hv + 2 * bx + w + L.h * ((4 * by + jj) + L.nc * (4 * bz + kk));
    if (unpack)
      *p = buf[t];
    else
      buf[t] = *p;
  }
}

void launch_deep_copy(const LevelView& L, int iv, int c, int per, const int* items, int n, double* buf, bool unpack,
                      hipStream_t st) {
  if (L.nc != 16 || (per != 32 && per != 64)) throw std::runtime_error("launch_deep_copy: 16^3 boxes, 32 or 64");
  const long long work = (long long)n * per;
  if (work == 0) return;
  k_deep_copy<<<grid_for(work), 256, 0, st>>>(L, iv, c, per, items, n, buf, unpack ? 1 : 0);
}

// the boundary layer of variable iv at the listed faces (items b*6+nb-1) into
// the halo send buffer, nc*nc doubles per face in the order k_unpack_faces
// writes the peer's ghosts: after a pass that does not pack (k_gsrb3 /
// k_gsrb4 on split levels; iv 4: the res its RES form stores)
__global__ void __launch_bounds__(256) k_face_pack(LevelView L, int iv, const int* items, int n_items,
                                                   double* buf) {
  const int nc = L.nc, nc2 = nc * nc;
  GRID_STRIDE(t, (long long)n_items * nc2) {
    const int q = (int)(t / nc2), cell = (int)(t % nc2);
    const int f = items[q], b = f / 6, nb = f % 6 + 1;
    buf[t] = boxp(L, iv, b)[off_face_cell(L, nb, (nb & 1) ? 1 : nc, cell % nc + 1, cell / nc + 1)];
  }
}

void launch_face_pack(const LevelView& L, int iv, const int* items, int n, double* buf, hipStream_t st) {
  const long long work = (long long)n * L.nc * L.nc;
  if (work == 0) return;
  k_face_pack<<<grid_for(work), 256, 0, st>>>(L, iv, items, n, buf);
}

// buffer_for_fine_nb (m_ghost_cells.f90:385-422) on the coarse rank: the
// coarse face next to a fine neighbour on another rank, interpolated by
// box_gc_for_fine_neighbor (:500-577).  Item = (coarse box, coarse-side nb,
// packed child offset of the fine box).
__global__ void __launch_bounds__(256) k_rb_pack(LevelView C, int iv, const int* items, int n_items, int nc,
                                                 double* buf) {
  const int nc2 = nc * nc;
  GRID_STRIDE(t, (long long)n_items * nc2) {
    const int q = (int)(t / nc2), cell = (int)(t % nc2);
    const int cb = items[3 * q], nbc = items[3 * q + 1], dp = items[3 * q + 2];
    const int dix[3] = {dp & 1023, (dp >> 10) & 1023, dp >> 20};
    const int a = cell % nc + 1, c = cell / nc + 1;
    const int d = (nbc + 1) >> 1;
    const int t1 = (d == 1) ? 1 : 0, t2 = (d == 3) ? 1 : 2;
    const int clayer = (nbc & 1) ? 1 : C.nc;     // low side: cc(1,..), high: cc(nc,..)
    const double* cu = boxp(C, iv, cb);
    const int i = (a + 1) >> 1, j = (c + 1) >> 1;
    auto T = [&](int p, int r) { return cu[off_face_cell(C, nbc, clayer, dix[t1] + p, dix[t2] + r)]; };
    const double tc = T(i, j);
    const double g1 = 0.125 * (T(i + 1, j) - T(i - 1, j));
    const double g2 = 0.125 * (T(i, j + 1) - T(i, j - 1));
    double gv = ((a - 1) & 1) ? tc + g1 : tc - g1;
    gv = ((c - 1) & 1) ? gv + g2 : gv - g2;
    buf[t] = gv;
  }
}

// fill_refinement_bnd with a remote coarse neighbour (m_ghost_cells.f90:
// 305-311) + sides_rb (:769-861) on the fine rank.
__global__ void __launch_bounds__(256) k_rb_unpack(LevelView L, int iv, const int* items, int n_items,
                                                   const double* recv) {
  const int nc = L.nc, nc2 = nc * nc;
  GRID_STRIDE(t, (long long)n_items * nc2) {
    const int q = (int)(t / nc2), cell = (int)(t % nc2);
    const int it = items[q], b = it / 6, nb = it % 6 + 1;
    const int a = cell % nc + 1, c = cell / nc + 1;
    const bool low = nb & 1;
    const int x1 = low ? 1 : nc, x2 = low ? 2 : nc - 1;
    double* u = boxp(L, iv, b);
    u[off_gh(L, nb, a, c)] = 0.5 * recv[t] + 0.75 * u[off_face_cell(L, nb, x1, a, c)] -
                             0.25 * u[off_face_cell(L, nb, x2, a, c)];
  }
}

// Custom refinement-boundary faces served on the host (omg_set_refinement_bnd,
// the reference's mg%bc(nb,iv)%refinement_bnd, m_ghost_cells.f90:321-325).
// Record q = fine box b, face nb (item b*6+nb-1): the coarse face gc that
// box_gc_for_fine_neighbor gives (:500-577; from the local coarse neighbour,
// or for NB_RBREM the face the refinement-boundary exchange delivered, slot
// rslot[q]) and the box's variable iv in the reference layout (edges and
// corners 0), for the host callback.
__global__ void __launch_bounds__(256) k_rbh_gather(LevelView L, LevelView C, int iv, const RBRec* rb,
                                                    const int* items, const int* rslot, int n,
                                                    const double* rbrecv, double* cgc, double* cc) {
  const int nc = L.nc, nc2 = nc * nc, s = nc + 2;
  const long long per = (long long)s * s * s;
  GRID_STRIDE(t, (long long)n * (nc2 + per)) {
    if (t < (long long)n * nc2) {
      const int q = (int)(t / nc2), cell = (int)(t % nc2);
      const int b = items[q] / 6, nb = items[q] % 6 + 1;
      const int a = cell % nc + 1, c = cell / nc + 1;
      if (rslot[q] >= 0) {
        cgc[t] = rbrecv[(long long)rslot[q] * nc2 + cell];
        continue;
      }
      const RBRec R = rb[L.nba[(long long)b * 6 + nb - 1]];
      const double* cu = boxp(C, iv, R.coarse_idx);
      const int d = (nb + 1) >> 1;
      const int t1 = (d == 1) ? 1 : 0, t2 = (d == 3) ? 1 : 2;
      const int clayer = (nb & 1) ? nc : 1;   // the coarse face toward us
      const int i = (a + 1) >> 1, j = (c + 1) >> 1;
      auto T = [&](int p, int r) { return cu[off_face_cell(C, nb, clayer, R.dix[t1] + p, R.dix[t2] + r)]; };
      const double tc = T(i, j);
      const double g1 = 0.125 * (T(i + 1, j) - T(i - 1, j));
      const double g2 = 0.125 * (T(i, j + 1) - T(i, j - 1));
      double gv = ((a - 1) & 1) ? tc + g1 : tc - g1;
      gv = ((c - 1) & 1) ? gv + g2 : gv - g2;
      cgc[t] = gv;
    } else {
      const long long u = t - (long long)n * nc2;
      const int q = (int)(u / per), r = (int)(u % per);
      const int b = items[q] / 6, i = r % s, j = (r / s) % s, k = r / (s * s);
      const int nbnd = (i == 0 || i == s - 1) + (j == 0 || j == s - 1) + (k == 0 || k == s - 1);
      cc[u] = nbnd >= 2 ? 0.0 : boxp(L, iv, b)[off_cell(L, i, j, k)];
    }
  }
}

// the callback's ghost cells of face nb of every record back into the boxes
__global__ void __launch_bounds__(256) k_rbh_scatter(LevelView L, int iv, const int* items, int n,
                                                     const double* cc) {
  const int nc = L.nc, nc2 = nc * nc, s = nc + 2;
  const long long per = (long long)s * s * s;
  GRID_STRIDE(t, (long long)n * nc2) {
    const int q = (int)(t / nc2), cell = (int)(t % nc2);
    const int b = items[q] / 6, nb = items[q] % 6 + 1;
    const int a = cell % nc + 1, c = cell / nc + 1, g = (nb & 1) ? 0 : nc + 1, d = (nb + 1) >> 1;
    const int i = d == 1 ? g : a, j = d == 1 ? a : (d == 2 ? g : c), k = d == 3 ? g : c;
    boxp(L, iv, b)[off_gh(L, nb, a, c)] = cc[(long long)q * per + i + (long long)s * (j + (long long)s * k)];
  }
}

// ---------------------------------------------------------------------------
// Gauss-Seidel substep over a level, generic box size: one workgroup per box.
// Updates the cells of colour e (i+j+k ≡ e, the cells box_gs_* visits for
// redblack_cntr n with n ≡ e (mod 2), m_laplacian.f90:101-103), then performs
// the ghost fill the reference runs after the substep (smooth_boxes,
// m_multigrid.f90:412-423): colour-e boundary values pushed to same-GPU
// neighbours, physical and refinement-boundary ghosts recomputed, remote
// faces packed for the halo exchange.  Colour e reads only colour 1-e, so
// the in-place update is race-free across boxes.
template <int OP>
__global__ void __launch_bounds__(256) k_gs_sub(LevelView L, double lambda, int e, int colours, LevelView C,
                                                const RBRec* rb, GcBC bc, double* sendbuf) {
  const int nc = L.nc;
  const OpCoef<OP> K(L, lambda);
  for (int b = blockIdx.x; b < L.n; b += gridDim.x) {
    double* u = boxp(L, 1, b);
    const double* f = boxp(L, 2, b);
    for (int q = threadIdx.x; q < L.hv; q += blockDim.x) {
      const int ih = q % L.h, row = q / L.h, j = row % nc + 1, k = row / nc + 1;
      const int i = 2 * ih + 1 + ((1 + j + k + e) & 1);
      if (i > nc) continue;
      const int o = e * L.hv + q;
      const Nbr7 s = load7(L, u, i, j, k);
      if (is_varop(OP))
        u[o] = ags_value<OP>(K, s, load_eps<OP>(L, b, i, j, k), f[o]);
      else
        u[o] = gs_value<OP>(K, s, f[o]);
    }
    __syncthreads();
    if (nc == 1) {
      // (the reference's face order, box1_fill; colours 0: odd box sizes push
      // nothing and a full fill follows, which alone may set the ghosts, since
      // a 1^3 box's physical ghosts read each other)
      if (threadIdx.x == 0 && colours) {
        box1_fill(L, 1, b, C, rb, bc, sendbuf);
      } else if (threadIdx.x == 0) {   // (the remote faces still go out)
        for (int nb = 1; nb <= 6; nb++)
          if (L.nbk[(long long)b * 6 + nb - 1] == NB_REMOTE) face_cell_fill(L, 1, b, nb, 1, 1, 0, C, rb, bc, sendbuf);
      }
    } else {
      for (int p = threadIdx.x; p < 6 * nc * nc; p += blockDim.x) {
        const int nb = p / (nc * nc) + 1, cell = p % (nc * nc);
        face_cell_fill(L, 1, b, nb, cell % nc + 1, cell / nc + 1, colours, C, rb, bc, sendbuf);
      }
    }
    __syncthreads();
  }
}

// Lexicographic Gauss-Seidel (the reference's default mg_smoother_gs), exact
// order: one workgroup per box sweeps hyperplanes i+j+k = d in increasing d;
// within a plane all updates are independent and see planes < d updated and
// planes > d old — the values the i-fastest loop nest reads.
template <int OP>
__global__ void __launch_bounds__(256) k_gs_lex(LevelView L, double lambda) {
  const int nc = L.nc;
  const OpCoef<OP> K(L, lambda);
  for (int b = blockIdx.x; b < L.n; b += gridDim.x) {
    double* u = boxp(L, 1, b);
    const double* f = boxp(L, 2, b);
    for (int d = 3; d <= 3 * nc; d++) {
      for (int p = threadIdx.x; p < nc * nc; p += blockDim.x) {
        const int j = p % nc + 1, k = p / nc + 1, i = d - j - k;
        if (i < 1 || i > nc) continue;
        const int o = off_int(L, i, j, k);
        const Nbr7 s = load7(L, u, i, j, k);
        if (is_varop(OP))
          u[o] = ags_value<OP>(K, s, load_eps<OP>(L, b, i, j, k), f[o]);
        else
          u[o] = gs_value<OP>(K, s, f[o]);
      }
      __syncthreads();
    }
  }
}

// The same sweep with the box in LDS (gs_lex_box, omg_gsrb.h): bit-identical.
template <int OP, int NC>
__global__ void __launch_bounds__(256) k_gs_lex_lds(LevelView L, double lambda) {
  __shared__ double lds[gs_lex_lds<NC>()];
  for (int b = blockIdx.x; b < L.n; b += gridDim.x) gs_lex_box<OP, NC>(L, lambda, b, lds);
}

// Lexicographic GS with one wave per box (64-thread workgroups, so the
// plane-to-plane barrier is free) and the box dense in LDS, (NC+2)^3 with i
// fastest: 46.6 KB for 16^3, so three boxes share a CU.  The stored box
// (colour-split interior + face ghosts, omg_device.h) comes in and the
// interior goes back as whole 16-B rows.  Hyperplanes i+j+k = d in increasing
// d as in gs_lex_box, same operands and gs_value: bit-identical to the
// reference's i-fastest loop.  Lane l owns the lines (j, k) = l + 64 r; rhs of
// its cells is read from L2 GS_PF planes ahead (one wave per box hides no
// latency by itself).
constexpr int kGsPF = 4;
// + one dummy slot per thread: off-plane lanes store there, so the sweep is
// branch-free and the same every plane (the compiler then keeps the rhs
// prefetch in flight instead of draining it at each plane)
template <int NC, int T>
constexpr int gs_wave_lds() { return (NC + 2) * (NC + 2) * (NC + 2) + T; }

// WPS: waves per SIMD the register budget must allow (the LDS-bound
// workgroups per CU x T/64 / 4)
template <int OP, int NC, int T, int WPS>
__global__ void __launch_bounds__(T, WPS) k_gs_lex_wave(LevelView L, double lambda) {
  using TL = Tl<NC>;
  constexpr int S = NC + 2, NL = (NC * NC + T - 1) / T, H = TL::H, HV = TL::HV, FS = TL::FS;
  constexpr int D0 = 3, D1 = 3 * NC, PF = kGsPF, NQ = (TL::NST / 2 + T - 1) / T;
  // planes D0 .. D1 padded to whole groups of PF (the padding planes update nothing)
  constexpr int DP = D0 + ((D1 - D0 + PF) / PF) * PF - 1;
  __shared__ double P[gs_wave_lds<NC, T>()];
  const int tid = threadIdx.x, G = gridDim.x;
  const OpCoef<OP> K(L, lambda);
  // stored slot q -> dense index (edges and corners are neither stored nor read)
  auto dense = [&](int q) {
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
  };
  // per line: j + k, its dense base (c - i) and its row offset in rhs
  int jk[NL], cbase[NL], roff[NL];
#pragma unroll
  for (int r = 0; r < NL; r++) {
    const int p = tid + T * r, j = p % NC + 1, k = p / NC + 1;
    jk[r] = p < NC * NC ? j + k : 1 << 20;   // lanes past the last line never fall in range
    cbase[r] = S * (j + S * k);
    roff[r] = H * ((j - 1) + NC * (k - 1));
  }
  auto rhs_plane = [&](const double* f, int d, double* out) {
#pragma unroll
    for (int r = 0; r < NL; r++) {
      const int i = min(max(d - jk[r], 1), NC);   // off-plane lanes load a valid dummy
      out[r] = f[(d & 1) * HV + ((i - 1) >> 1) + roff[r]];
    }
  };
  // Persistent workgroups: box sequence q = blockIdx.x + G t (G a multiple of
  // 8, so every box of one workgroup sits on its XCD's run, xcd_box).  The
  // next box's stored data and first rhs planes are loaded into registers
  // while this box sweeps.
  // this thread's LDS slots for the scatter (stored slot 2 q2, 2 q2 + 1) and
  // the gather (interior slots), as 16-bit pairs: the same for every box
  constexpr int NG2 = (HV + T - 1) / T;
  unsigned scat[NQ], gath[NG2];
#pragma unroll
  for (int r = 0; r < NQ; r++) {
    const int q2 = min(tid + T * r, TL::NST / 2 - 1);
    scat[r] = (unsigned)dense(2 * q2) | ((unsigned)dense(2 * q2 + 1) << 16);
  }
#pragma unroll
  for (int r = 0; r < NG2; r++) {
    const int q2 = min(tid + T * r, HV - 1);
    gath[r] = (unsigned)dense(2 * q2) | ((unsigned)dense(2 * q2 + 1) << 16);
  }
  double ring[PF][NL], ringn[PF][NL];
  v2d buf[NQ];
  auto issue = [&](int q, double (*rg)[NL]) {
    const int b = xcd_box(q, L.n);
    const double* f = boxp(L, 2, b);
#pragma unroll
    for (int s = 0; s < PF; s++) rhs_plane(f, D0 + s, rg[s]);
    const double* u = boxp(L, 1, b);
#pragma unroll
    for (int r = 0; r < NQ; r++) {
      const int q2 = tid + T * r;
      if (q2 < TL::NST / 2) buf[r] = *reinterpret_cast<const v2d*>(u + 2 * q2);
    }
  };
  int q = blockIdx.x;
  if (q >= L.n) return;
  issue(q, ring);
  for (; q < L.n; q += G) {
    const int b = xcd_box(q, L.n);
    double* __restrict__ u = boxp(L, 1, b);
    const double* __restrict__ f = boxp(L, 2, b);
#pragma unroll
    for (int r = 0; r < NQ; r++) {
      const int q2 = tid + T * r;
      if (q2 < TL::NST / 2) {
        P[scat[r] & 0xffff] = buf[r].x;
        P[scat[r] >> 16] = buf[r].y;
      }
    }
    if (q + G < L.n) issue(q + G, ringn);
    __syncthreads();
#pragma unroll 1
    for (int d0 = D0; d0 <= DP; d0 += PF) {
#pragma unroll
      for (int s = 0; s < PF; s++) {
        const int d = d0 + s;
        // all stencil reads of the plane first, then the updates: the cells of
        // a plane are independent, and a store between them would order every
        // later read behind it
        Nbr7 st[NL];
        int w[NL];
#pragma unroll
        for (int r = 0; r < NL; r++) {
          const int i0 = d - jk[r], i = min(max(i0, 1), NC);
          const int c = cbase[r] + i;
          st[r].c = P[c];
          st[r].xm = P[c - 1];
          st[r].xp = P[c + 1];
          st[r].ym = P[c - S];
          st[r].yp = P[c + S];
          st[r].zm = P[c - S * S];
          st[r].zp = P[c + S * S];
          w[r] = (i0 >= 1 && i0 <= NC) ? c : S * S * S + tid;
        }
        double nv[NL];
#pragma unroll
        for (int r = 0; r < NL; r++) {
          if constexpr (is_varop(OP)) {
            const int i = min(max(d - jk[r], 1), NC), j = (cbase[r] / S) % S, k = cbase[r] / (S * S);
            nv[r] = ags_value<OP>(K, st[r], load_eps<OP>(L, b, i, j, k), ring[s][r]);
          } else {
            nv[r] = gs_value<OP>(K, st[r], ring[s][r]);
          }
        }
#pragma unroll
        for (int r = 0; r < NL; r++) P[w[r]] = nv[r];
        rhs_plane(f, d + PF, ring[s]);   // past the last plane: clamped, unused
        __syncthreads();
      }
    }
#pragma unroll
    for (int r = 0; r < NG2; r++) {
      const int q2 = tid + T * r;
      if (q2 >= HV) break;
      v2d v;
      v.x = P[gath[r] & 0xffff];
      v.y = P[gath[r] >> 16];
      *reinterpret_cast<v2d*>(u + 2 * q2) = v;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PF; s++)
#pragma unroll
      for (int r = 0; r < NL; r++) ring[s][r] = ringn[s][r];
  }
}

// ---------------------------------------------------------------------------
// Lexicographic GS with the box in registers (round 3).  Kernels that keep
// the box in LDS (k_gs_lex_wave: 46.6 KB, three boxes per CU) pay a workgroup
// barrier per hyperplane; their sweep is latency-bound at 34-37 % of HBM.
//
// Here one wave sweeps one 16^3 box.  Lane l owns the four x-lines
// (j, k) = (l % 16 + 1, 4 (l / 16) + r + 1), r = 0..3, and keeps each line's
// 18 cells (interior i = 1..16 and the two x ghosts) in a ring of registers:
// cell i of line (j, k) in slot (i + j + k) mod 18.  Step t updates cell
// i = t - j - k of every line, i.e. the hyperplane i + j + k = t.  In the
// skewed ring every operand of step t sits in a slot that is the same for all
// lanes and lines:
//   xm, and the y-/z-lower neighbours' cell i: slot t - 1 (updated at t - 1),
//   xp, and the y-/z-upper neighbours' cell i: slot t + 1 (not yet updated),
// so the unrolled sweep indexes registers statically.  The y neighbours are
// the lanes beside this one in its 16-lane row (DPP row shifts; the lanes at
// the row ends keep the y ghost, read from LDS, as the shift's old value), the
// z neighbours the lane's own next line or, across lane groups, the lane 16
// away (ds_bpermute), with the z ghosts at the box faces.  No LDS traffic for
// phi and no barrier per step: the box passes through LDS only to be rotated
// into and out of the ring (18 KB per box, so 8 boxes share a CU).  rhs comes
// from a copy in the ring's order (k_rhs_reg, rebuilt after every write of
// the level's rhs): the step-t values of all 256 lines are one
// contiguous 2 KB run, prefetched PF steps ahead.  Every cell is updated
// after its lower neighbours and before its upper ones, with the same
// operands and gs_value as the reference's i-fastest loop: bit-identical.
constexpr int kLexRing = 18;                       // interior + 2 x ghosts per line
constexpr int kLexGPad = 16;                       // slack around each y/z ghost face in LDS
constexpr int kLexGFace = 256 + 2 * kLexGPad;

// value of the lane one below / above in this lane's 16-lane row; the first /
// last lane of the row keeps `old` (row_shr:1 / row_shl:1, bound_ctrl off)
__device__ __forceinline__ double dpp_row_prev(double v, double old) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x111, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x111, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
// the value of the lane two further on in this lane's 16-lane row (row_shl:2;
// the last two lanes of the row get their own value, unused)
__device__ __forceinline__ double dpp_row_shl2(double v) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), 0x102, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), 0x102, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_row_next(double v, double old) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x101, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x101, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// z crossings between lane groups by the gfx950 row swaps: the 16-lane rows
// hold the lane groups kq = 0, 1, 3, 2, so that every crossing (kq 0-1, 1-2,
// 2-3) is a v_permlane16_swap or v_permlane32_swap partner (against
// ds_bpermute: 837 -> 827 us per 512^3 sweep, profiles/r03)
// lane group of 16-lane row x, and the row of lane group x (an involution)
__device__ __forceinline__ int lex_grp(int x) { return x >= 2 ? 5 - x : x; }
// the value of v in the lane of the partner row: x16 swaps rows 0-1, 2-3,
// x32 rows 0-2, 1-3
__device__ __forceinline__ double row_partner(double v, bool x32) {
  // both swaps in every lane (the partner lanes must be active), then select
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const int row = threadIdx.x >> 4;
  const auto a32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const auto a16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double p32 = row >= 2 ? __hiloint2double((int)b32[0], (int)a32[0]) : __hiloint2double((int)b32[1], (int)a32[1]);
  const double p16 = (row & 1) ? __hiloint2double((int)b16[0], (int)a16[0]) : __hiloint2double((int)b16[1], (int)a16[1]);
  return x32 ? p32 : p16;
}

// rhs of every 16^3 box in ring order:
// rl[b*4096 + ((i+j+k+b) & 15)*256 + (r/2)*128 + 2*l + r%2]
// for cell (i, j, k) of lane l = (j-1) + 16*((k-1)/4), line r = (k-1) % 4;
// the step blocks rotated by the box index, so that boxes at the same step
// (32 KB apart) spread over the memory channels;
// a bijection (each line has one cell per value of (i+j+k) mod 16)
__global__ void __launch_bounds__(256) k_rhs_reg(LevelView L, double* __restrict__ rl) {
  using TL = Tl<16>;
  __shared__ double F[4096];
  const int b = blockIdx.x;
  const v2d* f = reinterpret_cast<const v2d*>(boxp(L, 2, b));
  for (int q = threadIdx.x; q < 2048; q += blockDim.x) reinterpret_cast<v2d*>(F)[q] = f[q];
  __syncthreads();
  double* o = rl + (long long)b * 4096;
  for (int d = threadIdx.x; d < 4096; d += blockDim.x) {
    // lines 2 rp and 2 rp + 1 of lane l side by side: one 16-B load per lane
    // and line pair
    const int s = d >> 8, r = 2 * ((d >> 7) & 1) + (d & 1), l = (d >> 1) & 63;
    const int j = (l & 15) + 1, k = 4 * lex_grp(l >> 4) + r + 1, i = ((s - j - k - 1) & 15) + 1;
    o[(((s + b) & 15) << 8) | (d & 255)] = F[TL::oint(i, j, k)];
  }
}

// phi streams (rotation in and out) non-temporal, the rhs copy with the
// default policy (939 -> 833 us per 512^3 sweep against non-temporal rhs
// loads, profiles/r03); two waves per SIMD (234 VGPRs)
// DBL: two ghost-face sets (GhostSets, omg_kernels.h): the ghosts come from
// gs.in (the physical ones formed here from the box's own boundary cells when
// gs.phys_load), and the new boundary layers go to the same-GPU neighbours'
// ghosts in gs.out instead of a fill pass after the sweep.
template <int OP, int PF, bool DBL>
__global__ void __launch_bounds__(64, 2) k_gs_lex_reg(LevelView L, double lambda, const double* __restrict__ rl,
                                                                 double* __restrict__ xl, GhostSets gs, GcBC bc) {
  using TL = Tl<16>;
  constexpr int NC = 16, H = 8, HV = 2048, FH = 128, FS = 256, R = kLexRing, T0 = 3, T1 = 3 * NC;
  static_assert(R % PF == 0, "the rhs ring index must repeat with the register ring");
  // stage rows of 65 doubles: the four lanes that scatter one row's cells
  // into different slots then hit different banks
  constexpr int SR = 65;
  __shared__ double stage[R * SR];          // one line of every lane, slot-major
  __shared__ double G[4 * kLexGFace];       // y/z ghost faces, plain [c][a] with slack
  const int l = threadIdx.x, kq = lex_grp(l >> 4), j = (l & 15) + 1;
  const int b = xcd_box(blockIdx.x, gridDim.x, L.rev);
  double* __restrict__ u = boxp(L, 1, b);
  const double* __restrict__ rb = rl + (long long)b * (NC * NC * NC);
  const OpCoef<OP> K(L, lambda);
  FaceTopo T{};
  if (DBL) T = load_topo(L, b);
  // this box's ghost faces (face nb at gb + (nb-1)*FS, the stored layout)
  const double* __restrict__ gb = DBL ? gs.in + (long long)b * gs.in_stride : u + 2 * HV;
  const bool pl = DBL && gs.phys_load;
  // physical ghost (a, c) of face nb (bc_to_gc) from the boundary cells x1, x2
  auto phys = [&](int nb, int a, int c, double x1, double x2) {
    return phys_ghost(L, bc, b, (long long)b * 6 + nb - 1, nb, T.phys_code(nb - 1), a, c, TL::ogh(nb, a, c), x1, x2);
  };

  // y/z ghost faces (nb = 3..6: j = 0, j = 17, k = 0, k = 17; tangential
  // (a, c) = (i, k) or (i, j)) into G[f][c-1][a-1]
  {
    const double* gf = gb + 2 * FS;
#pragma unroll
    for (int n = 0; n < 8; n++) {
      const int q = l + 64 * n;                      // double pair of faces 3..6
      const v2d x = ld_nt(gf + 2 * q);
      const int f = q >> 7, r1 = (2 * q) & (FS - 1);
      const int e = r1 >= FH, rr = r1 - e * FH, ah = rr % H, c = rr / H + 1;
      const int g = (f & 1) ? NC + 1 : 0;            // f = nb - 3: even f is a low face
      const int a = 2 * ah + 1 + ((1 + g + c + e) & 1);
      double* gp = G + f * kLexGFace + kLexGPad + NC * (c - 1) + (a - 1);
      gp[0] = x.x;
      gp[2] = x.y;
    }
  }

  // the ring: interior planes k = 4 kq' + r + 1 (both colours) and the x
  // ghosts of line r go through `stage` in slot-major order
  double ring[4][R];
  const int jr = (l >> 2) + 1, ihr = 2 * (l & 3);    // row / first colour index of this lane's loads
#pragma unroll
  for (int r = 0; r < 4; r++) {
    v2d buf[8];
#pragma unroll
    for (int n = 0; n < 8; n++) {
      const int k = 4 * (n >> 1) + r + 1, e = n & 1;
      const double* src = u + e * HV + FH * (k - 1) + 2 * l;
      buf[n] = ld_nt(src);
    }
    const int kr = 4 * kq + r + 1;
    const double gx0 = gb[((j + kr) & 1) * FH + ((j - 1) >> 1) + H * (kr - 1)];
    const double gx1 = gb[FS + ((NC + 1 + j + kr) & 1) * FH + ((j - 1) >> 1) + H * (kr - 1)];
    __syncthreads();                                 // the previous line's reads of stage are done
#pragma unroll
    for (int n = 0; n < 8; n++) {
      const int kq2 = n >> 1, k = 4 * kq2 + r + 1, e = n & 1;
      const int i = 2 * ihr + 1 + ((1 + jr + k + e) & 1);
      const int ln = (jr - 1) + 16 * lex_grp(kq2);
      stage[((i + jr + k) % R) * SR + ln] = buf[n].x;
      stage[((i + 2 + jr + k) % R) * SR + ln] = buf[n].y;
    }
    stage[((j + kr) % R) * SR + l] = gx0;
    stage[((NC + 1 + j + kr) % R) * SR + l] = gx1;
    __syncthreads();
    if (pl) {
      // physical ghosts from the boundary cells in stage: x faces (this
      // lane's own line), y faces (the lines of the j = 1, 2 / 16, 15 lanes),
      // z faces (planes k = 1, 2 / 16, 15 arrive in lines 0, 1 / 3, 2 of
      // groups 0 / 3: the first layer is parked in G until the second comes)
      if (T.kind(0) == NB_PHYS)
        stage[((j + kr) % R) * SR + l] =
            phys(1, j, kr, stage[((1 + j + kr) % R) * SR + l], stage[((2 + j + kr) % R) * SR + l]);
      if (T.kind(1) == NB_PHYS)
        stage[((NC + 1 + j + kr) % R) * SR + l] =
            phys(2, j, kr, stage[((NC + j + kr) % R) * SR + l], stage[((NC - 1 + j + kr) % R) * SR + l]);
      const int a = (l & 15) + 1, gq = l >> 4, kg = 4 * gq + r + 1, lg = 16 * lex_grp(gq);
      if (T.kind(2) == NB_PHYS)
        G[kLexGPad + NC * (kg - 1) + (a - 1)] =
            phys(3, a, kg, stage[((a + 1 + kg) % R) * SR + lg], stage[((a + 2 + kg) % R) * SR + lg + 1]);
      if (T.kind(3) == NB_PHYS)
        G[kLexGFace + kLexGPad + NC * (kg - 1) + (a - 1)] =
            phys(4, a, kg, stage[((a + NC + kg) % R) * SR + lg + 15], stage[((a + NC - 1 + kg) % R) * SR + lg + 14]);
#pragma unroll
      for (int ii = 0; ii < 4; ii++) {
        const int i = 4 * (l >> 4) + ii + 1;   // (i, j) of the z faces
        double* gz0 = G + 2 * kLexGFace + kLexGPad + NC * (j - 1) + (i - 1);
        double* gz1 = G + 3 * kLexGFace + kLexGPad + NC * (j - 1) + (i - 1);
        const int l3 = (j - 1) + 16 * lex_grp(3);
        if (T.kind(4) == NB_PHYS) {
          if (r == 0) *gz0 = stage[((i + j + 1) % R) * SR + (j - 1)];
          if (r == 1) *gz0 = phys(5, i, j, *gz0, stage[((i + j + 2) % R) * SR + (j - 1)]);
        }
        if (T.kind(5) == NB_PHYS) {
          if (r == 2) *gz1 = stage[((i + j + NC - 1) % R) * SR + l3];
          if (r == 3) *gz1 = phys(6, i, j, stage[((i + j + NC) % R) * SR + l3], *gz1);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < R; s++) ring[r][s] = stage[s * SR + l];
  }
  if (pl) __syncthreads();   // the physical y/z ghosts in G

  // per line: j + k; G index of the y ghost at step 0 (lanes of the low half
  // of the row read face j = 0 as lane j = 1 needs it, the others face j = 17
  // as lane j = 16 needs it; the slack keeps every step's index inside G)
  const int jk0 = j + 4 * kq + 1;                   // line r: jk0 + r
  const int gy0 = (j <= 8 ? kLexGPad - 18 : kLexGFace + kLexGPad - 33) + 15 * (4 * kq + 1);   // line r: + 15 r
  // z ghosts: lanes of group 0 (line 0, k = 1) read face k = 0, group 3
  // (line 3, k = 16) face k = 17
  const int gz = kq < 2 ? 2 * kLexGFace + kLexGPad + 15 * j - 18 : 3 * kLexGFace + kLexGPad + 15 * j - 33;

  double rf[PF][4];
  // the four lines' rhs of step t: two 16-B loads
  auto ld_rhs = [&](int t, double* out) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const v2d* p = reinterpret_cast<const v2d*>(rb + ((t + b) & 15) * 256 + h * 128 + 2 * l);
      const v2d x = *p;
      out[2 * h] = x.x;
      out[2 * h + 1] = x.y;
    }
  };
#pragma unroll
  for (int p = 0; p < PF; p++) ld_rhs(T0 + p, rf[(T0 + p) % PF]);

#pragma unroll 1
  for (int m = 0; m < 3; m++) {
#pragma unroll
    for (int s = 0; s < R; s++) {
      const int t = R * m + s;
      if (t < T0 || t > T1) continue;                 // wave-uniform
      const int sm = (s + R - 1) % R, sp = (s + 1) % R;
      double gv[4];
#pragma unroll
      for (int r = 0; r < 4; r++) gv[r] = G[gy0 + 15 * r + t];
      const double gzv = G[gz + t];
      // z crossings: group kq takes line 3 of group kq - 1 and line 0 of
      // group kq + 1; pairs 0-1 and 2-3 are x16 partners, 1-2 x32 partners
      const double zlo_n = row_partner(ring[3][sm], kq == 2);
      const double zhi_n = row_partner(ring[0][sp], kq == 1);
      const double zlo = kq == 0 ? gzv : zlo_n;
      const double zhi = kq == 3 ? gzv : zhi_n;
      double nv[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        Nbr7 st;
        st.c = ring[r][s];
        st.xm = ring[r][sm];
        st.xp = ring[r][sp];
        st.ym = dpp_row_prev(ring[r][sm], gv[r]);
        st.yp = dpp_row_next(ring[r][sp], gv[r]);
        st.zm = r > 0 ? ring[r - 1][sm] : zlo;
        st.zp = r < 3 ? ring[r + 1][sp] : zhi;
        nv[r] = gs_value<OP>(K, st, rf[s % PF][r]);
      }
#pragma unroll
      for (int r = 0; r < 4; r++)
        if ((unsigned)(t - jk0 - r - 1) < (unsigned)NC) ring[r][s] = nv[r];
      // unconditional (past the last step it reads this box's copy again,
      // unused): a conditional load would be waited for at once
      ld_rhs(t + PF, rf[s % PF]);
      // keep the scheduler from interleaving steps (that raises the register
      // pressure past the ring's budget)
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // the interior back, through stage in the stored order (the box pointer
  // made opaque: otherwise the store addresses are shared with the loads'
  // and held across the sweep, which spills)
  double* ub = u;
  asm volatile("" : "+s"(ub));
#pragma unroll
  for (int r = 0; r < 4; r++) {
    __syncthreads();
#pragma unroll
    for (int s = 0; s < R; s++) stage[s * SR + l] = ring[r][s];
    __syncthreads();
    if (DBL) {
      // the new boundary layers of line r into the same-GPU neighbours'
      // ghosts of the other set: x faces from this lane's line, y faces from
      // the j = 1 / 16 lanes, z faces from planes k = 1 (line 0, group 0)
      // and k = 16 (line 3, group 3)
      // Every push is a 16-B pair: the two same-colour cells a and a+2 of a
      // face row are adjacent in the stored face (index (a-1)>>1).  Along a
      // 16-lane row the partner is the lane two further on (DPP row_shl:2),
      // and the lanes whose index is even store the pair.
      const int kr = 4 * kq + r + 1;
      auto push2 = [&](int f, int a, int c, double v0, double v1) {   // toward face f+1's neighbour
        const int nbo = (f & 1) ? f : f + 2;                           // the neighbour's opposite face
        st_v2(gs.out + (long long)T.arg(f) * gs.out_stride + TL::ogh(nbo, a, c) - 2 * HV, v0, v1);
      };
      const bool pair_lane = !(((l & 15) >> 1) & 1);   // index ((l & 15)) >> 1 even
      if (T.kind(0) == NB_LOCAL) {
        const double v = stage[((1 + j + kr) % R) * SR + l], w = dpp_row_shl2(v);
        if (pair_lane) push2(0, j, kr, v, w);
      }
      if (T.kind(1) == NB_LOCAL) {
        const double v = stage[((NC + j + kr) % R) * SR + l], w = dpp_row_shl2(v);
        if (pair_lane) push2(1, j, kr, v, w);
      }
      const int a = (l & 15) + 1, gq = l >> 4, kg = 4 * gq + r + 1, lg = 16 * lex_grp(gq);
      if (T.kind(2) == NB_LOCAL) {
        const double v = stage[((a + 1 + kg) % R) * SR + lg], w = dpp_row_shl2(v);
        if (pair_lane) push2(2, a, kg, v, w);
      }
      if (T.kind(3) == NB_LOCAL) {
        const double v = stage[((a + NC + kg) % R) * SR + lg + 15], w = dpp_row_shl2(v);
        if (pair_lane) push2(3, a, kg, v, w);
      }
      if ((r == 0 && T.kind(4) == NB_LOCAL) || (r == 3 && T.kind(5) == NB_LOCAL)) {
        // a lane's four cells i = 4q+1 .. 4q+4: the two of each colour are
        // i and i+2, one pair per colour
        const int ln = (j - 1) + (r == 0 ? 0 : 16 * lex_grp(3)), k0 = r == 0 ? 1 : NC;
#pragma unroll
        for (int ii = 0; ii < 2; ii++) {
          const int i = 4 * (l >> 4) + ii + 1;
          push2(r == 0 ? 4 : 5, i, j, stage[((i + j + k0) % R) * SR + ln], stage[((i + 2 + j + k0) % R) * SR + ln]);
        }
      }
    }
    // the new x boundary layers (i = 1, i = 16) of line r, for the ghost
    // fill that follows (k_fill_tile_xl): xl[b][face][(j-1) + 16 (k-1)]
    if (xl && !DBL) {
      const int kr = 4 * kq + r + 1;
      double* xo = xl + (long long)b * 512 + (j - 1) + NC * (kr - 1);
      xo[0] = stage[((1 + j + kr) % R) * SR + l];
      xo[256] = stage[((NC + j + kr) % R) * SR + l];
    }
#pragma unroll
    for (int n = 0; n < 8; n++) {
      const int kq2 = n >> 1, k = 4 * kq2 + r + 1, e = n & 1;
      const int i = 2 * ihr + 1 + ((1 + jr + k + e) & 1);
      const int ln = (jr - 1) + 16 * lex_grp(kq2);
      double* dst = ub + e * HV + FH * (k - 1) + 2 * l;
      const double x0 = stage[((i + jr + k) % R) * SR + ln], x1 = stage[((i + 2 + jr + k) % R) * SR + ln];
      st_nt(dst, x0, x1);
    }
  }
}

template <int OP>
__device__ __forceinline__ double apply_op(const LevelView& L, const OpCoef<OP>& K, int b, int i, int j,
                                           int k) {
  const Nbr7 s = load7(L, boxp(L, 1, b), i, j, k);
  if (is_varop(OP)) return aop_value<OP>(K, s, load_eps<OP>(L, b, i, j, k));
  return op_value<OP>(K, s);
}

// Operator into variable i_out (mg_apply_op / box_op), interior cells in
// storage order.
template <int OP>
__global__ void __launch_bounds__(256) k_box_op(LevelView L, double lambda, int i_out) {
  const OpCoef<OP> K(L, lambda);
  const long long per = 2LL * L.hv;
  GRID_STRIDE(t, per * L.n) {
    const int b = (int)(t / per), o = (int)(t % per);
    int i, j, k;
    if (!cell_of(L, o, i, j, k)) continue;
    boxp(L, i_out, b)[o] = apply_op<OP>(L, K, b, i, j, k);
  }
}

// residual_box (m_multigrid.f90:426-436): res = rhs - L(phi); optionally the
// max |res| of the level (max_residual_lvl :296-311, exact in any order).
template <int OP>
__global__ void __launch_bounds__(256) k_residual(LevelView L, double lambda, unsigned long long* maxbits) {
  const OpCoef<OP> K(L, lambda);
  const long long per = 2LL * L.hv;
  double mx = 0.0;
  GRID_STRIDE(t, per * L.n) {
    const int b = (int)(t / per), o = (int)(t % per);
    int i, j, k;
    if (!cell_of(L, o, i, j, k)) continue;
    const double res = boxp(L, 2, b)[o] - apply_op<OP>(L, K, b, i, j, k);
    boxp(L, 4, b)[o] = res;
    mx = amax(mx, fabs(res));
  }
  if (maxbits) launch_max<256>(maxbits, mx);
}

// Folds the kMaxSlots slots of launch_max into *out (into max(*out, .) when
// accumulating over levels) and zeroes them.
__global__ void __launch_bounds__(kMaxSlots) k_max_fold(unsigned long long* slots, unsigned long long* out,
                                                        int accumulate) {
  unsigned long long* s = slots + threadIdx.x * kMaxSlotStride;
  double mx = __longlong_as_double((long long)*s);
  *s = 0ull;
  for (int off = 32; off > 0; off >>= 1) mx = amax(mx, __shfl_down(mx, off, 64));
  __shared__ double wmax[kMaxSlots / 64];
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kMaxSlots / 64; w++) mx = amax(mx, wmax[w]);
    if (accumulate) mx = amax(mx, __longlong_as_double((long long)*out));
    *out = (unsigned long long)__double_as_longlong(mx);
  }
}

void launch_max_fold(unsigned long long* slots, unsigned long long* out, bool accumulate, hipStream_t st) {
  k_max_fold<<<1, kMaxSlots, 0, st>>>(slots, out, accumulate ? 1 : 0);
}

// ---------------------------------------------------------------------------
// Restriction (restrict_onto, m_restrict.f90:165-214): coarse cell =
// 0.125 * SUM(2x2x2 fine cells) accumulated column-major from +0.0.
__device__ __forceinline__ double restrict_cell(const LevelView& F, const double* fu, int i, int j, int k) {
  double acc = 0.0;
#pragma unroll
  for (int kk = 0; kk < 2; kk++)
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int ii = 0; ii < 2; ii++) acc += fu[off_int(F, 2 * i - 1 + ii, 2 * j - 1 + jj, 2 * k - 1 + kk)];
  return 0.125 * acc;
}

__global__ void __launch_bounds__(256) k_restrict(LevelView F, LevelView Cv, int iv, const int* pairs,
                                                  int n_pairs, const int* parent_local, const int* dixp) {
  const int hnc = F.nc / 2;
  const long long per = (long long)hnc * hnc * hnc;
  GRID_STRIDE(t, per * n_pairs) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int cb = pairs[q], pb = parent_local[cb], dp = dixp[cb];
    const int i = r % hnc + 1, j = (r / hnc) % hnc + 1, k = r / (hnc * hnc) + 1;
    const double v = restrict_cell(F, boxp(F, iv, cb), i, j, k);
    boxp(Cv, iv, pb)[off_int(Cv, (dp & 1023) + i, ((dp >> 10) & 1023) + j, (dp >> 20) + k)] = v;
  }
}

// restrict_set_buffer (m_restrict.f90:116-163): restricted child into buffer.
__global__ void __launch_bounds__(256) k_restrict_pack(LevelView F, int iv, const int* items, int n_items,
                                                       double* buf) {
  const int hnc = F.nc / 2;
  const long long per = (long long)hnc * hnc * hnc;
  GRID_STRIDE(t, per * n_items) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int i = r % hnc + 1, j = (r / hnc) % hnc + 1, k = r / (hnc * hnc) + 1;
    buf[t] = restrict_cell(F, boxp(F, iv, items[q]), i, j, k);
  }
}

// Whole stored boxes of one variable (replicated coarse levels: the host's
// boxes go to every peer after an upload).
__global__ void __launch_bounds__(256) k_box_pack(LevelView L, int iv, const int* items, int n_items,
                                                  double* buf) {
  GRID_STRIDE(t, L.stride * n_items) {
    const int q = (int)(t / L.stride);
    buf[t] = boxp(L, iv, items[q])[t % L.stride];
  }
}
__global__ void __launch_bounds__(256) k_box_unpack(LevelView L, int iv, const int* items, int n_items,
                                                    const double* buf) {
  GRID_STRIDE(t, L.stride * n_items) {
    const int q = (int)(t / L.stride);
    boxp(L, iv, items[q])[t % L.stride] = buf[t];
  }
}

// restrict_onto's remote branch: items = (parent local idx, packed dix) pairs.
__global__ void __launch_bounds__(256) k_restrict_unpack(LevelView Cv, int iv, const int* items,
                                                         int n_items, int hnc, const double* buf) {
  const long long per = (long long)hnc * hnc * hnc;
  GRID_STRIDE(t, per * n_items) {
    const int q = (int)(t / per), r = (int)(t % per);
    const int pb = items[2 * q], dp = items[2 * q + 1];
    const int i = r % hnc + 1, j = (r / hnc) % hnc + 1, k = r / (hnc * hnc) + 1;
    boxp(Cv, iv, pb)[off_int(Cv, (dp & 1023) + i, ((dp >> 10) & 1023) + j, (dp >> 20) + k)] = buf[t];
  }
}

// ---------------------------------------------------------------------------
// update_coarse's parent loop (m_multigrid.f90:369-383): rhs = L(phi) + res
// on the interior, old = phi on the whole (stored) box.
template <int OP>
__global__ void __launch_bounds__(256) k_coarse_rhs(LevelView Cv, double lambda, const int* parents,
                                                    int n_par) {
  const OpCoef<OP> K(Cv, lambda);
  const long long per = 2LL * Cv.hv + 6LL * Cv.fs;
  GRID_STRIDE(t, per * n_par) {
    const int b = parents[t / per], o = (int)(t % per);
    int i, j, k;
    if (!cell_of(Cv, o, i, j, k)) continue;
    if (o < 2 * Cv.hv) boxp(Cv, 2, b)[o] = apply_op<OP>(Cv, K, b, i, j, k) + boxp(Cv, 4, b)[o];
    boxp(Cv, 3, b)[o] = boxp(Cv, 1, b)[o];
  }
}

// correct_children's parent loop (m_multigrid.f90:392-399): res = phi - old.
__global__ void __launch_bounds__(256) k_sub_parents(LevelView Cv, const int* parents, int n_par) {
  const long long per = 2LL * Cv.hv + 6LL * Cv.fs;
  GRID_STRIDE(t, per * n_par) {
    const int b = parents[t / per], o = (int)(t % per);
    int i, j, k;
    if (!cell_of(Cv, o, i, j, k)) continue;
    boxp(Cv, 4, b)[o] = boxp(Cv, 1, b)[o] - boxp(Cv, 3, b)[o];
  }
}

// mg_prolong_sparse (m_prolong.f90:159-240) value at fine cell (fi,fj,fk).
__device__ __forceinline__ double prolong_cell(const LevelView& C, const double* cu, int dx, int dy, int dz,
                                               int fi, int fj, int fk) {
  const int ic = ((fi + 1) >> 1) + dx, jc = ((fj + 1) >> 1) + dy, kc = ((fk + 1) >> 1) + dz;
  const double f0 = 0.25 * cu[off_int(C, ic, jc, kc)];
  const double fx = 0.25 * cu[off_cell(C, (fi & 1) ? ic - 1 : ic + 1, jc, kc)];
  const double fy = 0.25 * cu[off_cell(C, ic, (fj & 1) ? jc - 1 : jc + 1, kc)];
  const double fz = 0.25 * cu[off_cell(C, ic, jc, (fk & 1) ? kc - 1 : kc + 1)];
  return f0 + fx + fy + fz;
}

// mg_prolong + prolong_onto (m_prolong.f90:51-85,124-156) for local parents.
__global__ void __launch_bounds__(256) k_prolong(LevelView Cv, LevelView F, int iv, int iv_to, int add,
                                                 const int* pairs, int n_pairs, const int* parent_local,
                                                 const int* dixp) {
  const long long per = 2LL * F.hv;
  GRID_STRIDE(t, per * n_pairs) {
    const int q = (int)(t / per), o = (int)(t % per);
    int i, j, k;
    if (!cell_of(F, o, i, j, k)) continue;
    const int fb = pairs[q], pb = parent_local[fb], dp = dixp[fb];
    const double v = prolong_cell(Cv, boxp(Cv, iv, pb), dp & 1023, (dp >> 10) & 1023, dp >> 20, i, j, k);
    double* dst = boxp(F, iv_to, fb) + o;
    *dst = add ? *dst + v : v;
  }
}

// prolong_set_buffer (m_prolong.f90:91-121): items = (parent idx, packed dix);
// the fine values travel in the fine box's storage order.
__global__ void __launch_bounds__(256) k_prolong_pack(LevelView Cv, LevelView F, int iv, const int* items,
                                                      int n_items, double* buf) {
  const long long per = 2LL * F.hv;
  GRID_STRIDE(t, per * n_items) {
    const int q = (int)(t / per), o = (int)(t % per);
    int i, j, k;
    if (!cell_of(F, o, i, j, k)) continue;
    const int pb = items[2 * q], dp = items[2 * q + 1];
    buf[t] = prolong_cell(Cv, boxp(Cv, iv, pb), dp & 1023, (dp >> 10) & 1023, dp >> 20, i, j, k);
  }
}

__global__ void __launch_bounds__(256) k_prolong_unpack(LevelView F, int iv_to, int add, const int* items,
                                                        int n_items, const double* buf) {
  const long long per = 2LL * F.hv;
  GRID_STRIDE(t, per * n_items) {
    const int q = (int)(t / per), o = (int)(t % per);
    int i, j, k;
    if (!cell_of(F, o, i, j, k)) continue;
    double* dst = boxp(F, iv_to, items[q]) + o;
    *dst = add ? *dst + buf[t] : buf[t];
  }
}

// subtract_mean's update (m_multigrid.f90:262-275): interior, or every stored cell.
__global__ void __launch_bounds__(256) k_subtract(LevelView L, int iv, const double* mean, int ghosts) {
  const double m = *mean;
  const long long per = ghosts ? 2LL * L.hv + 6LL * L.fs : 2LL * L.hv;
  GRID_STRIDE(t, per * L.n) {
    const int b = (int)(t / per), o = (int)(t % per);
    int i, j, k;
    if (!cell_of(L, o, i, j, k)) continue;
    double* u = boxp(L, iv, b) + o;
    *u = *u - m;
  }
}

// Even box sizes: every slot of the stored range is a cell, so the variable
// streams as contiguous double2 per box.
typedef double v2d_t __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) k_subtract_even(LevelView L, int iv, const double* mean, int per2) {
  const double m = *mean;
  GRID_STRIDE(t, (long long)per2 * L.n) {
    const int b = (int)(t / per2), o = (int)(t % per2);
    v2d_t* u = reinterpret_cast<v2d_t*>(boxp(L, iv, b)) + o;
    v2d_t x = __builtin_nontemporal_load(u);
    x.x = x.x - m;
    x.y = x.y - m;
    __builtin_nontemporal_store(x, u);
  }
}

// m_diffusion's set_rhs (src/m_diffusion.f90:144-159): rhs = f1*phi + f2*rhs
// on the interior of the given leaves, one thread per cell.
__global__ void __launch_bounds__(256) k_set_rhs(LevelView L, const int* __restrict__ leaves, int n_leaves,
                                                 double f1, double f2) {
  const long long per = 2LL * L.hv;
  GRID_STRIDE(t, per * n_leaves) {
    const int b = leaves[t / per], o = (int)(t % per);
    int i, j, k;
    if (!cell_of(L, o, i, j, k)) continue;
    const double u = boxp(L, 1, b)[o];
    double* f = boxp(L, 2, b) + o;
    *f = f1 * u + f2 * *f;
  }
}

// Whole-box copy / zero of one variable (FMG's old = phi and phi = 0).
__global__ void __launch_bounds__(256) k_copy_var(LevelView L, int src, int dst) {
  GRID_STRIDE(t, (long long)L.n * L.stride) {
    const int b = (int)(t / L.stride);
    const long long o = t % L.stride;
    boxp(L, dst, b)[o] = src > 0 ? boxp(L, src, b)[o] : 0.0;
  }
}

// Reference layout cc(0:nc+1,0:nc+1,0:nc+1) <-> device layout (edges and
// corners are not stored; they read back as 0).
__global__ void __launch_bounds__(256) k_from_ref(LevelView L, int iv, const double* ref) {
  const int s = L.nc + 2;
  const long long per = (long long)s * s * s;
  GRID_STRIDE(t, per * L.n) {
    const int b = (int)(t / per);
    const int r = (int)(t % per), i = r % s, j = (r / s) % s, k = r / (s * s);
    const int nbnd = (i == 0 || i == s - 1) + (j == 0 || j == s - 1) + (k == 0 || k == s - 1);
    if (nbnd >= 2) continue;
    boxp(L, iv, b)[off_cell(L, i, j, k)] = ref[t];
  }
}

// (unstored: what the edge and corner cells read back as, 0 or, in debug
// mode, a signalling NaN)
__global__ void __launch_bounds__(256) k_to_ref(LevelView L, int iv, double* ref, double unstored) {
  const int s = L.nc + 2;
  const long long per = (long long)s * s * s;
  GRID_STRIDE(t, per * L.n) {
    const int b = (int)(t / per);
    const int r = (int)(t % per), i = r % s, j = (r / s) % s, k = r / (s * s);
    const int nbnd = (i == 0 || i == s - 1) + (j == 0 || j == s - 1) + (k == 0 || k == s - 1);
    ref[t] = nbnd >= 2 ? unstored : boxp(L, iv, b)[off_cell(L, i, j, k)];
  }
}

// Debug mode (OMG_DEBUG): every ghost face slot of every variable set to
// `poison` (a signalling NaN), the reference's DEBUG=1 -finit-real=snan for
// the cells that only a ghost fill, an upload or a store may define
// (makerules.make:13-17); the interior keeps the reference's zeros
// (m_allocate_storage.f90:75-76).
__global__ void __launch_bounds__(256) k_poison_ghosts(LevelView L, int n_vars, double poison) {
  const long long per = 6LL * L.fs;
  GRID_STRIDE(t, per * L.n * n_vars) {
    const long long q = t / per;
    const int b = (int)(q % L.n), iv = (int)(q / L.n) + 1;
    boxp(L, iv, b)[2LL * L.hv + t % per] = poison;
  }
}

void launch_poison_ghosts(const LevelView& L, int n_vars, double poison, hipStream_t st) {
  const long long work = 6LL * L.fs * L.n * n_vars;
  if (work == 0) return;
  k_poison_ghosts<<<grid_for(work), 256, 0, st>>>(L, n_vars, poison);
}

// mg_phi_bc_store_lvl (m_ghost_cells.f90:80-117): bc values -> rhs ghosts,
// bc type -> neighbour code.
__global__ void __launch_bounds__(256) k_phi_bc_store(LevelView L, GcBC bc, int* nba) {
  const int nc = L.nc, nc2 = nc * nc;
  GRID_STRIDE(t, (long long)L.n * 6 * nc2) {
    const int cell = (int)(t % nc2), f = (int)(t / nc2);
    if (L.nbk[f] != NB_PHYS) continue;
    const int b = f / 6, nb = f % 6 + 1, a = cell % nc + 1, c = cell / nc + 1;
    double bv;
    int type;
    if (bc.face_off && bc.face_off[f] >= 0) {
      bv = bc.face_data[bc.face_off[f] + (a - 1) + (long long)nc * (c - 1)];
      type = bc.face_type[f];
    } else {
      bv = bc.value[nb - 1];
      type = bc.type[nb - 1];
    }
    boxp(L, 2, b)[off_gh(L, nb, a, c)] = bv;
    if (cell == 0) nba[f] = type;
  }
}

void launch_phi_bc_store(const LevelView& L, const GcBC& bc, int* nba, hipStream_t st) {
  const long long work = (long long)L.n * 6 * L.nc * L.nc;
  if (work == 0) return;
  k_phi_bc_store<<<grid_for(work), 256, 0, st>>>(L, bc, nba);
}

// ---------------------------------------------------------------------------
// launchers
#define OP_SWITCH(op, KERNEL, GRID, BLOCK, ST, ...)                              \
  switch (op) {                                                                  \
    case OP_HELM: KERNEL<OP_HELM><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__); break;   \
    case OP_AHELM: KERNEL<OP_AHELM><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__); break; \
    case OP_VLPL: KERNEL<OP_VLPL><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__); break;   \
    case OP_VHELM: KERNEL<OP_VHELM><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__); break; \
    default: KERNEL<OP_LPL><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__); break;         \
  }

void launch_gs_sub(const LevelView& L, int op, double lambda, int e, int colours, const LevelView& C,
                   const RBRec* rb, const GcBC& bc, double* sendbuf, hipStream_t st) {
  if (L.n == 0) return;
  const unsigned g = (unsigned)std::min(L.n, 65535 * 8);
  OP_SWITCH(op, k_gs_sub, g, 256, st, L, lambda, e, colours, C, rb, bc, sendbuf);
}

template <int OP>
static void gs_lex_lds(const LevelView& L, double lambda, unsigned g, int block, hipStream_t st) {
  switch (L.nc) {
    case 16: k_gs_lex_lds<OP, 16><<<g, block, 0, st>>>(L, lambda); break;
    case 8: k_gs_lex_lds<OP, 8><<<g, block, 0, st>>>(L, lambda); break;
    case 4: k_gs_lex_lds<OP, 4><<<g, block, 0, st>>>(L, lambda); break;
    default: k_gs_lex_lds<OP, 2><<<g, block, 0, st>>>(L, lambda); break;
  }
}

// persistent grid: `per_cu` workgroups per CU (the LDS limit), a multiple of 8
static unsigned gs_grid(int n, int per_cu) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  const long long g = std::min<long long>(n, (long long)cus * per_cu);
  return (unsigned)(g < 8 ? g : g & ~7LL);
}

template <int OP>
static void gs_lex_wave(const LevelView& L, double lambda, hipStream_t st) {
  switch (L.nc) {
    case 16:
      // 46.6 KB of LDS per box: 3 workgroups per CU
      k_gs_lex_wave<OP, 16, 256, 3><<<gs_grid(L.n, 3), 256, 0, st>>>(L, lambda);
      break;
    default: k_gs_lex_wave<OP, 8, 64, 4><<<gs_grid(L.n, 16), 64, 0, st>>>(L, lambda); break;
  }
}

bool gs_lex_ring_ok(int nc, int op) { return nc == 16 && (op == OP_LPL || op == OP_HELM); }

// bc_to_gc (m_ghost_cells.f90:665-766) of phi on the physical faces of the
// listed boxes, from their stored boundary cells: what the fill after the last
// sweep of a ghost-set chain would still have to do (the pushes covered the
// same-GPU faces)
__global__ void __launch_bounds__(256) k_phys_gc(LevelView L, GcBC bc, const int* __restrict__ boxes) {
  const int b = boxes[blockIdx.x];
  const FaceTopo T = load_topo(L, b);
  double* u = boxp(L, 1, b);
  const int nc = L.nc, n2 = nc * nc;
  for (int p = threadIdx.x; p < 6 * n2; p += blockDim.x) {
    const int f = p / n2, nb = f + 1, a = p % nc + 1, c = (p % n2) / nc + 1;
    if (T.kind(f) != NB_PHYS) continue;
    const bool low = nb & 1;
    const int x1 = low ? 1 : nc, x2 = low ? 2 : nc - 1, gi = off_gh(L, nb, a, c);
    u[gi] = phys_ghost(L, bc, b, (long long)b * 6 + f, nb, T.phys_code(f), a, c, gi,
                       u[off_face_cell(L, nb, x1, a, c)], u[off_face_cell(L, nb, x2, a, c)]);
  }
}

void launch_phys_gc(const LevelView& L, const GcBC& bc, const int* boxes, int n_boxes, hipStream_t st) {
  if (n_boxes > 0) k_phys_gc<<<n_boxes, 256, 0, st>>>(L, bc, boxes);
}

void launch_rhs_lex(const LevelView& L, double* rl, hipStream_t st) {
  if (L.n == 0) return;
  if (L.nc != 16) throw std::runtime_error("launch_rhs_lex: 16^3 boxes only");
  k_rhs_reg<<<L.n, 256, 0, st>>>(L, rl);
}

// rhs prefetch depth of the ring kernel in steps (a divisor of the ring's
// 18): 1 measured fastest (973 against 999 us for 3; 9 and 18 at one wave per
// SIMD slower)
constexpr int kGsRegPF = 1;

void launch_gs_lex(const LevelView& L, int op, double lambda, hipStream_t st, const double* rl, double* xl,
                   const GhostSets* gs, const GcBC* bc) {
  if (L.n == 0) return;
  if (rl) {
    if (!gs_lex_ring_ok(L.nc, op)) throw std::runtime_error("launch_gs_lex: no ring kernel for this level");
    // one wave per box, one box per workgroup (8 per CU by their LDS)
    if (gs && !bc) throw std::runtime_error("launch_gs_lex: ghost sets need the boundary conditions");
    const GhostSets g0{nullptr, 0, nullptr, 0, 0};
    const GcBC b0{};
    if (gs) {
      if (op == OP_HELM)
        k_gs_lex_reg<OP_HELM, kGsRegPF, true><<<L.n, 64, 0, st>>>(L, lambda, rl, xl, *gs, *bc);
      else
        k_gs_lex_reg<OP_LPL, kGsRegPF, true><<<L.n, 64, 0, st>>>(L, lambda, rl, xl, *gs, *bc);
    } else if (op == OP_HELM) {
      k_gs_lex_reg<OP_HELM, kGsRegPF, false><<<L.n, 64, 0, st>>>(L, lambda, rl, xl, g0, b0);
    } else {
      k_gs_lex_reg<OP_LPL, kGsRegPF, false><<<L.n, 64, 0, st>>>(L, lambda, rl, xl, g0, b0);
    }
    return;
  }
  if ((L.nc == 16 || L.nc == 8) && (op == OP_LPL || op == OP_HELM)) {
    // persistent, software-pipelined (k_gs_lex_wave); the variable-coefficient
    // operators keep the one-box-per-workgroup kernel (their eps loads would
    // spill the pipelined kernel)
    if (op == OP_HELM)
      gs_lex_wave<OP_HELM>(L, lambda, st);
    else
      gs_lex_wave<OP_LPL>(L, lambda, st);
    return;
  }
  const unsigned g = (unsigned)std::min(L.n, 65535 * 8);
  const int block = L.nc * L.nc >= 256 ? 256 : ((L.nc * L.nc + 63) / 64) * 64;
  if (L.nc == 16 || L.nc == 8 || L.nc == 4 || L.nc == 2) {
    switch (op) {
      case OP_HELM: gs_lex_lds<OP_HELM>(L, lambda, g, block, st); break;
      case OP_AHELM: gs_lex_lds<OP_AHELM>(L, lambda, g, block, st); break;
      case OP_VLPL: gs_lex_lds<OP_VLPL>(L, lambda, g, block, st); break;
      case OP_VHELM: gs_lex_lds<OP_VHELM>(L, lambda, g, block, st); break;
      default: gs_lex_lds<OP_LPL>(L, lambda, g, block, st); break;
    }
    return;
  }
  OP_SWITCH(op, k_gs_lex, g, block, st, L, lambda);
}

void launch_box_op(const LevelView& L, int op, double lambda, int i_out, hipStream_t st) {
  const long long work = 2LL * L.hv * L.n;
  if (work == 0) return;
  OP_SWITCH(op, k_box_op, grid_for(work), 256, st, L, lambda, i_out);
}

void launch_residual(const LevelView& L, int op, double lambda, unsigned long long* maxbits, hipStream_t st) {
  const long long work = 2LL * L.hv * L.n;
  if (work == 0) return;
  OP_SWITCH(op, k_residual, grid_for(work), 256, st, L, lambda, maxbits);
}

void launch_rb_pack(const LevelView& C, int iv, const int* items, int n, int nc, double* buf, hipStream_t st) {
  if (n == 0) return;
  const long long work = (long long)n * nc * nc;
  k_rb_pack<<<grid_for(work), 256, 0, st>>>(C, iv, items, n, nc, buf);
}

void launch_rbh_gather(const LevelView& L, const LevelView& C, int iv, const RBRec* rb, const int* items,
                       const int* rslot, int n, const double* rbrecv, double* cgc, double* cc, hipStream_t st) {
  if (n == 0) return;
  const long long s = L.nc + 2, work = (long long)n * (L.nc * L.nc + s * s * s);
  k_rbh_gather<<<grid_for(work), 256, 0, st>>>(L, C, iv, rb, items, rslot, n, rbrecv, cgc, cc);
}

void launch_rbh_scatter(const LevelView& L, int iv, const int* items, int n, const double* cc, hipStream_t st) {
  if (n == 0) return;
  k_rbh_scatter<<<grid_for((long long)n * L.nc * L.nc), 256, 0, st>>>(L, iv, items, n, cc);
}

void launch_rb_unpack(const LevelView& L, int iv, const int* items, int n, const double* recv, hipStream_t st) {
  if (n == 0) return;
  const long long work = (long long)n * L.nc * L.nc;
  k_rb_unpack<<<grid_for(work), 256, 0, st>>>(L, iv, items, n, recv);
}

void launch_fill_gc(const LevelView& L, int iv, int colours, const LevelView& C, const RBRec* rb,
                    const GcBC& bc, double* sendbuf, hipStream_t st) {
  const long long work = (long long)L.n * 6 * L.nc * L.nc;
  if (work == 0) return;
  k_fill_gc<<<grid_for(work), 256, 0, st>>>(L, iv, colours, C, rb, bc, sendbuf);
}

void launch_unpack_faces(const LevelView& L, int iv, const int* items, int n, const double* recv,
                         hipStream_t st, int colours) {
  const long long work = (long long)n * L.nc * L.nc;
  if (work == 0) return;
  k_unpack_faces<<<grid_for(work), 256, 0, st>>>(L, iv, items, n, recv, colours);
}

void launch_restrict(const LevelView& F, const LevelView& C, int iv, const int* pairs, int n_pairs,
                     const int* parent_local, const int* dixp, hipStream_t st) {
  const int h = F.nc / 2;
  const long long work = (long long)h * h * h * n_pairs;
  if (work == 0) return;
  k_restrict<<<grid_for(work), 256, 0, st>>>(F, C, iv, pairs, n_pairs, parent_local, dixp);
}

void launch_restrict_pack(const LevelView& F, int iv, const int* items, int n, double* buf, hipStream_t st) {
  const int h = F.nc / 2;
  const long long work = (long long)h * h * h * n;
  if (work == 0) return;
  k_restrict_pack<<<grid_for(work), 256, 0, st>>>(F, iv, items, n, buf);
}

void launch_box_pack(const LevelView& L, int iv, const int* items, int n, double* buf, hipStream_t st) {
  const long long work = L.stride * n;
  if (work == 0) return;
  k_box_pack<<<grid_for(work), 256, 0, st>>>(L, iv, items, n, buf);
}

void launch_box_unpack(const LevelView& L, int iv, const int* items, int n, const double* buf, hipStream_t st) {
  const long long work = L.stride * n;
  if (work == 0) return;
  k_box_unpack<<<grid_for(work), 256, 0, st>>>(L, iv, items, n, buf);
}

void launch_restrict_unpack(const LevelView& C, int iv, const int* items, int n, int hnc, const double* buf,
                            hipStream_t st) {
  const long long work = (long long)hnc * hnc * hnc * n;
  if (work == 0) return;
  k_restrict_unpack<<<grid_for(work), 256, 0, st>>>(C, iv, items, n, hnc, buf);
}

void launch_coarse_rhs(const LevelView& C, int op, double lambda, const int* parents, int n_par,
                       hipStream_t st) {
  const long long work = (2LL * C.hv + 6LL * C.fs) * n_par;
  if (work == 0) return;
  OP_SWITCH(op, k_coarse_rhs, grid_for(work), 256, st, C, lambda, parents, n_par);
}

void launch_sub_parents(const LevelView& C, const int* parents, int n_par, hipStream_t st) {
  const long long work = (2LL * C.hv + 6LL * C.fs) * n_par;
  if (work == 0) return;
  k_sub_parents<<<grid_for(work), 256, 0, st>>>(C, parents, n_par);
}

void launch_prolong(const LevelView& C, const LevelView& F, int iv, int iv_to, int add, const int* pairs,
                    int n_pairs, const int* parent_local, const int* dixp, hipStream_t st) {
  const long long work = 2LL * F.hv * n_pairs;
  if (work == 0) return;
  k_prolong<<<grid_for(work), 256, 0, st>>>(C, F, iv, iv_to, add, pairs, n_pairs, parent_local, dixp);
}

void launch_prolong_pack(const LevelView& C, const LevelView& F, int iv, const int* items, int n, double* buf,
                         hipStream_t st) {
  const long long work = 2LL * F.hv * n;
  if (work == 0) return;
  k_prolong_pack<<<grid_for(work), 256, 0, st>>>(C, F, iv, items, n, buf);
}

void launch_prolong_unpack(const LevelView& F, int iv_to, int add, const int* items, int n,
                           const double* buf, hipStream_t st) {
  const long long work = 2LL * F.hv * n;
  if (work == 0) return;
  k_prolong_unpack<<<grid_for(work), 256, 0, st>>>(F, iv_to, add, items, n, buf);
}

void launch_subtract(const LevelView& L, int iv, const double* mean, int ghosts, hipStream_t st) {
  const long long work = (2LL * L.hv + 6LL * L.fs) * L.n;
  if (work == 0) return;
  if ((L.nc & 1) == 0) {
    const int per2 = (int)((ghosts ? 2LL * L.hv + 6LL * L.fs : 2LL * L.hv) / 2);
    k_subtract_even<<<grid_for((long long)per2 * L.n), 256, 0, st>>>(L, iv, mean, per2);
    return;
  }
  k_subtract<<<grid_for(work), 256, 0, st>>>(L, iv, mean, ghosts);
}

void launch_set_rhs(const LevelView& L, const int* leaves, int n_leaves, double f1, double f2, hipStream_t st) {
  const long long work = 2LL * L.hv * n_leaves;
  if (work == 0) return;
  k_set_rhs<<<grid_for(work), 256, 0, st>>>(L, leaves, n_leaves, f1, f2);
}

__global__ void __launch_bounds__(256) k_copy_ghosts(LevelView L) {
  const long long per = (L.stride - 2LL * L.hv) / 2;   // 16-B pairs per box
  GRID_STRIDE(t, per * L.n) {
    const int b = (int)(t / per);
    const long long o = 2LL * L.hv + 2 * (t % per);
    *reinterpret_cast<double2*>(boxp(L, 3, b) + o) = *reinterpret_cast<const double2*>(boxp(L, 1, b) + o);
  }
}

void launch_copy_ghosts(const LevelView& L, hipStream_t st) {
  const long long work = (L.stride - 2LL * L.hv) / 2 * L.n;
  if (work <= 0) return;
  k_copy_ghosts<<<grid_for(work), 256, 0, st>>>(L);
}

void launch_copy_var(const LevelView& L, int src, int dst, hipStream_t st) {
  const long long work = (long long)L.stride * L.n;
  if (work == 0) return;
  k_copy_var<<<grid_for(work), 256, 0, st>>>(L, src, dst);
}

void launch_from_ref(const LevelView& L, int iv, const double* ref, hipStream_t st) {
  const long long s = L.nc + 2, work = s * s * s * L.n;
  if (work == 0) return;
  k_from_ref<<<grid_for(work), 256, 0, st>>>(L, iv, ref);
}

void launch_to_ref(const LevelView& L, int iv, double* ref, double unstored, hipStream_t st) {
  const long long s = L.nc + 2, work = s * s * s * L.n;
  if (work == 0) return;
  k_to_ref<<<grid_for(work), 256, 0, st>>>(L, iv, ref, unstored);
}

}  // namespace omg
