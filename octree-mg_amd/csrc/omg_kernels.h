// omg_kernels.h — launchers of the level kernels (omg_kernels.hip, omg_sweep.hip).
#pragma once

#include "omg_internal.h"

namespace omg {

// Physical-boundary description passed to the ghost-cell kernels.
struct GcBC {
  int type[6];
  double value[6];
  const long long* face_off;   // [n*6] or null (tabulated callback)
  const int* face_type;
  const double* face_data;
  int phi_stored;              // mg%phi_bc_data_stored
};

// red-black substep (colour e) + the ghost fill after it; picks the LDS-tiled
// kernel (omg_sweep.hip) when the level allows, else the generic one
// shift (device scalar or null): subtract it from every value the substep
// loads (a pending subtract_mean of phi, bit-identical to applying it first)
// boxes/n_boxes: only these boxes (local indices), else the whole level
// rbgv / rbgv_mode: the level's buffer of refinement-boundary coarse parts
// (RbSide::gv: 1 = compute and store, 2 = read; tiled kernel only)
void launch_gs_substep(const LevelView& L, int op, double lambda, int e, int colours, const LevelView& C,
                       const RBRec* rb, bool has_rb, const GcBC& bc, double* sendbuf, const double* shift,
                       hipStream_t st, const int* boxes = nullptr, int n_boxes = 0, double* rbgv = nullptr,
                       int rbgv_mode = 0);
// whether launch_gs_substep takes the LDS-tiled kernel (which alone takes a shift)
// M(NC, BS, OPV) for the operator op (OPV a compile-time Op)
#define OMG_FOR_OP(op, M, NC, BS)         \
  switch (op) {                           \
    case OP_HELM: M(NC, BS, OP_HELM) break;   \
    case OP_VLPL: M(NC, BS, OP_VLPL) break;   \
    case OP_VHELM: M(NC, BS, OP_VHELM) break; \
    case OP_AHELM: M(NC, BS, OP_AHELM) break; \
    default: M(NC, BS, OP_LPL) break;         \
  }

// (every operator; refinement-boundary faces are filled in its epilogue)
inline bool gs_tiled(int nc, int op, bool has_rb) {
  (void)op;
  (void)has_rb;
  return nc == 16 || nc == 8 || nc == 4 || nc == 2;
}
// Three red-black substeps (colours e, 1-e, e) of a level in one pass
// (k_gsrb3, omg_block.hip): reads phi from L.phi, writes every interior cell
// and ghost face to dst (the level's other phi buffer).  cols: per workgroup a
// record of kB3Rec ints, [0] = number of boxes in the column (1..kB3MaxZ),
// then for slots zs = 0..len+1 (the box below the column, its boxes from
// low to high z, the box above) at 1 + kB3S*zs the boxes xs + (kB3TX+2)*ys
// (xs = 0: the x neighbour below the tile, 1..kB3TX: the tile's boxes,
// kB3TX+1: the one above; ys = 0 / 1 / 2 likewise in y; edges by neighbour of
// neighbour).  Levels of 16^3 boxes whose faces are all same-GPU boxes.
constexpr int kB3TX = 2;                         // boxes per tile in x
constexpr int kB3S = 3 * (kB3TX + 2);            // record slots per z slot
constexpr int kB3MaxZ = 16;                      // boxes per column in z (at most)
constexpr int kB3Rec = (1 + kB3S * (kB3MaxZ + 2) + 15) / 16 * 16;
bool gsrb3_op_ok(int op);
// Physical faces (round 6): [0] also holds the column's physical faces,
// len | flags << 8 (bit f: face f+1 of the column, x-, x+, y-, y+ of its
// boxes, z- of its first, z+ of its last); a slot across such a face names
// the box whose face it is.  The ghost there is bc_to_gc's
// (m_ghost_cells.f90:665-766) c0 * b + c1 * x1 + c2 * x2 with constant b per
// face: k = c0 * b (formed on the host, the same product), c1, c2.
constexpr int kB3LenMask = 255;
struct B3Phys {
  double k[6], c1[6], c2[6];
};
// four substeps (colours e, 1-e, e, 1-e) per pass, same columns (k_gsrb4,
// omg_block.hip): the down-smoothing of a level whose residual + restriction
// then runs unfused (the default; OMG_NO_BLOCK4)
// coarse (PRO 2, round 6): the up-smoothing's correct_children form with all
// four substeps, the correction from the coarse res its last pass stored
// (k_gsrb3's coarse_mode 2; ccols as for launch_gsrb3)
// push false: the interior only, no ghost face written (the caller marks the
// level's ghosts deferred: Level::gc_deferred)
void launch_gsrb4(const LevelView& L, double* dst, const int* cols, int n_cols, int op, double lambda, int e,
                  const double* shift, hipStream_t st, const LevelView* coarse = nullptr,
                  const int* ccols = nullptr, const B3Phys* phys = nullptr, bool push = true);
// push1 false: the ghost faces get the colour-e cells only (the colour-(1-e)
// halves are left stale: only for a pass that k_smooth_resid follows, which
// reads colour e's and forms colour 1-e's itself)
// coarse (k_gsrb3's correct_children form): before substep 1 the pass adds the
// prolonged correction phi - old of the coarse level (mg_prolong_sparse of
// correct_children, m_multigrid.f90:127-136) to the colour-(1-e) cells it
// reads, and stores the coarse level's res = phi - old (interior and faces).
// ccols: per workgroup kB3CRec ints, [0] = the column's y offset inside its
// coarse boxes (0 / 8), then at 1 + 9*zc + 3*ys + xs the coarse boxes around
// the column (zc = 0: below, 1..len/2: the column's own, then above).  The
// column's fine boxes are the children of those (len even).  coarse_mode 1:
// the correction from the coarse phi and old, and the pass stores the coarse
// res; 2: the coarse res is already stored (its last pass ran with `res`) and
// is what the pass reads.
// res: the pass also stores this level's res = phi - old (interior and faces),
// what correct_children of the level above stores before it prolongs
// (a plain pass only, push1).
constexpr int kB3CSlots = 9 * (kB3MaxZ / 2 + 2);                // coarse boxes per record
constexpr int kB3CRec = (1 + kB3CSlots + 15) / 16 * 16;
void launch_gsrb3(const LevelView& L, double* dst, const int* cols, int n_cols, int op, double lambda, int e,
                  const double* shift, hipStream_t st, bool push1 = true, const LevelView* coarse = nullptr,
                  const int* ccols = nullptr, int coarse_mode = 1, bool res = false,
                  const B3Phys* phys = nullptr);
void launch_gs_sub(const LevelView& L, int op, double lambda, int e, int colours, const LevelView& C,
                   const RBRec* rb, const GcBC& bc, double* sendbuf, hipStream_t st);
// rl: rhs copy in ring order (launch_rhs_lex) for the register-ring kernel,
// on gs_lex_ring_ok levels; null: the line-per-thread kernels
// xl (register ring only, may be null): the swept boxes' new x boundary
// layers, 512 doubles per box, for launch_fill_tile_xl
// Two ghost-face sets for chains of register-ring sweeps (round 4): the
// sweep reads its ghosts from `in` and pushes its new boundary layers into
// the same-GPU neighbours' ghosts in `out` (per box `stride` doubles, the
// six faces laid out as in the box storage from 2*HV on), so no fill pass
// runs between sweeps; phys_load: the physical ghosts of `in` are formed at
// load from the box's own (final) boundary cells, as the fill after the
// previous sweep would have (bc_to_gc).  Levels whose faces are same-GPU or
// physical only.
struct GhostSets {
  const double* in;
  long long in_stride;
  double* out;
  long long out_stride;
  int phys_load;
};
void launch_gs_lex(const LevelView& L, int op, double lambda, hipStream_t st, const double* rl = nullptr,
                   double* xl = nullptr, const GhostSets* gs = nullptr, const GcBC* bc = nullptr);
// custom refinement-boundary faces on the host (omg_set_refinement_bnd): per
// record (item b*6+nb-1) the coarse face and the box in the reference layout,
// and the callback's ghost face back
void launch_rbh_gather(const LevelView& L, const LevelView& C, int iv, const RBRec* rb, const int* items,
                       const int* rslot, int n, const double* rbrecv, double* cgc, double* cc, hipStream_t st);
void launch_rbh_scatter(const LevelView& L, int iv, const int* items, int n, const double* cc, hipStream_t st);
// the physical ghosts of phi of the listed boxes (bc_to_gc from the boxes'
// final boundary cells), after a chain of ghost-set sweeps
void launch_phys_gc(const LevelView& L, const GcBC& bc, const int* boxes, int n_boxes, hipStream_t st);
// the physical and refinement-boundary ghosts of phi of the listed boxes from
// their final boundary cells (C: the coarse level), after a split fused
// down-step
void launch_face_gc(const LevelView& L, const LevelView& C, const GcBC& bc, const int* boxes, int n_boxes,
                    hipStream_t st);
bool gs_lex_ring_ok(int nc, int op);
// rhs copied into the ring kernel's order
void launch_rhs_lex(const LevelView& L, double* rl, hipStream_t st);
void launch_box_op(const LevelView& L, int op, double lambda, int i_out, hipStream_t st);
void launch_residual(const LevelView& L, int op, double lambda, unsigned long long* maxbits,
                     hipStream_t st);
void launch_max_fold(unsigned long long* slots, unsigned long long* out, bool accumulate, hipStream_t st);
void launch_fill_gc(const LevelView& L, int iv, int colours, const LevelView& C, const RBRec* rb,
                    const GcBC& bc, double* sendbuf, hipStream_t st);
void launch_unpack_faces(const LevelView& L, int iv, const int* items, int n, const double* recv,
                         hipStream_t st, int colours = 3);
// deep halo (split levels of k_gsrb3 / k_gsrb4): bricks of 4^3 cells of one
// colour c (per 32) or both (per 64) between boxes / proxies and a buffer
void launch_deep_copy(const LevelView& L, int iv, int c, int per, const int* items, int n, double* buf, bool unpack,
                      hipStream_t st);
// the boundary layer of variable iv at the listed faces (b*6+nb-1) into the halo send buffer
void launch_face_pack(const LevelView& L, int iv, const int* items, int n, double* buf, hipStream_t st);
void launch_rb_pack(const LevelView& C, int iv, const int* items, int n, int nc, double* buf, hipStream_t st);
void launch_rb_unpack(const LevelView& L, int iv, const int* items, int n, const double* recv, hipStream_t st);
void launch_restrict(const LevelView& F, const LevelView& C, int iv, const int* pairs, int n_pairs,
                     const int* parent_local, const int* dixp, hipStream_t st);
void launch_restrict_pack(const LevelView& F, int iv, const int* items, int n, double* buf,
                          hipStream_t st);
void launch_box_pack(const LevelView& L, int iv, const int* items, int n, double* buf, hipStream_t st);
void launch_box_unpack(const LevelView& L, int iv, const int* items, int n, const double* buf, hipStream_t st);
void launch_restrict_unpack(const LevelView& C, int iv, const int* items, int n, int hnc,
                            const double* buf, hipStream_t st);
void launch_coarse_rhs(const LevelView& C, int op, double lambda, const int* parents, int n_par,
                       hipStream_t st);
void launch_sub_parents(const LevelView& C, const int* parents, int n_par, hipStream_t st);
void launch_prolong(const LevelView& C, const LevelView& F, int iv, int iv_to, int add, const int* pairs,
                    int n_pairs, const int* parent_local, const int* dixp, hipStream_t st);
void launch_prolong_pack(const LevelView& C, const LevelView& F, int iv, const int* items, int n,
                         double* buf, hipStream_t st);
void launch_prolong_unpack(const LevelView& F, int iv_to, int add, const int* items, int n,
                           const double* buf, hipStream_t st);
void launch_subtract(const LevelView& L, int iv, const double* mean, int ghosts, hipStream_t st);
void launch_set_rhs(const LevelView& L, const int* leaves, int n_leaves, double f1, double f2, hipStream_t st);
void launch_copy_var(const LevelView& L, int src, int dst, hipStream_t st);
void launch_from_ref(const LevelView& L, int iv, const double* ref, hipStream_t st);
void launch_to_ref(const LevelView& L, int iv, double* ref, double unstored, hipStream_t st);
void launch_poison_ghosts(const LevelView& L, int n_vars, double poison, hipStream_t st);
void launch_phi_bc_store(const LevelView& L, const GcBC& bc, int* nba, hipStream_t st);

// The coarse end of the V-cycle in ONE single-workgroup launch (omg_tiles.hip):
// levels lowest..top (each a handful of boxes, all on this GPU), from the
// down-smoothing of `top` through the coarse solve to the up-smoothing of
// `top`, with every level step separated by a workgroup barrier instead of a
// kernel boundary and the coarse-solve convergence test on the device.
constexpr int kTailMaxLevels = 12;
constexpr int kTailMaxBoxes = 1;
struct TailLevel {
  LevelView L;
  GcBC bc;
  const int* parents;      // my_parents (local indices)
  int n_par;
  const int* parent_local; // per box: parent's local index at lvl-1
  const int* dixp;         // per box: packed child offset
  int foff[6];             // bc.face_off / face_type of the level's first box
  signed char ftype[6];    // (-1: not tabulated, -2: beyond int, read bc.face_off),
                           // resolved on the host
};
struct TailArgs {
  int n_lvls;              // lv[0] = lowest .. lv[n_lvls-1] = top
  TailLevel lv[kTailMaxLevels];
  double lambda;
  int n_down, n_up, max_coarse;
  double res_abs, res_rel;
  unsigned long long* maxbits;   // device scratch
  int* coarse_its;               // device: sweeps the coarse solve took
  int gs_lex;                    // smoother: lexicographic GS (else red-black)
  long long* stamps;             // OMG_TAIL_TIMING: wall clock per phase (thread 0), or null
  // levels 0..lds_levels-1 run with their box resident in LDS (at most 8^3
  // cells, a single box whose local faces are itself), and lds_top: the 16^3
  // top level above them too (tail_lds_plan in omg_api.cpp)
  int lds_levels, lds_top;
  // the tail forms the top level's ghosts and its coarse rhs = L(phi) + res,
  // old = phi itself (update_coarse of top+1 stopped after the restriction)
  int top_crhs, pad_;
};
// how many of the tail's lowest levels qualify for the LDS-resident program
constexpr int kTailLdsMaxLevels = 3;   // 8^3, 4^3, 2^3

void launch_coarse_tail(const TailArgs* dA, int gs_lex, int op, hipStream_t st);   // dA: device memory
void launch_store_tail(const TailArgs& A, TailArgs* d, hipStream_t st);   // *d = A in stream order

// LDS-tiled fused kernels (omg_tiles.hip), even box sizes 2..16
bool tiled_nc(int nc);
// the ghost fill of phi for a level without refinement boundaries, box sizes
// 4, 8, 16 (false: use launch_fill_gc)
bool launch_fill_tile(const LevelView& L, const GcBC& bc, double* sendbuf, hipStream_t st);
// the same fill right after a register-ring GS sweep of a 16^3 level without
// refinement boundaries: boxes without a physical face read only their
// boundary layers (y/z from phi, x from the sweep's xl)
void launch_fill_tile_xl(const LevelView& L, const GcBC& bc, double* sendbuf, const double* xl, hipStream_t st);
// the last down-smoothing substep (colour 0) + residual + restriction in one
// pass (k_smooth_resid); false: not available for this op / box size
bool launch_smooth_resid(const LevelView& F, const LevelView& C, int op, double lambda, int restrict_on,
                         const int* parent_local, const int* dixp, hipStream_t st, const int* list,
                         int n_list, const GcBC& bc, bool has_rb, bool has_phys, const double* rbgv = nullptr);
void launch_resid_restrict(const LevelView& F, const LevelView& C, int op, double lambda,
                           unsigned long long* maxbits, int restrict_on, const int* parent_local,
                           const int* dixp, hipStream_t st, const int* list = nullptr, int n_list = 0);
// sub: form the parent's res = phi - old on the fly (and store it) instead of
// reading it (correct_children's parent loop fused in); skip1: a colour-1
// red-black substep follows, so all-local boxes correct and push colour 0 only
// save_old (with !skip1): also old = phi on the interior, from the values
// before the correction (FMG, launch_copy_ghosts for the ghost faces)
// rb: the fine level's refinement-boundary records (its NB_RB ghosts are
// interpolated from C, sides_rb), or null when it has none
void launch_prolong_fill(const LevelView& C, const LevelView& F, int iv, const int* parent_local,
                         const int* dixp, const GcBC& bc, double* sendbuf, bool sub, bool skip1,
                         hipStream_t st, const int* list = nullptr, int n_list = 0, bool save_old = false,
                         const RBRec* rb = nullptr);
// old = phi on the ghost faces (and padding) of every box: [2*hv, stride)
void launch_copy_ghosts(const LevelView& L, hipStream_t st);
// correct_children + fill + the first up-smoothing substep (colour 1) in one
// pass; fine boxes with their parent here and no remote faces (all, or the
// `list`); push0: per box, faces to push the corrected colour 0 to; rb: the
// level has refinement-boundary faces (one GPU, 16^3 / 8^3 boxes)
void launch_prolong_smooth(const LevelView& C, const LevelView& F, int op, double lambda, const int* parent_local,
                           const int* dixp, const GcBC& bc, int one_child, const int* list, int n_list,
                           const uint8_t* push0, hipStream_t st, bool rb = false, double* rbgv = nullptr);
// update_coarse's parent loop, LDS-tiled; false when the box size / operator
// has no tiled kernel (caller falls back to launch_coarse_rhs)
// update_coarse's fill of the coarse level + its parents' coarse rhs in one
// pass (levels whose faces are same-GPU or physical, 16^3 / 8^3 / 4^3 boxes)
void launch_fill_crhs(const LevelView& C, int op, double lambda, const GcBC& bc, const uint8_t* parmask,
                      hipStream_t st);
bool launch_coarse_rhs_tile(const LevelView& C, int op, double lambda, const int* parents, int n_par,
                            hipStream_t st);
void launch_box_sums(const LevelView& L, int iv, const int* leaves, int n, double* out, hipStream_t st);
bool subtract_sums_nc(int nc);
void launch_subtract_sums(const LevelView& L, int iv, const int* leaves, int n, const double* mean, double* out,
                          hipStream_t st);
void launch_mean(const double* all, int n, double volume, double* mean, hipStream_t st);
// init: start from +0.0 instead of *acc
void launch_seq_sum(const double* box_sums, int n, double w, double* acc, bool init, hipStream_t st);

}  // namespace omg
