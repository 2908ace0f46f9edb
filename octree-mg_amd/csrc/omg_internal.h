// omg_internal.h — device data model of the MI355X octree-mg V-cycle.
//
// Every octree level that this rank owns boxes on is one contiguous HBM arena
//     data[var][box][stride]        stride = stored_cells(nc) padded to 64 doubles
// with boxes in the reference's my_ids order; inside a box, the interior split
// by red-black colour and the six ghost faces (omg_device.h).  Per-level topology
// tables let one kernel launch cover a whole level: for every (box, face) a
// kind + argument (local neighbour index / physical bc code / refinement-
// boundary record / halo receive slot), parent and child offsets for the grid
// transfers, and the per-peer RCCL pack lists for multi-GPU halos.
#pragma once

#include <cstdlib>
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/omg.h"   // (the host-transport callback types)

namespace omg {

// NB_RBREM: refinement boundary whose coarse neighbour lives on another rank;
// its interpolated coarse face arrives with the halo (buffer_for_fine_nb).
enum NbKind : int8_t { NB_LOCAL = 0, NB_PHYS = 1, NB_RB = 2, NB_REMOTE = 3, NB_RBREM = 4 };

enum Op : int { OP_LPL = 1, OP_VLPL = 2, OP_HELM = 3, OP_VHELM = 4, OP_AHELM = 5 };

constexpr int kMaxVars = 16;

// k_gsrb3 (omg_block.hip): levels of fewer boxes take one substep per launch
// (a 512-box level: 57 us per pass against 3 x 8.5 us, latency-bound; 4096
// boxes: 102 against 126)
constexpr int kB3MinBoxes = 4096;

// Physical boundary condition of one variable (mg%bc(:, iv)).
struct BCVar {
  int type[6];
  double value[6];
  long long* d_face_off = nullptr;   // per level: [n*6] offsets (or -1), device
  int* d_face_type = nullptr;
};

// A view of one level, passed to kernels by value (layout: omg_device.h).
struct LevelView {
  double* data;          // [n_vars][n][stride]
  double* phi;           // phi (= var 1 of data)
  long long stride;      // doubles per box and variable
  long long vstride;     // doubles per variable = (n + proxies) * stride
  int n;                 // local boxes
  int nc;                // box size (cells per dim)
  int h, hf;             // ceil(nc/2): cells of one colour per row / per face row
  int hv;                // h*nc*nc: slots of one colour of the interior
  int fs;                // 2*hf*nc: slots of one ghost face
  double idr2[3];        // 1/dr^2 per dim
  double dr[3];
  const int8_t* nbk;     // [n*6]
  const int* nba;        // [n*6]
  const int* sendpos;    // [n*6] halo send slot of remote faces (or -1)
  const int* topo;       // [n*8] packed face kinds + arguments (FaceTopo, omg_face.h; pack_topo)
  int rev;               // walk each XCD's run of boxes backwards (xcd_box)
};

// doubles of one stored ghost face (both colour halves)
inline int stored_face(int nc) { return 2 * ((nc + 1) / 2) * nc; }

// stored doubles per box and variable for box size nc (2 colours + 6 faces)
inline int stored_cells(int nc) {
  const int h = (nc + 1) / 2;
  return 2 * h * nc * nc + 6 * 2 * h * nc;
}

// Grid-transfer records.
struct RBRec {             // refinement boundary: coarse neighbour + child offset
  int coarse_idx;          // local index at lvl-1 of the parent's neighbour
  int dix[3];
};

struct PeerList {          // one peer's part of a transfer, in wire order
  int peer;
  std::vector<long long> keys;   // ordering keys (sort_and_transfer_buffers' ix)
  std::vector<int> items;  // meaning depends on the transfer type
  int offset = 0;          // first item in the device list / buffer
};

struct Transfer {          // one p2p pattern (halo, restrict, prolong)
  std::vector<PeerList> send, recv;
  int* d_send_items = nullptr;  // concatenated send items
  int* d_recv_items = nullptr;
  int n_send = 0, n_recv = 0;   // total items
  int item_doubles = 0;         // payload per item
  int send_ints = 1, recv_ints = 1;  // ints per item in the send / recv lists
};

// The faces of one level and variable whose refinement-boundary ghosts a host
// callback sets (omg_set_refinement_bnd): records (b*6+nb-1) sorted by face,
// the receive slot of NB_RBREM faces (-1: coarse neighbour on this rank), and
// the staging buffers of the coarse faces and the boxes (reference layout).
struct RbHostFaces {
  std::vector<int> items, slot, ids, nbs;
  int n = 0;
  int* d_items = nullptr;
  int* d_slot = nullptr;
  double* d_cgc = nullptr;
  double* d_cc = nullptr;
  double* h_cgc = nullptr;   // pinned
  double* h_cc = nullptr;    // pinned
};

struct Level {
  int lvl = 0, nc = 0, n = 0;
  long long stride = 0;
  double dr[3] = {0, 0, 0};
  std::vector<int> ids;                 // global ids of my boxes (my_ids order)
  // Replicated coarse level (omg_set_coarse_replication): every rank holds
  // every box; host_local lists the boxes the host's partition gives this rank
  // (what upload/download/level_size see), repl copies them to the peers.
  bool replicated = false;
  std::vector<int> host_local;
  Transfer repl;
  double* d_data = nullptr;
  double* d_phi = nullptr;              // phi (d_data's var 1)
  bool phi_gc_ok = false;               // phi's ghost faces equal what a fill would give
  // phi's ghost faces are stale only because the level's last pass left them
  // unwritten (the V-cycle's last up pass, correct_block3's defer_gc): the
  // reference's ghosts are a fill of the interior, which every ghost reader
  // runs first (fill_gc_lvl); the block passes read no ghosts on such a level
  bool gc_deferred = false;
  bool has_rb = false, has_remote = false, has_phys = false;
  // the same flags over the level's boxes on EVERY rank (from the global
  // tree): decisions that choose collective calls use these, never the local
  // ones, so every rank takes the same branch (fas_vcycle's stand-alone fill)
  bool any_rb = false, any_phys = false;
  // some refinement-boundary face of this level (on any rank) has its coarse
  // box on another rank than its fine box (refinement-boundary exchange,
  // finish_rb); the fused kernels that form refinement-boundary ghosts
  // themselves need the coarse box on the same GPU
  bool any_rbx = false;
  bool all_parents = false;      // every box of this rank at this level is a parent
  bool prolong_smooth_ok = false;  // k_prolong_smooth can serve this level (see build_plan)
  bool shift_pending = false;    // phi -= mean still to apply (see subtract_mean)
  int8_t* d_nbk = nullptr;
  int* d_nba = nullptr;
  int* d_sendpos = nullptr;
  std::vector<int> h_sendpos;
  // per box 8 words: the 6 faces' kind + argument packed (FaceTopo in
  // omg_face.h, built by pack_topo from h_nbk / h_nba / h_sendpos / h_rb),
  // word 6 = mask of the faces that are not same-GPU neighbours
  int* d_topo = nullptr;
  std::vector<int8_t> h_nbk;
  std::vector<int> h_nba;
  // refinement boundary records (fine side)
  RBRec* d_rb = nullptr;
  std::vector<RBRec> h_rb;
  // my_parents / my_leaves as local indices
  std::vector<int> parents, leaves;
  int* d_parents = nullptr;
  int* d_leaves = nullptr;
  uint8_t* d_parmask = nullptr;     // per box: 1 = a parent (k_fill_crhs)
  // refinement-boundary levels (one GPU): the coarse part of every rb ghost,
  // [box][face][nc*nc] (RbSide::gv), valid while the level below is unchanged
  double* d_rbgv = nullptr;
  bool rbgv_ok = false;
  // restriction onto this level from lvl+1 happens per fine box: for each of my
  // boxes at this level, the parent (local idx at lvl-1, or -1 if remote) and
  // its child offset inside the parent.
  std::vector<int> parent_local;        // [n]
  std::vector<int> dix_packed;          // [n]  dx | dy<<10 | dz<<20
  int* d_parent_local = nullptr;
  int* d_dix = nullptr;
  // local (child, parent) pairs for restriction / prolongation at this level
  // (this level = fine level)
  int* d_pairs = nullptr;               // [n_pairs] child local idx
  int n_pairs = 0;
  // transfers
  Transfer halo;        // ghost faces of this level (items: box*6+nb)
  Transfer restr;       // restriction this level -> lvl-1 (send: child idx; recv: parent*8+slot)
  Transfer prol;        // prolongation lvl-1 -> this level (send: child global → parent idx*8+slot; recv: my child idx)
  Transfer rbx;         // refinement-boundary faces across ranks at this level (send: coarse idx at
                        // lvl-1, coarse-side nb, child offset; recv: box*6+nb of my fine face)
  double* d_scratch_rhs = nullptr;   // leaf sums of rhs for the next get_sum
  double* d_rhs_lex = nullptr;       // rhs in ring order for the lexicographic smoother (ensure_rhs_lex)
  bool rhs_lex_ok = false;           // d_rhs_lex equals rhs (dropped by every rhs writer)
  double* d_xlay = nullptr;          // x boundary layers of the last register-ring sweep (k_fill_tile_xl)
  // the second ghost-face set of phi for chains of register-ring sweeps (6
  // faces per box, the stored face layout; GhostSets in omg_kernels.h)
  double* d_galt = nullptr;
  // three substeps per pass (k_gsrb3, launch_gsrb3): phi's second buffer (the
  // pass reads d_phi and writes the other one; d_phi is d_data's var 1 or
  // this) and the workgroups' box records (n_b3 columns); null: not eligible
  double* d_phi_buf = nullptr;
  int* d_b3 = nullptr;
  int n_b3 = 0;
  std::vector<int> h_b3;   // (host copy, for the coarse records below)
  // some columns have physical faces (round 6): the passes take the ghosts
  // there from constant boundary values (b3_phys, omg_api.cpp)
  bool b3_phys = false;
  // k_gsrb3's correct_children form: per column the coarse boxes around it
  // (launch_gsrb3's ccols); null: the level's up-smoothing starts with
  // k_prolong_smooth
  int* d_b3c = nullptr;
  // Deep halo (k_gsrb3 / k_gsrb4 on a level split over GPUs, plan_deep in
  // omg_api.cpp): the remote boxes the columns read are proxy boxes
  // n .. n+n_prox-1 of every variable (vstride covers them); before a pass the
  // cells the columns read travel as 4^3-cell bricks, phi of the colour the
  // pass reads (deep, 32 doubles per brick) and rhs when it changed since
  // (deep_rhs, 64: both colours); after it the remote faces' ghosts by the
  // halo plan.  Decided alike on every rank from the global tree.
  bool deep = false;
  int n_prox = 0;
  std::vector<int> prox_ids;     // global ids of the proxies, ascending
  Transfer deep_phi, deep_rhs;   // items: (box or n + proxy, brick)
  bool prox_rhs_ok = false;      // the proxies' rhs equals the owners' rhs
  bool faces_pending = false;    // deep_after's remote faces still in flight on the comm stream
  int* d_physbox = nullptr;          // boxes with a physical face (k_phys_gc after such a chain)
  int n_physbox = 0;
  int* d_bnd = nullptr;              // boxes with a face on another GPU / the others
  int* d_int = nullptr;
  int n_bnd = 0, n_int = 0;
  // the boxes of d_bnd with a physical or refinement-boundary face: their
  // ghosts there formed again (k_face_gc) after a split fused down-step
  int* d_bndface = nullptr;
  int n_bndface = 0;
  // [n]: for a box without remote faces, the faces (bit f = face f+1) whose
  // same-GPU neighbour has one (k_prolong_smooth pushes colour 0 there)
  uint8_t* d_push0 = nullptr;
  double* d_rbsend = nullptr;
  double* d_rbrecv = nullptr;
  double* d_sendbuf = nullptr;
  double* d_recvbuf = nullptr;
  size_t sendbuf_doubles = 0, recvbuf_doubles = 0;
  // per-leaf partial sums scratch
  double* d_scratch = nullptr;
  std::map<int, RbHostFaces> rbh;    // by variable: faces with a host refinement_bnd callback

  LevelView view() const {
    LevelView v;
    v.data = d_data;
    v.phi = d_phi;
    v.stride = stride;
    v.vstride = stride * (n + n_prox);
    v.n = n;
    v.nc = nc;
    v.h = v.hf = (nc + 1) / 2;
    v.hv = v.h * nc * nc;
    v.fs = 2 * v.hf * nc;
    for (int d = 0; d < 3; d++) {
      v.idr2[d] = 1 / (dr[d] * dr[d]);
      v.dr[d] = dr[d];
    }
    v.nbk = d_nbk;
    v.nba = d_nba;
    v.sendpos = d_sendpos;
    v.topo = d_topo;
    v.rev = 0;
    return v;
  }
  // the view for a level-wide pass: successive passes walk the boxes in
  // alternating directions, so each starts on the boxes the previous one
  // touched last (still in the 256 MiB Infinity Cache) instead of the ones
  // it touched first (evicted long ago)
  // (OMG_NO_REV=1: always forwards, for A/B timing)
  mutable int dir = 0;
  LevelView sweep_view() const {
    static const int on = getenv("OMG_NO_REV") ? 0 : 1;
    LevelView v = view();
    v.rev = dir & on;
    dir ^= 1;
    return v;
  }
};

struct PendingEv {
  const char* name;
  hipEvent_t e0, e1;
  double cells;
  int lvl;   // level of the launch (stats are kept per name and per name@lvl)
};

struct KStat {
  long long launches = 0;
  double ms = 0, cells = 0;
};

}  // namespace omg

struct omg_loop;          // in-process loopback transport (omg_api.cpp)
struct omg_free_state;    // free-space boundary conditions (omg_api.cpp, omg_free.hip)

namespace omg {
struct TailArgs;   // omg_kernels.h
// slots of a multi-workgroup max-residual launch (launch_max, omg_device.h)
constexpr int kMaxSlots = 256, kMaxSlotStride = 16;
}

struct omg_ctx {
  int device = 0, rank = 0, n_ranks = 1;
  bool host_only = false;                   // plan-only context (OMG_DEVICE_NONE)
  hipStream_t stream = nullptr;
  void* nccl = nullptr;  // ncclComm_t
  std::shared_ptr<omg_loop> loop;           // set instead of nccl in loopback mode
  std::map<int, long long> loop_seq_send, loop_seq_recv;
  long long loop_ar_seq = 0;
  // tree (global, host)
  int n_boxes = 0, lowest = 0, highest = 0, first_normal = 0, box_size = 0, n_vars = 4;
  std::vector<int> lvl, parent, children, neighbors, ix, rank_of;
  std::map<int, int> bsl;                   // box_size_lvl
  std::map<int, std::vector<double>> drl;   // dr per level
  std::map<int, std::vector<int>> ids, leaves, parents, ref_bnds;
  std::vector<int> local_index;             // id -> local index at its level (or -1)
  long long rep_cells = 0;                  // replicate coarse levels up to this many cells (0: off)
  int rep_lvl = INT_MIN;                    // highest replicated level (INT_MIN: none)
  std::map<int, omg::Level> levels;
  // method configuration
  int op = omg::OP_LPL, smoother = 1, n_substeps = 1;
  int n_cycle_down = 2, n_cycle_up = 2, max_coarse_cycles = 1000;
  double lambda = 0, res_abs = 1e-8, res_rel = 1e-8;
  int subtract_mean = 0, phi_bc_data_stored = 0;
  omg::BCVar bc[omg::kMaxVars];
  std::vector<long long> h_face_off[omg::kMaxVars];
  std::vector<int> h_face_type[omg::kMaxVars];
  double* d_face_data[omg::kMaxVars] = {};
  std::map<int, long long*> d_face_off_lvl[omg::kMaxVars];
  std::map<int, int*> d_face_type_lvl[omg::kMaxVars];
  // host copies of the first box's entries (the coarse tail's one-box levels
  // carry them inline, TailLevel::foff)
  std::map<int, std::vector<long long>> h_face_off_lvl[omg::kMaxVars];
  std::map<int, std::vector<int>> h_face_type_lvl[omg::kMaxVars];
  // scalars
  double* d_red = nullptr;             // device reductions (get_sum / subtract_mean)
  hipStream_t stream2 = nullptr;       // side stream (rhs sum chain)
  hipStream_t stream_comm = nullptr;   // halo exchange overlapped with interior boxes (highest priority)
  int comm_priority = 0;               // its priority (hipDeviceGetStreamPriorityRange's greatest)
  hipEvent_t ev_bnd = nullptr, ev_comm = nullptr;
  hipEvent_t ev_main = nullptr, ev_side = nullptr, ev_phi = nullptr;
  bool phi_mean_on_side = false;
  bool no_tail = false;                // OMG_NO_TAIL: level-by-level coarse end (A/B checks)
  bool no_fuse_up = false;             // OMG_NO_FUSE_UP: separate prolongation and first up-substep
  bool no_skip1 = false;               // OMG_NO_SKIP1: correct colour 1 before the up-smoothing too
  bool no_fuse_down = false;           // OMG_NO_FUSE_DOWN: last down-substep and residual + restriction apart
  bool no_fill_tile = false;           // OMG_NO_FILL_TILE: the per-cell ghost fill kernel everywhere
  bool no_fill_crhs = false;           // OMG_NO_FILL_CRHS: update_coarse's fill and coarse rhs as two passes
  bool no_tail_crhs = false;           // OMG_NO_TAIL_CRHS: the tail top's fill + coarse rhs by update_coarse
  bool no_rbgv = false;                // OMG_NO_RBGV: no stored refinement-boundary coarse parts
  bool no_rb_fill_fuse = false;        // OMG_NO_RB_FUSE: unfused correction + fill on refinement-boundary levels
  bool no_gs_plane = false;            // OMG_NO_GS_PLANE: lexicographic GS with the line-per-thread kernel
  bool no_fill_xl = false;             // OMG_NO_FILL_XL: the plain tiled fill after register-ring sweeps
  bool no_fuse_down_bc = false;        // OMG_NO_FUSE_DOWN_BC: no fused down-step on levels with physical / rb faces
  bool no_gs_dbl = false;              // OMG_NO_GS_DBL: a fill after every register-ring sweep (no ghost sets)
  bool no_block3 = false;              // OMG_NO_BLOCK3: one red-black substep per launch everywhere
  bool no_block3_phys = false;         // OMG_NO_BLOCK3_PHYS: no block passes on levels with physical faces
  bool no_deep = false;                // OMG_NO_DEEP: split levels keep one substep per launch (no deep halo)
  bool no_block3p = false;             // OMG_NO_BLOCK3P: correct_children by k_prolong_smooth, not k_gsrb3
  bool block4 = true;                  // the down-smoothing as k_gsrb4 + the unfused residual (OMG_NO_BLOCK4: off)
  bool no_block4p = false;             // OMG_NO_BLOCK4P: the up-smoothing's correction form with three substeps (k_gsrb3)
  bool block4_phys = false;            // OMG_BLOCK4_PHYS: k_gsrb4 also on levels with physical faces (A/B)
  bool no_defer_gc = false;            // OMG_NO_DEFER_GC: the V-cycle's last up pass writes its ghosts
  bool no_block3r = false;             // OMG_NO_BLOCK3R: no res from the coarse level's last pass (k_gsrb3 forms phi - old)
  int b3_min_boxes = omg::kB3MinBoxes;  // smallest level for k_gsrb3 (OMG_BLOCK3_MIN_BOXES, tests)
  int b3_col_small = 2;                // column length on levels below kB3MinBoxes (OMG_BLOCK3_SMALL_COL)
  int b3_col = 0;                      // k_gsrb3 column length (0: by level size; OMG_BLOCK3_COLUMN, tests)
  bool rhs_cache_valid = false;        // red acc of rhs is the sum of the current rhs
  bool phi_shift_pending = false;      // some level has shift_pending
  double* d_scalar = nullptr;          // small device scratch
  unsigned long long* d_maxslots = nullptr;   // launch_max slots (kept zeroed)
  // arguments of the coarse-tail kernel in device memory (a by-value kernel
  // argument indexed by level is copied to scratch per lane); uploaded when
  // they change
  omg::TailArgs* d_tail = nullptr;
  omg::TailArgs* h_tail = nullptr;   // the last uploaded copy (host)
  // host transport (omg_set_host_transport): the caller's messaging, staged
  // through pinned host memory
  bool host_xport = false;
  omg_host_exchange_fn hx_exchange = nullptr;
  omg_host_allgather_fn hx_allgather = nullptr;
  void* hx_user = nullptr;
  double* h_xsend = nullptr;
  double* h_xrecv = nullptr;
  size_t h_xsend_n = 0, h_xrecv_n = 0;
  bool tail_timing = false;             // OMG_TAIL_TIMING: print the tail's phase times
  long long* d_tail_stamps = nullptr;
  double* h_scalar = nullptr;          // pinned host scratch
  double* d_stage = nullptr;           // upload/download staging (reference layout)
  size_t stage_n = 0;
  omg_free_state* free_state = nullptr;   // m_free_space's free_bc (created on first use)
  // cycles as HIP graphs (run_cycle): each call is captured, its executable
  // graph updated in place and launched
  bool no_graph = true;                // unless OMG_GRAPH is set: launch kernel by kernel
  bool capturing = false;              // inside a capture: no host synchronisation
  bool max_deferred = false;           // the max residual is read after the graph ran
  std::map<int, hipGraphExec_t> graphs;   // by entry (run_cycle's key)
  int graph_fail_at = 0;               // OMG_GRAPH_FAIL (tests): inject a failure in run_cycle
  // profiling
  bool profiling = false;
  bool roctx = false;                  // OMG_ROCTX: roctx ranges per level step (rocprofv3 --marker-trace)
  // OMG_DEBUG: ghost faces start as signalling NaN, unstored edge / corner
  // cells download as signalling NaN (the reference's DEBUG=1 -finit-real=snan)
  bool debug = false;
  // OMG_CHECK_COLLECTIVE: multi-rank decisions that are made without
  // communication (rank-invariant by construction) are also agreed over the
  // transport and an error is raised when they differ (tests)
  bool check_collective = false;
  // host refinement-boundary callbacks (omg_set_refinement_bnd), per variable
  // and face: omg_rb_fn of include/omg.h and its user pointer
  void* rb_fn[omg::kMaxVars][6] = {};
  void* rb_user[omg::kMaxVars][6] = {};
  bool rbh_any = false;
  long long n_host_syncs = 0;          // host waits on a stream (host_sync; omg_host_sync_count)
  std::map<std::string, omg::KStat> stats;
  std::vector<omg::PendingEv> pending;
};
