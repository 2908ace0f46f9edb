/* omg.h — C-ABI of the MI355X-native octree-mg V-cycle (libomg.so).
 *
 * Drop-in boundary for the per-level box loops of the reference octree-mg
 * (FermiQ/octree-mg @ 2025-06-14).  The reference has no C boundary: its plug
 * points are Fortran procedure pointers called once per box
 * (mg%box_op / mg%box_smoother / mg%box_prolong, src/m_data_structures.f90:
 * 330-336, interfaces :381-407) and the per-level loops of src/m_multigrid.f90.
 * This header replaces those loops at LEVEL granularity: the host (the Fortran
 * drop-in m_multigrid in octree-mg_amd/fortran/, or the Python mirror in
 * octree-mg_amd/) hands over the mg_t tree once, and every per-level step
 * runs as HIP kernels over level-contiguous device arrays.
 *
 * Conventions
 *   - Plain C types only; every call returns 0 on success, nonzero on error
 *     with the message in omg_last_error() (the Fortran wrapper turns it into
 *     `error stop`, like the reference's error stops).
 *   - Box ids are the reference's 1-based ids; neighbour ids follow the
 *     reference encoding (>0 box, 0 = mg_no_box (refinement boundary),
 *     <0 = physical boundary / bc code).  Variables iv are 1-based
 *     (1 phi, 2 rhs, 3 old, 4 res, 5.. extra), src/m_data_structures.f90:43-65.
 *   - Box data is exchanged as the reference stores it: cc(0:nc+1,0:nc+1,
 *     0:nc+1) of one variable, Fortran column-major (i fastest).
 *   - One context per process/GPU; calls are stream-ordered on the context's
 *     stream and not re-entrant.  Multi-GPU: one rank per GPU, halos over
 *     RCCL (ncclSend/ncclRecv, xGMI), bootstrapped from omg_get_unique_id().
 */
#ifndef OMG_H
#define OMG_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct omg_ctx omg_ctx;

#define OMG_UNIQUE_ID_BYTES 128
#define OMG_DEVICE_NONE (-2)

/* Operators / smoothers / bc codes: same values as the reference
 * (src/m_data_structures.f90:14-37, 73-79). */
enum { OMG_LAPLACIAN = 1, OMG_VLAPLACIAN = 2, OMG_HELMHOLTZ = 3, OMG_VHELMHOLTZ = 4,
       OMG_AHELMHOLTZ = 5 };
enum { OMG_SMOOTHER_GS = 1, OMG_SMOOTHER_GSRB = 2 };
enum { OMG_BC_DIRICHLET = -10, OMG_BC_NEUMANN = -11, OMG_BC_CONTINUOUS = -12 };

const char *omg_last_error(void);

/* RCCL bootstrap: rank 0 calls this and broadcasts the bytes to all ranks
 * (replaces mg_comm_init's MPI set-up, src/m_communication.f90:14-35). */
int omg_get_unique_id(void *out /* OMG_UNIQUE_ID_BYTES */);

/* Loopback transport (testing the multi-rank path on ONE GPU): fills `out`
 * with an id that makes omg_ctx_create join an in-process group `tag` of
 * n_ranks contexts, one host thread each, exchanging halos by device copies
 * instead of RCCL (same plans, kernels and reduction orders). */
int omg_loopback_unique_id(long long tag, void *out /* OMG_UNIQUE_ID_BYTES */);

/* Host transport: fills `out` with an id that makes omg_ctx_create use the
 * caller's own host messaging instead of RCCL; omg_set_host_transport then
 * installs it.  For ranks that cannot use RCCL, above all several MPI ranks
 * sharing one GPU (RCCL refuses two ranks on one device): every exchange
 * stages its segments through pinned host memory and waits on the host.
 * Same plans, wire order, packing kernels and reduction orders as RCCL.  The
 * Fortran drop-in installs MPI here (m_multigrid.f90), which is the
 * reference's own transport (sort_and_transfer_buffers,
 * src/m_communication.f90:37-66; mpi_allreduce, src/m_multigrid.f90:232,255). */
int omg_host_unique_id(void *out /* OMG_UNIQUE_ID_BYTES */);
/* One grouped round: send_bufs[i] (send_counts[i] doubles) to send_peers[i],
 * receive recv_counts[i] doubles from recv_peers[i] into recv_bufs[i]; a
 * pair's messages arrive in the order they were sent (every rank makes the
 * same sequence of rounds).  Returns 0 on success. */
typedef int (*omg_host_exchange_fn)(void *user, int n_send, const int *send_peers, const long long *send_counts,
                                    const double *const *send_bufs, int n_recv, const int *recv_peers,
                                    const long long *recv_counts, double *const *recv_bufs);
/* MPI_Allgather of n doubles per rank into all (n_ranks * n, rank order). */
typedef int (*omg_host_allgather_fn)(void *user, const double *mine, int n, double *all);
int omg_set_host_transport(omg_ctx *ctx, omg_host_exchange_fn exchange, omg_host_allgather_fn allgather,
                           void *user);
/* Number of visible HIP devices (a rank count above it means ranks share a
 * GPU, where only the host transport works). */
int omg_device_count(int *n);

/* Create a context on HIP device `device` (device < 0: rank modulo the number
 * of visible devices; OMG_DEVICE_NONE: a plan-only context that builds the
 * host tables of omg_tree_setup and touches no device, for inspecting the
 * communication plans with omg_plan_transfer) for rank `rank` of `n_ranks`.  unique_id may be NULL
 * when n_ranks == 1.  Replaces the device side of mg_comm_init
 * (src/m_communication.f90:14-35). */
int omg_ctx_create(omg_ctx **ctx, int device, int rank, int n_ranks, const void *unique_id);
int omg_ctx_destroy(omg_ctx *ctx);

/* Hand over the mg_t tree (replaces the device side of mg_allocate_storage,
 * src/m_allocate_storage.f90:51-99): per-box arrays indexed by id-1
 * (children 8/box, neighbors 6/box, ix 3/box, rank 1/box), per-level arrays
 * indexed by lvl-lowest (box_size_lvl, dr 3/level) and, for every level and
 * list type t in {ids, leaves, parents, ref_bnds}, the slice
 * lists[list_off[4*(lvl-lowest)+t] .. list_off[4*(lvl-lowest)+t+1]).
 * Allocates n_vars variables for every box owned by this rank, zeroed. */
int omg_tree_setup(omg_ctx *ctx, int n_boxes, const int *lvl, const int *parent,
                   const int *children, const int *neighbors, const int *ix,
                   const int *rank, int lowest_lvl, int highest_lvl,
                   int first_normal_lvl, int box_size, const int *box_size_lvl,
                   const double *dr, const int *list_off, const int *lists,
                   int n_vars);

/* mg_set_methods equivalents (src/m_multigrid.f90:27-60; the operators'
 * *_set_methods: m_laplacian.f90:13-49, m_vlaplacian.f90:13-49,
 * m_helmholtz.f90:18-37, m_vhelmholtz.f90:19-49, m_ahelmholtz.f90:19-57;
 * lambda as helmholtz_set_lambda m_helmholtz.f90:39-46 and its v/a forms). */
int omg_set_operator(omg_ctx *ctx, int op, double lambda);
int omg_set_smoother(omg_ctx *ctx, int smoother, int n_cycle_down, int n_cycle_up,
                     int max_coarse_cycles, double residual_coarse_abs,
                     double residual_coarse_rel);
int omg_set_subtract_mean(omg_ctx *ctx, int on);

/* Replicated coarse levels (no reference counterpart: a scaling option of
 * this library, call before omg_tree_setup).  With n_ranks > 1, the lowest
 * levels, as long as each holds at most max_cells cells and has neither leaves
 * nor refinement boundaries, are kept on EVERY rank instead of being split by
 * mg%boxes(:)%rank: the restriction into the highest such level is sent to all
 * ranks and the levels below it run without any exchange (the latency-bound
 * part of a multi-GPU V-cycle).  Results are bit-identical (every box computes
 * the same arithmetic; get_sum only reads leaves).  The host still sees its
 * own partition: omg_level_size / omg_download_level cover the boxes
 * mg_load_balance gave this rank, and omg_upload_level on a replicated level
 * is collective (every rank calls it, with its own boxes, possibly none).
 * Boundary tables (omg_set_bc_faces) must cover every box of a replicated
 * level.  0 (the default) = off.  omg_replicated_level gives the highest
 * replicated level (lowest_lvl - 1: none). */
int omg_set_coarse_replication(omg_ctx *ctx, long long max_cells);
int omg_replicated_level(omg_ctx *ctx, int *lvl);

/* Boundary conditions for variable iv (mg%bc(nb, iv), src/m_data_structures
 * .f90:235-242).  omg_set_bc_faces tabulates a boundary_cond callback:
 * face_off[(id-1)*6 + nb-1] = offset of nc*nc values in data (first
 * tangential index fastest) or -1; face_type = the bc type it returned. */
int omg_set_bc(omg_ctx *ctx, int iv, int nb, int bc_type, double bc_value);
int omg_set_bc_faces(omg_ctx *ctx, int iv, const long long *face_off,
                     const int *face_type, const double *data, long long n_data);

/* Number of boxes this rank owns at lvl (size(mg%lvls(lvl)%my_ids),
 * src/m_data_structures.f90:196-206). */
int omg_level_size(omg_ctx *ctx, int lvl, int *n_boxes, int *nc);

/* Bulk copy of variable iv of all my_ids boxes at lvl, in my_ids order,
 * (nc+2)^3 doubles per box as mg%boxes(id)%cc(:,:,:,iv) stores them
 * (src/m_data_structures.f90:209-221), host memory (blocking).
 * Multi-rank: an upload of phi (iv = 1) is collective, like every other call
 * that writes the device state: each rank calls it for the level, with its own
 * boxes, possibly none.  A stand-alone omg_fas_vcycle decides on every rank
 * alike, without communication, whether its ghost fill can be skipped; a phi
 * upload made on some ranks only would make that decision differ
 * (OMG_CHECK_COLLECTIVE=1 detects it: the decision is then also agreed over
 * the transport and a mismatch is an error). */
int omg_upload_level(omg_ctx *ctx, int lvl, int iv, const double *host);
int omg_download_level(omg_ctx *ctx, int lvl, int iv, double *host);

/* The hot path.  omg_fas_vcycle = mg_fas_vcycle (src/m_multigrid.f90:150-243);
 * highest_lvl < lowest_lvl means "not present".  omg_fas_fmg = mg_fas_fmg
 * (:84-147).  max_res is written when want_max_res (the optional argument). */
int omg_fas_vcycle(omg_ctx *ctx, int highest_lvl, int want_max_res, double *max_res,
                   int standalone);
int omg_fas_fmg(omg_ctx *ctx, int have_guess, int want_max_res, double *max_res);

/* Per-level steps, each the reference routine named (all in src/). */
int omg_apply_op(omg_ctx *ctx, int i_out);            /* mg_apply_op, m_multigrid.f90:439-456 */
int omg_restrict(omg_ctx *ctx, int iv);               /* mg_restrict, m_restrict.f90:72-80 */
int omg_restrict_lvl(omg_ctx *ctx, int iv, int lvl);  /* mg_restrict_lvl, m_restrict.f90:83-114 */
int omg_fill_ghost_cells(omg_ctx *ctx, int iv);       /* mg_fill_ghost_cells, m_ghost_cells.f90:120-128 */
int omg_fill_ghost_cells_lvl(omg_ctx *ctx, int lvl, int iv);
                                                      /* mg_fill_ghost_cells_lvl, m_ghost_cells.f90:131-175 */
int omg_prolong(omg_ctx *ctx, int lvl, int iv, int iv_to, int add);
                                                      /* mg_prolong + mg_prolong_sparse, m_prolong.f90:51-85,159-240 */
int omg_smooth_boxes(omg_ctx *ctx, int lvl, int n_cycle);
                                                      /* smooth_boxes, m_multigrid.f90:404-424 */
int omg_update_coarse(omg_ctx *ctx, int lvl);         /* update_coarse, m_multigrid.f90:347-384 */
int omg_correct_children(omg_ctx *ctx, int lvl);      /* correct_children, m_multigrid.f90:387-402 */
int omg_residual_lvl(omg_ctx *ctx, int lvl);          /* residual_box over my_ids, m_multigrid.f90:426-436 */
int omg_max_residual_lvl(omg_ctx *ctx, int lvl, double *out);
                                                      /* max_residual_lvl, m_multigrid.f90:296-311 */
int omg_get_sum(omg_ctx *ctx, int iv, double *out);   /* get_sum + MPI_Allreduce, m_multigrid.f90:253-294 */
int omg_subtract_mean(omg_ctx *ctx, int iv, int include_ghostcells);
                                                      /* subtract_mean, m_multigrid.f90:245-276 */
int omg_phi_bc_store(omg_ctx *ctx);                   /* mg_phi_bc_store, m_ghost_cells.f90:66-117 */

/* m_diffusion (src/m_diffusion.f90).  omg_set_rhs: its set_rhs (:144-159),
 * rhs = f1*phi + f2*rhs on the interior of this rank's leaves.
 * omg_diffusion_solve: diffusion_solve (:19-57) for op = OMG_HELMHOLTZ,
 * diffusion_solve_vcoeff (:63-101) for OMG_VHELMHOLTZ (coefficient in var 5),
 * diffusion_solve_acoeff (:108-142) for OMG_AHELMHOLTZ (vars 5..7), which
 * take diffusion_coeff = 1.  One implicit step of order 1 or 2 on phi: the
 * context's operator and lambda are left as the reference leaves them, then
 * FMG and up to 10 V-cycles until max_res.  *n_vcycles = V-cycles after the
 * FMG, *res = the last max residual.  Errors: "order should be 1 or 2",
 * "no convergence" (the reference's error stops). */
int omg_set_rhs(omg_ctx *ctx, double f1, double f2);
int omg_diffusion_solve(omg_ctx *ctx, int op, double dt, double diffusion_coeff, int order,
                        double max_res, int *n_vcycles, double *res);

/* m_free_space (src/m_free_space.f90).  omg_poisson_free_3d is
 * mg_poisson_free_3d (:36-214): on the first call (new_rhs must be set) and
 * whenever the FFT level changes, rhs is restricted down to the highest
 * uniform level with at most max_fft_frac of the unknowns and the free-space
 * Green's function of that grid is built (PSolver's createKernel, geocode
 * 'F', poisson_3d_fft/build_kernel.f90:55-199); with new_rhs the Poisson
 * problem is solved there by FFT convolution (PSolver, psolver_main.f90:
 * 91-556), phi gets Dirichlet values interpolated from that solution on every
 * physical face of every level (ghost_cells_free_bc + mg_phi_bc_store) and
 * the solution as initial guess (restricted down, prolonged up); then one FMG
 * (fmgcycle) or V-cycle runs unless the FFT level is the highest.  r_min:
 * mg%r_min of the domain (3 doubles); box_r_min: mg%boxes(id)%r_min, 3 per
 * box indexed by id-1, or NULL (then r_min + (ix-1)*nc*dr).  Operators other
 * than the Laplacian are refused ("mg_poisson_free_3d: laplacian operator
 * required"), as is a first call without new_rhs.  The transforms run on the
 * device (hipFFT); results agree with the reference at round-off.
 * omg_free_planes: the FFT level, nx (3 ints: the FFT level's domain + 2) and,
 * if planes holds cap >= 2*(nx2*nx3 + nx1*nx3 + nx1*nx2) doubles (else
 * nothing is copied), the six boundary planes bc_x0, bc_x1 (nx2*nx3 each),
 * bc_y0, bc_y1 (nx1*nx3), bc_z0, bc_z1 (nx1*nx2), first index fastest
 * (m_free_space.f90:163-171), for host copies of the boundary callback. */
int omg_poisson_free_3d(omg_ctx *ctx, int new_rhs, double max_fft_frac, int fmgcycle,
                        int want_max_res, double *max_res, const double *r_min,
                        const double *box_r_min);
int omg_free_planes(omg_ctx *ctx, int *fft_lvl, int *nx, double *planes, long long cap);

/* The communication plan of level lvl as built by omg_tree_setup: transfer
 * `which` (0 ghost faces, 1 restriction to lvl-1, 2 prolongation from lvl-1,
 * 3 refinement-boundary faces, 4 copies of the host's boxes of a replicated
 * level), direction dir (0 send, 1 receive); fills
 * min(cap, n) (peer, key) pairs in wire order.  Keys are the ordering keys of
 * sort_and_transfer_buffers (src/m_communication.f90:37-66): 6*id+nb for
 * faces, 8*parent+child slot for restriction, child id for prolongation,
 * box id for replicated-level copies. */
int omg_plan_transfer(omg_ctx *ctx, int lvl, int which, int dir, int cap, int *peers,
                      long long *keys, int *n_items, int *item_doubles);

/* The context's communicator (no reference counterpart; mg%n_cpu of
 * mg_comm_init, src/m_communication.f90:14-35, as the transport sees it):
 * *n_ranks = the ranks it joins (ncclCommCount for RCCL), *transport = one of
 * OMG_TRANSPORT_*. */
enum { OMG_TRANSPORT_NONE = 0, OMG_TRANSPORT_RCCL = 1, OMG_TRANSPORT_LOOPBACK = 2, OMG_TRANSPORT_HOST = 3 };
int omg_comm_info(omg_ctx *ctx, int *n_ranks, int *transport);

/* Stream / timing helpers for benchmarks. */
int omg_synchronize(omg_ctx *ctx);
void *omg_stream(omg_ctx *ctx);                 /* the hipStream_t all work runs on */
/* Custom refinement-boundary ghost cells: mg%bc(nb,iv)%refinement_bnd
 * (src/m_data_structures.f90:241, interface mg_subr_rb :364-378), which
 * fill_refinement_bnd calls instead of sides_rb (src/m_ghost_cells.f90:
 * 321-325).  fn runs on the host after every ghost fill of variable iv on a
 * level with refinement-boundary faces nb (the reference calls it once per
 * fill too), with n records: ids[n] (global box ids), nbs[n] (= nb),
 * cgc[n][nc*nc] (box_gc_for_fine_neighbor's coarse face, first index
 * fastest) and cc[n][(nc+2)^3] (the box's variable iv as
 * mg%boxes(id)%cc(:,:,:,iv) stores it: the interior and the other faces'
 * ghosts current, edges and corners 0).  fn sets the ghost cells of face nb
 * in cc; only those come back.  fn = NULL restores sides_rb.  A compat path:
 * each such fill waits for the GPU and copies the boxes both ways. */
typedef void (*omg_rb_fn)(void *user, int lvl, int iv, int n, const int *ids, const int *nbs, int nc,
                          const double *cgc, double *cc);
int omg_set_refinement_bnd(omg_ctx *ctx, int iv, int nb, omg_rb_fn fn, void *user);

/* Diagnostics (no reference counterpart): the number of times the host has
 * waited for one of the context's streams so far (a multi-rank stand-alone
 * V-cycle over RCCL waits only when max_res is requested, m_multigrid.f90:
 * 226-234; the loopback transport also waits to gather the periodic mean on
 * the host), and the priority of the halo-overlap stream (the greatest of
 * hipDeviceGetStreamPriorityRange). */
int omg_host_sync_count(omg_ctx *ctx, long long *n);
int omg_comm_stream_priority(omg_ctx *ctx, int *priority);
/* Per-kernel HIP-event timing (off by default): when on, every launch of the
 * named kernel families is bracketed by events on the stream it runs on, and
 * kept per family and per family@level.  "comm" / "comm_overlap" are the
 * RCCL (or loopback) rounds on the context stream / on the halo-overlap
 * stream, with cells = doubles received.
 * Environment switches read at omg_ctx_create ("0" = off):
 *   OMG_ROCTX=1  roctx ranges per level step (rocprofv3 --marker-trace);
 *   OMG_DEBUG=1  ghost faces start as signalling NaN and unstored edge /
 *                corner cells download as signalling NaN (the reference's
 *                DEBUG=1 -finit-real=snan, makerules.make:13-17);
 *   OMG_GRAPH=1  capture each cycle as a HIP graph.
 * Failure detection: a requested max residual (omg_fas_vcycle / omg_fas_fmg /
 * omg_max_residual_lvl / omg_poisson_free_3d, and diffusion_solve's loop)
 * that is NaN or Inf is an error, "non-finite residual", with max_res still
 * written; the reference's max() drops NaN (m_multigrid.f90:226-234). */
int omg_set_profiling(omg_ctx *ctx, int on);
int omg_kernel_stats(omg_ctx *ctx, const char *name, long long *launches,
                     double *total_ms, double *cells);
int omg_reset_stats(omg_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
