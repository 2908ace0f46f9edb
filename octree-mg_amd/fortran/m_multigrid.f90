!> Drop-in m_multigrid for octree-mg, backed by the MI355X kernels of libomg.so.
!>
!> Same module name and public API as the reference's src/m_multigrid.f90
!> (mg_fas_vcycle :150-243, mg_fas_fmg :84-147, mg_set_methods :27-60,
!> mg_apply_op :439-456), so the reference's programs (tests/test_*.f90) and
!> callers compile unchanged against it.  The tree (mg_t, m_build_tree,
!> m_load_balance, m_allocate_storage) stays host Fortran; every per-level box
!> loop of the cycle runs on the GPU through the C-ABI of include/omg.h
!> (bindings in m_omg_capi.f90).
!>
!> Host/device coherence: mg%boxes(:)%cc stays the owner of the data.  Each
!> call uploads every variable of every level this rank owns, runs the cycle on
!> the device and copies phi, rhs, old and res back (interior and face ghosts;
!> edge and corner ghosts are not device state: no reference operator reads
!> them, src/m_ghost_cells.f90 never sets them).  The device context is built
!> on first use and rebuilt when the tree changes.
!>
!> Boundary conditions: mg%bc(nb, iv)%bc_type/bc_value go over as they are; a
!> boundary_cond callback is tabulated on every physical face of every box of
!> this rank at each call (the reference evaluates it at each ghost fill, with
!> the same arguments).  A refinement_bnd callback runs on the host after
!> each ghost fill of a level with such faces (rb_trampoline, through
!> omg_set_refinement_bnd).  Non-Cartesian geometry and NDIM /= 3 are
!> rejected with error stop.  All five operators
!> of the reference run on the GPU (Laplacian, Helmholtz and their variable-
!> coefficient forms via the generic kernels; aniso-Helmholtz likewise).
module m_multigrid
  use iso_c_binding
  use mpi
  use m_data_structures
  use m_prolong
  use m_omg_capi

  implicit none
  private

  type(c_ptr) :: ctx = c_null_ptr

  !> The identity of the tree the device context was built for (tree_key):
  !> every array omg_tree_setup took, plus the scalars.  A tree rebuilt after
  !> mg_deallocate_storage (AMRVAC's regrid,
  !> coupling_amrvac/mod_multigrid_coupling.t:116-130,272-351) or re-balanced
  !> can keep n_boxes and the level range while its neighbours, children,
  !> ranks and ids order change; any difference rebuilds the context and
  !> uploads the host data.
  integer(c_int), allocatable :: ctx_key(:)
  real(c_double), allocatable :: ctx_key_dr(:)

  !> The communicator of the host transport (mpi_exchange, mpi_allgather_dp)
  integer :: xport_comm = MPI_COMM_NULL

  !> Resident mode (opt-in, see mg_gpu_set_resident): the data stays on the
  !> GPU between calls instead of round-tripping through mg%boxes(:)%cc.
  logical :: resident = .false.
  logical :: device_current = .false.

  !> The mg_t of the call in progress, for the refinement_bnd callbacks the
  !> device hands back to the host (rb_trampoline); set by every public entry
  !> point that runs device work, null otherwise.
  type(mg_t), pointer :: cb_mg => null()

  integer :: timer_device_vcycle = -1
  integer :: timer_device_fmg    = -1
  integer :: timer_host_to_dev   = -1
  integer :: timer_dev_to_host   = -1

  integer, parameter :: key_head = 9   !< scalars at the head of tree_key

  public :: mg_fas_vcycle
  public :: mg_fas_fmg
  public :: mg_set_methods
  public :: mg_apply_op
  ! additions of the GPU backend (not in the reference's API)
  public :: mg_gpu_set_resident
  public :: mg_gpu_to_host
  public :: mg_gpu_to_device
  public :: mg_gpu_diffusion_solve
  public :: mg_gpu_poisson_free_3d

contains

  !> Operator/smoother selection, unchanged semantics (m_multigrid.f90:27-60):
  !> the host procedure pointers are still set (mg%box_op stays callable), and
  !> the device picks the operator from mg%operator_type at the next call.
  subroutine mg_set_methods(mg)
    use m_laplacian
    use m_vlaplacian
    use m_helmholtz
    use m_vhelmholtz
    use m_ahelmholtz
    type(mg_t), intent(inout) :: mg

    mg%box_prolong => mg_prolong_sparse

    select case (mg%operator_type)
    case (mg_laplacian)
       call laplacian_set_methods(mg)
    case (mg_vlaplacian)
       call vlaplacian_set_methods(mg)
    case (mg_helmholtz)
       call helmholtz_set_methods(mg)
    case (mg_vhelmholtz)
       call vhelmholtz_set_methods(mg)
    case (mg_ahelmholtz)
       call ahelmholtz_set_methods(mg)
    case default
       error stop "mg_set_methods: unknown operator"
    end select

    if (mg%smoother_type == mg_smoother_gsrb) then
       mg%n_smoother_substeps = 2
    else
       mg%n_smoother_substeps = 1
    end if
  end subroutine mg_set_methods

  subroutine check_methods(mg)
    type(mg_t), intent(inout) :: mg
    if (.not. associated(mg%box_op) .or. &
         .not. associated(mg%box_smoother)) then
       call mg_set_methods(mg)
    end if
  end subroutine check_methods

  subroutine add_timers(mg)
    type(mg_t), intent(inout) :: mg
    timer_device_vcycle = mg_add_timer(mg, "omg V-cycle (GPU)")
    timer_device_fmg    = mg_add_timer(mg, "omg FMG (GPU)")
    timer_host_to_dev   = mg_add_timer(mg, "omg host->GPU")
    timer_dev_to_host   = mg_add_timer(mg, "omg GPU->host")
  end subroutine add_timers

  subroutine omg_ok(ierr, what)
    integer(c_int), intent(in)   :: ierr
    character(len=*), intent(in) :: what
    if (ierr /= 0) then
       print *, "octree-mg GPU backend: ", what, ": ", omg_error_message()
       error stop "octree-mg GPU backend error"
    end if
  end subroutine omg_ok

  !> Perform FAS-FMG cycle (m_multigrid.f90:84-147) on the GPU.
  subroutine mg_fas_fmg(mg, have_guess, max_res)
    type(mg_t), intent(inout), target :: mg
    logical, intent(in)             :: have_guess
    real(dp), intent(out), optional :: max_res
    real(c_double)                  :: res
    integer(c_int)                  :: want

    call check_methods(mg)
    if (timer_device_vcycle == -1) call add_timers(mg)
    cb_mg => mg
    call sync_in(mg)
    want = merge(1_c_int, 0_c_int, present(max_res))
    call mg_timer_start(mg%timers(timer_device_fmg))
    call omg_ok(omg_fas_fmg(ctx, merge(1_c_int, 0_c_int, have_guess), want, res), &
         "mg_fas_fmg")
    nullify(cb_mg)
    call omg_ok(omg_synchronize(ctx), "synchronize")
    call mg_timer_end(mg%timers(timer_device_fmg))
    call sync_out(mg)
    if (present(max_res)) max_res = res
  end subroutine mg_fas_fmg

  !> Perform FAS V-cycle (m_multigrid.f90:150-243) on the GPU.
  subroutine mg_fas_vcycle(mg, highest_lvl, max_res, standalone)
    type(mg_t), intent(inout), target :: mg
    integer, intent(in), optional   :: highest_lvl
    real(dp), intent(out), optional :: max_res
    logical, intent(in), optional   :: standalone
    real(c_double)                  :: res
    integer(c_int)                  :: hl, sa, want

    call check_methods(mg)
    if (timer_device_vcycle == -1) call add_timers(mg)
    cb_mg => mg
    call sync_in(mg)
    hl = mg%lowest_lvl - 1              ! "absent" for the C side
    if (present(highest_lvl)) hl = highest_lvl
    sa = 1
    if (present(standalone)) sa = merge(1_c_int, 0_c_int, standalone)
    want = merge(1_c_int, 0_c_int, present(max_res))
    call mg_timer_start(mg%timers(timer_device_vcycle))
    call omg_ok(omg_fas_vcycle(ctx, hl, want, res, sa), "mg_fas_vcycle")
    nullify(cb_mg)
    call omg_ok(omg_synchronize(ctx), "synchronize")
    call mg_timer_end(mg%timers(timer_device_vcycle))
    call sync_out(mg)
    if (present(max_res)) max_res = res
  end subroutine mg_fas_vcycle

  !> Apply the operator on all levels (m_multigrid.f90:439-456).  A custom
  !> per-box `op` is a host procedure: it runs on the host boxes as before.
  subroutine mg_apply_op(mg, i_out, op)
    type(mg_t), intent(inout)      :: mg
    integer, intent(in)            :: i_out
    procedure(mg_box_op), optional :: op
    integer                        :: lvl, i, id, nc

    if (present(op)) then
       do lvl = mg%lowest_lvl, mg%highest_lvl
          nc = mg%box_size_lvl(lvl)
          do i = 1, size(mg%lvls(lvl)%my_ids)
             id = mg%lvls(lvl)%my_ids(i)
             call op(mg, id, nc, i_out)
          end do
       end do
       return
    end if
    call check_methods(mg)
    if (timer_device_vcycle == -1) call add_timers(mg)
    call sync_in(mg)
    call omg_ok(omg_apply_op(ctx, int(i_out, c_int)), "mg_apply_op")
    if (.not. resident) call copy_var_to_host(mg, i_out)
  end subroutine mg_apply_op

  !> One implicit diffusion step on the GPU for the drop-in m_diffusion
  !> (omg_diffusion_solve: lambda, set_rhs, FMG and the V-cycle loop of
  !> src/m_diffusion.f90:19-142 without a host round trip).  converged is
  !> .false. where the reference stops with "diffusion_solve: no convergence".
  subroutine mg_gpu_diffusion_solve(mg, dt, diffusion_coeff, order, max_res, converged)
    type(mg_t), intent(inout), target :: mg
    real(dp), intent(in)      :: dt, diffusion_coeff, max_res
    integer, intent(in)       :: order
    logical, intent(out)      :: converged
    integer(c_int)            :: ierr, n_v
    real(c_double)            :: res

    call check_methods(mg)
    if (timer_device_vcycle == -1) call add_timers(mg)
    cb_mg => mg
    call sync_in(mg)
    call mg_timer_start(mg%timers(timer_device_fmg))
    ierr = omg_diffusion_solve(ctx, int(mg%operator_type, c_int), real(dt, c_double), &
         real(diffusion_coeff, c_double), int(order, c_int), real(max_res, c_double), n_v, res)
    nullify(cb_mg)
    converged = ierr == 0
    if (.not. converged .and. omg_error_message() /= "diffusion_solve: no convergence") &
         call omg_ok(ierr, "diffusion_solve")
    call omg_ok(omg_synchronize(ctx), "synchronize")
    call mg_timer_end(mg%timers(timer_device_fmg))
    call sync_out(mg)
  end subroutine mg_gpu_diffusion_solve

  !> mg_poisson_free_3d's work on the GPU for the drop-in m_free_space
  !> (omg_poisson_free_3d: FFT level, Green's function, hipFFT solve,
  !> boundary table, guess, FMG or V-cycle; m_free_space.f90:36-214).  The
  !> six boundary planes come back in planes (allocated here; bc_x0, bc_x1,
  !> bc_y0, bc_y1, bc_z0, bc_z1, first index fastest) with the FFT level and
  !> its nx, for the host copy of the boundary callback.
  subroutine mg_gpu_poisson_free_3d(mg, new_rhs, max_fft_frac, fmgcycle, want, res, &
       fft_lvl, nx, planes)
    type(mg_t), intent(inout), target    :: mg
    logical, intent(in)                  :: new_rhs, fmgcycle, want
    real(dp), intent(in)                 :: max_fft_frac
    real(dp), intent(out)                :: res
    integer, intent(out)                 :: fft_lvl, nx(3)
    real(dp), allocatable, intent(inout) :: planes(:)
    real(c_double), allocatable          :: rmin(:, :)
    real(c_double)                       :: r, dummy(1)
    integer(c_int)                       :: lvl_c, nx_c(3)
    integer                              :: id

    call check_methods(mg)
    if (timer_device_vcycle == -1) call add_timers(mg)
    call sync_in(mg)
    allocate(rmin(NDIM, mg%n_boxes))
    do id = 1, mg%n_boxes
       rmin(:, id) = mg%boxes(id)%r_min
    end do
    call mg_timer_start(mg%timers(timer_device_fmg))
    cb_mg => mg
    call omg_ok(omg_poisson_free_3d(ctx, merge(1_c_int, 0_c_int, new_rhs), &
         real(max_fft_frac, c_double), merge(1_c_int, 0_c_int, fmgcycle), &
         merge(1_c_int, 0_c_int, want), r, mg%r_min, rmin), "mg_poisson_free_3d")
    nullify(cb_mg)
    call omg_ok(omg_synchronize(ctx), "synchronize")
    call mg_timer_end(mg%timers(timer_device_fmg))
    call omg_ok(omg_free_planes(ctx, lvl_c, nx_c, dummy, 0_c_long_long), "free_planes")
    fft_lvl = lvl_c
    nx = nx_c
    if (allocated(planes)) deallocate(planes)
    allocate(planes(2 * (nx(2)*nx(3) + nx(1)*nx(3) + nx(1)*nx(2))))
    call omg_ok(omg_free_planes(ctx, lvl_c, nx_c, planes, int(size(planes), c_long_long)), &
         "free_planes")
    call sync_out(mg)
    res = r
  end subroutine mg_gpu_poisson_free_3d

  !> Resident mode on/off.  When on, mg_fas_vcycle / mg_fas_fmg / mg_apply_op
  !> neither upload mg%boxes(:)%cc before nor download it after: the GPU copy
  !> is the current one until mg_gpu_to_host (after the host changed nothing)
  !> or mg_gpu_to_device (after the host changed data) is called.  Switching
  !> it off downloads the GPU state first.
  subroutine mg_gpu_set_resident(mg, on)
    type(mg_t), intent(inout) :: mg
    logical, intent(in)       :: on
    if (resident .and. .not. on .and. device_current) call to_host(mg)
    resident = on
  end subroutine mg_gpu_set_resident

  !> Copy phi, rhs, old and res of the GPU into mg%boxes(:)%cc.
  subroutine mg_gpu_to_host(mg)
    type(mg_t), intent(inout) :: mg
    if (device_current) call to_host(mg)
  end subroutine mg_gpu_to_host

  !> Copy every variable of mg%boxes(:)%cc to the GPU (and the methods and
  !> boundary conditions in mg).
  subroutine mg_gpu_to_device(mg)
    type(mg_t), intent(inout) :: mg
    call check_methods(mg)
    if (timer_device_vcycle == -1) call add_timers(mg)
    call to_device(mg)
    device_current = .true.
  end subroutine mg_gpu_to_device

  subroutine sync_in(mg)
    type(mg_t), intent(inout) :: mg
    if (resident .and. device_current) then
       if (same_tree(mg)) return
    end if
    call to_device(mg)
    device_current = .true.
  end subroutine sync_in

  subroutine sync_out(mg)
    type(mg_t), intent(inout) :: mg
    if (.not. resident) call to_host(mg)
  end subroutine sync_out

  ! ------------------------------------------------------------------------
  ! Host <-> device

  !> The tree's identity, laid out as omg_tree_setup takes it: key holds
  !> [n_boxes, n_vars, lowest_lvl, highest_lvl, first_normal_lvl, box_size,
  !> n_cpu, my_rank, n_lists, then lvl(n), parent(n), children(8,n),
  !> neighbors(6,n), ix(3,n), rank(n), box_size_lvl(nlev), list_off(4nlev+1),
  !> lists], dr holds dr(3,nlev).
  subroutine tree_key(mg, key, dr)
    type(mg_t), intent(in)                     :: mg
    integer(c_int), allocatable, intent(inout) :: key(:)
    real(c_double), allocatable, intent(inout) :: dr(:)
    integer                                    :: n, nlev, n_lists, lvl, t, p, o, id

    n = mg%n_boxes
    nlev = mg%highest_lvl - mg%lowest_lvl + 1
    n_lists = 0
    do lvl = mg%lowest_lvl, mg%highest_lvl
       n_lists = n_lists + size(mg%lvls(lvl)%ids) + size(mg%lvls(lvl)%leaves) + &
            size(mg%lvls(lvl)%parents) + size(mg%lvls(lvl)%ref_bnds)
    end do
    if (allocated(key)) deallocate(key)
    if (allocated(dr)) deallocate(dr)
    allocate(key(key_head + 20*n + nlev + 4*nlev+1 + max(n_lists, 1)), dr(NDIM*nlev))
    key(1:key_head) = [n, mg_num_vars + mg%n_extra_vars, mg%lowest_lvl, mg%highest_lvl, &
         mg%first_normal_lvl, mg%box_size, mg%n_cpu, mg%my_rank, n_lists]
    o = key_head
    do id = 1, n
       key(o + id)              = mg%boxes(id)%lvl
       key(o + n + id)          = mg%boxes(id)%parent
       key(o + 2*n + 8*(id-1) + 1 : o + 2*n + 8*id)   = mg%boxes(id)%children
       ! physical faces as mg_physical_boundary: the bc type that
       ! mg_phi_bc_store / mg_poisson_free_3d write into those slots
       ! (m_ghost_cells.f90:66-78) is device state that omg_phi_bc_store
       ! keeps, not a change of the tree
       key(o + 10*n + 6*(id-1) + 1 : o + 10*n + 6*id) = &
            merge(mg_physical_boundary, mg%boxes(id)%neighbors, mg%boxes(id)%neighbors < mg_no_box)
       key(o + 16*n + 3*(id-1) + 1 : o + 16*n + 3*id) = mg%boxes(id)%ix
       key(o + 19*n + id)       = mg%boxes(id)%rank
    end do
    o = o + 20*n
    do lvl = mg%lowest_lvl, mg%highest_lvl
       t = lvl - mg%lowest_lvl
       key(o + t + 1) = mg%box_size_lvl(lvl)
       dr(NDIM*t+1 : NDIM*t+NDIM) = mg%dr(:, lvl)
    end do
    o = o + nlev
    ! list_off (4*nlev+1 entries, starting at 0) and the lists after it
    p = 0
    key(o + 1) = 0
    do lvl = mg%lowest_lvl, mg%highest_lvl
       t = lvl - mg%lowest_lvl
       call put_list(mg%lvls(lvl)%ids, 4*t+2)
       call put_list(mg%lvls(lvl)%leaves, 4*t+3)
       call put_list(mg%lvls(lvl)%parents, 4*t+4)
       call put_list(mg%lvls(lvl)%ref_bnds, 4*t+5)
    end do
    if (n_lists == 0) key(o + 4*nlev+1 + 1) = 0

  contains

    subroutine put_list(ids, slot)
      integer, intent(in) :: ids(:)
      integer, intent(in) :: slot
      integer             :: m
      m = size(ids)
      if (m > 0) key(o + 4*nlev+1 + p + 1 : o + 4*nlev+1 + p + m) = ids
      p = p + m
      key(o + slot) = p
    end subroutine put_list
  end subroutine tree_key

  !> Whether the device context was built for this tree (tree_key), compared
  !> in place against the stored key: no key is built (about 20 ints per box,
  !> 25 MB at 262k boxes, on every call in resident mode, ADVICE r05), and the
  !> first difference ends the walk.
  logical function same_tree(mg)
    type(mg_t), intent(in) :: mg
    integer                :: n, nlev, n_lists, lvl, t, o, id, p
    same_tree = .false.
    if (.not. c_associated(ctx) .or. .not. allocated(ctx_key)) return
    n = mg%n_boxes
    nlev = mg%highest_lvl - mg%lowest_lvl + 1
    if (size(ctx_key) < key_head) return
    n_lists = 0
    do lvl = mg%lowest_lvl, mg%highest_lvl
       n_lists = n_lists + size(mg%lvls(lvl)%ids) + size(mg%lvls(lvl)%leaves) + &
            size(mg%lvls(lvl)%parents) + size(mg%lvls(lvl)%ref_bnds)
    end do
    if (size(ctx_key) /= key_head + 20*n + nlev + 4*nlev+1 + max(n_lists, 1)) return
    if (any(ctx_key(1:key_head) /= [n, mg_num_vars + mg%n_extra_vars, mg%lowest_lvl, mg%highest_lvl, &
         mg%first_normal_lvl, mg%box_size, mg%n_cpu, mg%my_rank, n_lists])) return
    o = key_head
    do id = 1, n
       if (ctx_key(o + id) /= mg%boxes(id)%lvl .or. ctx_key(o + n + id) /= mg%boxes(id)%parent .or. &
            ctx_key(o + 19*n + id) /= mg%boxes(id)%rank) return
       if (any(ctx_key(o + 2*n + 8*(id-1) + 1 : o + 2*n + 8*id) /= mg%boxes(id)%children)) return
       if (any(ctx_key(o + 10*n + 6*(id-1) + 1 : o + 10*n + 6*id) /= &
            merge(mg_physical_boundary, mg%boxes(id)%neighbors, mg%boxes(id)%neighbors < mg_no_box))) return
       if (any(ctx_key(o + 16*n + 3*(id-1) + 1 : o + 16*n + 3*id) /= mg%boxes(id)%ix)) return
    end do
    o = o + 20*n
    do lvl = mg%lowest_lvl, mg%highest_lvl
       if (ctx_key(o + lvl - mg%lowest_lvl + 1) /= mg%box_size_lvl(lvl)) return
    end do
    o = o + nlev
    p = o + 4*nlev+1
    do lvl = mg%lowest_lvl, mg%highest_lvl
       t = lvl - mg%lowest_lvl
       if (.not. same_list(mg%lvls(lvl)%ids, 4*t+2)) return
       if (.not. same_list(mg%lvls(lvl)%leaves, 4*t+3)) return
       if (.not. same_list(mg%lvls(lvl)%parents, 4*t+4)) return
       if (.not. same_list(mg%lvls(lvl)%ref_bnds, 4*t+5)) return
    end do
    ! the level spacings, compared bit for bit
    do lvl = mg%lowest_lvl, mg%highest_lvl
       t = lvl - mg%lowest_lvl
       if (any(transfer(mg%dr(:, lvl), 0_c_int64_t, NDIM) /= &
            transfer(ctx_key_dr(NDIM*t+1 : NDIM*t+NDIM), 0_c_int64_t, NDIM))) return
    end do
    same_tree = .true.

  contains

    logical function same_list(ids, slot)
      integer, intent(in) :: ids(:)
      integer, intent(in) :: slot
      integer             :: m
      m = size(ids)
      same_list = ctx_key(o + slot) == ctx_key(o + slot - 1) + m
      if (same_list .and. m > 0) same_list = all(ctx_key(p + 1 : p + m) == ids)
      p = p + m
    end function same_list
  end function same_tree

  !> Build (or rebuild) the device context for the current tree.
  subroutine attach(mg)
    type(mg_t), intent(inout)    :: mg
    integer(c_int8_t)            :: uid(omg_unique_id_bytes)
    integer(c_int), allocatable  :: key(:)
    real(c_double), allocatable  :: dr(:)
    integer                      :: n, nlev, o, ierr
    logical                      :: host_xport

#if NDIM != 3
    error stop "octree-mg GPU backend: only NDIM == 3 is supported"
#endif
    if (.not. mg%is_allocated) error stop "mg_fas_vcycle: storage not allocated"
    if (mg%geometry_type /= mg_cartesian) &
         error stop "octree-mg GPU backend: only Cartesian geometry is supported"

    if (same_tree(mg)) return
    if (c_associated(ctx)) call omg_ok(omg_ctx_destroy(ctx), "ctx_destroy")
    ctx = c_null_ptr
    if (allocated(ctx_key)) deallocate(ctx_key)

    uid = 0
    host_xport = .false.
    if (mg%n_cpu > 1) then
       host_xport = use_host_transport(mg)
       if (host_xport) then
          call omg_ok(omg_host_unique_id(uid), "host_unique_id")
       else
          if (mg%my_rank == 0) call omg_ok(omg_get_unique_id(uid), "get_unique_id")
          call mpi_bcast(uid, omg_unique_id_bytes, MPI_BYTE, 0, mg%comm, ierr)
       end if
    end if
    call omg_ok(omg_ctx_create(ctx, -1_c_int, int(mg%my_rank, c_int), &
         int(mg%n_cpu, c_int), uid), "ctx_create")
    if (host_xport) then
       xport_comm = mg%comm
       call omg_ok(omg_set_host_transport(ctx, c_funloc(mpi_exchange), c_funloc(mpi_allgather_dp), &
            c_null_ptr), "set_host_transport")
    end if

    call tree_key(mg, key, dr)
    n = mg%n_boxes
    nlev = mg%highest_lvl - mg%lowest_lvl + 1
    o = key_head
    call omg_ok(omg_tree_setup(ctx, int(n, c_int), key(o+1:), key(o+n+1:), key(o+2*n+1:), &
         key(o+10*n+1:), key(o+16*n+1:), key(o+19*n+1:), &
         int(mg%lowest_lvl, c_int), int(mg%highest_lvl, c_int), &
         int(mg%first_normal_lvl, c_int), int(mg%box_size, c_int), key(o+20*n+1:), dr, &
         key(o+20*n+nlev+1:), key(o+20*n+nlev+4*nlev+1+1:), key(2)), "tree_setup")
    call move_alloc(key, ctx_key)
    call move_alloc(dr, ctx_key_dr)
  end subroutine attach

  !> Methods, boundary conditions and all data of this rank onto the device.
  subroutine to_device(mg)
    use m_helmholtz, only: helmholtz_lambda
    use m_vhelmholtz, only: vhelmholtz_lambda
    use m_ahelmholtz, only: ahelmholtz_lambda
    type(mg_t), intent(inout) :: mg
    real(c_double)            :: lambda
    integer                   :: iv, nb, lvl, n_vars

    call attach(mg)
    call mg_timer_start(mg%timers(timer_host_to_dev))

    select case (mg%operator_type)
    case (mg_laplacian, mg_vlaplacian)
       lambda = 0.0_dp
    case (mg_helmholtz)
       lambda = helmholtz_lambda
    case (mg_vhelmholtz)
       lambda = vhelmholtz_lambda
    case (mg_ahelmholtz)
       lambda = ahelmholtz_lambda
    case default
       error stop "octree-mg GPU backend: unknown operator"
    end select
    call omg_ok(omg_set_operator(ctx, int(mg%operator_type, c_int), lambda), "set_operator")
    call omg_ok(omg_set_smoother(ctx, int(mg%smoother_type, c_int), &
         int(mg%n_cycle_down, c_int), int(mg%n_cycle_up, c_int), &
         int(mg%max_coarse_cycles, c_int), real(mg%residual_coarse_abs, c_double), &
         real(mg%residual_coarse_rel, c_double)), "set_smoother")
    call omg_ok(omg_set_subtract_mean(ctx, merge(1_c_int, 0_c_int, mg%subtract_mean)), &
         "set_subtract_mean")

    n_vars = mg_num_vars + mg%n_extra_vars
    do iv = 1, n_vars
       do nb = 1, mg_num_neighbors
          if (associated(mg%bc(nb, iv)%refinement_bnd)) then
             call omg_ok(omg_set_refinement_bnd(ctx, int(iv, c_int), int(nb, c_int), &
                  c_funloc(rb_trampoline), c_null_ptr), "set_refinement_bnd")
          else
             call omg_ok(omg_set_refinement_bnd(ctx, int(iv, c_int), int(nb, c_int), &
                  c_null_funptr, c_null_ptr), "set_refinement_bnd")
          end if
          call omg_ok(omg_set_bc(ctx, int(iv, c_int), int(nb, c_int), &
               int(mg%bc(nb, iv)%bc_type, c_int), real(mg%bc(nb, iv)%bc_value, c_double)), &
               "set_bc")
       end do
       if (any([(associated(mg%bc(nb, iv)%boundary_cond), nb = 1, mg_num_neighbors)])) &
            call tabulate_bc(mg, iv)
    end do

    do lvl = mg%lowest_lvl, mg%highest_lvl
       do iv = 1, n_vars
          call copy_level(mg, lvl, iv, .true.)
       end do
    end do
    ! mg_phi_bc_store's data sits in the uploaded rhs ghost cells; the device
    ! flag follows the host one (m_ghost_cells.f90:66-78, 266-270)
    if (mg%phi_bc_data_stored) call omg_ok(omg_phi_bc_store(ctx), "phi_bc_store")
    call mg_timer_end(mg%timers(timer_host_to_dev))
  end subroutine to_device

  !> phi, rhs, old and res of every level back into mg%boxes(:)%cc.
  subroutine to_host(mg)
    type(mg_t), intent(inout) :: mg
    integer                   :: lvl, iv
    call mg_timer_start(mg%timers(timer_dev_to_host))
    do lvl = mg%lowest_lvl, mg%highest_lvl
       do iv = 1, mg_num_vars
          call copy_level(mg, lvl, iv, .false.)
       end do
    end do
    call mg_timer_end(mg%timers(timer_dev_to_host))
  end subroutine to_host

  subroutine copy_var_to_host(mg, iv)
    type(mg_t), intent(inout) :: mg
    integer, intent(in)       :: iv
    integer                   :: lvl
    do lvl = mg%lowest_lvl, mg%highest_lvl
       call copy_level(mg, lvl, iv, .false.)
    end do
  end subroutine copy_var_to_host

  !> One variable of all my boxes at lvl, in my_ids order, (nc+2)^3 per box.
  subroutine copy_level(mg, lvl, iv, up)
    type(mg_t), intent(inout)   :: mg
    integer, intent(in)         :: lvl, iv
    logical, intent(in)         :: up
    real(c_double), allocatable :: buf(:, :, :, :)
    integer                     :: i, id, nc, n

    n = size(mg%lvls(lvl)%my_ids)
    nc = mg%box_size_lvl(lvl)
    if (n == 0) then
       ! uploads are collective (include/omg.h): a rank without boxes here
       ! still makes the call
       if (up) then
          allocate(buf(1, 1, 1, 1))
          call omg_ok(omg_upload_level(ctx, int(lvl, c_int), int(iv, c_int), buf), "upload_level")
       end if
       return
    end if
    allocate(buf(0:nc+1, 0:nc+1, 0:nc+1, n))
    if (up) then
       do i = 1, n
          id = mg%lvls(lvl)%my_ids(i)
          buf(:, :, :, i) = mg%boxes(id)%cc(:, :, :, iv)
       end do
       call omg_ok(omg_upload_level(ctx, int(lvl, c_int), int(iv, c_int), buf), "upload_level")
    else
       call omg_ok(omg_download_level(ctx, int(lvl, c_int), int(iv, c_int), buf), &
            "download_level")
       do i = 1, n
          id = mg%lvls(lvl)%my_ids(i)
          associate (cc => mg%boxes(id)%cc)
            cc(1:nc, 1:nc, 1:nc, iv) = buf(1:nc, 1:nc, 1:nc, i)
            cc(0, 1:nc, 1:nc, iv)    = buf(0, 1:nc, 1:nc, i)
            cc(nc+1, 1:nc, 1:nc, iv) = buf(nc+1, 1:nc, 1:nc, i)
            cc(1:nc, 0, 1:nc, iv)    = buf(1:nc, 0, 1:nc, i)
            cc(1:nc, nc+1, 1:nc, iv) = buf(1:nc, nc+1, 1:nc, i)
            cc(1:nc, 1:nc, 0, iv)    = buf(1:nc, 1:nc, 0, i)
            cc(1:nc, 1:nc, nc+1, iv) = buf(1:nc, 1:nc, nc+1, i)
          end associate
       end do
    end if
  end subroutine copy_level

  !> Evaluate the boundary_cond callbacks of variable iv on every physical
  !> face of my boxes (set_ghost_cells' call, m_ghost_cells.f90:264-278).
  subroutine tabulate_bc(mg, iv)
    type(mg_t), intent(inout)         :: mg
    integer, intent(in)               :: iv
    integer(c_long_long), allocatable :: face_off(:)
    integer(c_int), allocatable       :: face_type(:)
    real(c_double), allocatable       :: data(:)
    real(dp), allocatable             :: bc(:, :)
    integer                           :: lvl, i, id, nb, nc, bc_type
    integer(c_long_long)              :: n_data, m

    allocate(face_off(6 * mg%n_boxes), face_type(6 * mg%n_boxes))
    face_off  = -1
    face_type = 0
    n_data = 0
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do i = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(i)
          do nb = 1, mg_num_neighbors
             if (mg%boxes(id)%neighbors(nb) < mg_no_box .and. &
                  associated(mg%bc(nb, iv)%boundary_cond)) n_data = n_data + nc * nc
          end do
       end do
    end do
    allocate(data(max(n_data, 1_c_long_long)))
    m = 0
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       allocate(bc(nc, nc))
       do i = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(i)
          do nb = 1, mg_num_neighbors
             if (mg%boxes(id)%neighbors(nb) < mg_no_box .and. &
                  associated(mg%bc(nb, iv)%boundary_cond)) then
                call mg%bc(nb, iv)%boundary_cond(mg%boxes(id), nc, iv, nb, bc_type, bc)
                face_off(6*(id-1) + nb) = m
                face_type(6*(id-1) + nb) = bc_type
                data(m+1:m+nc*nc) = reshape(bc, [nc*nc])
                m = m + nc * nc
             end if
          end do
       end do
       deallocate(bc)
    end do
    call omg_ok(omg_set_bc_faces(ctx, int(iv, c_int), face_off, face_type, data, n_data), &
         "set_bc_faces")
  end subroutine tabulate_bc

  !> The transport of a multi-rank context.  RCCL (xGMI) when every rank has
  !> a GPU of its own; the host transport over MPI, the reference's own
  !> transport (sort_and_transfer_buffers, m_communication.f90:37-66;
  !> mpi_allreduce, m_multigrid.f90:232,255), when ranks share a GPU (RCCL
  !> refuses two ranks on one device) or when OMG_TRANSPORT=host is set.
  !> Decided alike on every rank.  The GPUs a rank sees are its node's, so
  !> they are compared with the ranks on the same node (MPI_COMM_TYPE_SHARED),
  !> not with mg%n_cpu: 2 nodes x 8 GPUs run 16 ranks on RCCL.
  logical function use_host_transport(mg)
    type(mg_t), intent(in) :: mg
    integer(c_int)         :: nd
    integer                :: mine, lowest, ierr, ln, st, node_comm, n_node
    character(len=16)      :: env
    call get_environment_variable("OMG_TRANSPORT", env, ln, st)
    mine = 0
    if (st == 0 .and. trim(env) == "host") mine = 1
    call omg_ok(omg_device_count(nd), "device_count")
    call mpi_comm_split_type(mg%comm, MPI_COMM_TYPE_SHARED, mg%my_rank, MPI_INFO_NULL, node_comm, ierr)
    call mpi_comm_size(node_comm, n_node, ierr)
    call mpi_comm_free(node_comm, ierr)
    if (nd < n_node) mine = 1
    call mpi_allreduce(mine, lowest, 1, MPI_INTEGER, MPI_MAX, mg%comm, ierr)
    use_host_transport = lowest == 1
  end function use_host_transport

  !> omg_host_exchange_fn over MPI: nonblocking sends and receives of one
  !> round, then a wait on all (messages of a pair keep their order: same
  !> communicator, same tag).
  integer(c_int) function mpi_exchange(user, n_send, send_peers, send_counts, send_bufs, &
       n_recv, recv_peers, recv_counts, recv_bufs) bind(C)
    type(c_ptr), value            :: user
    integer(c_int), value         :: n_send, n_recv
    integer(c_int), intent(in)    :: send_peers(*), recv_peers(*)
    integer(c_long_long), intent(in) :: send_counts(*), recv_counts(*)
    type(c_ptr), intent(in)       :: send_bufs(*), recv_bufs(*)
    real(c_double), pointer       :: buf(:)
    integer, allocatable          :: req(:)
    integer                       :: i, ierr, nreq
    integer, parameter            :: tag = 7291

    allocate(req(max(n_send + n_recv, 1)))
    nreq = 0
    do i = 1, n_recv
       call c_f_pointer(recv_bufs(i), buf, [recv_counts(i)])
       nreq = nreq + 1
       call mpi_irecv(buf, int(recv_counts(i)), MPI_DOUBLE_PRECISION, int(recv_peers(i)), tag, &
            xport_comm, req(nreq), ierr)
    end do
    do i = 1, n_send
       call c_f_pointer(send_bufs(i), buf, [send_counts(i)])
       nreq = nreq + 1
       call mpi_isend(buf, int(send_counts(i)), MPI_DOUBLE_PRECISION, int(send_peers(i)), tag, &
            xport_comm, req(nreq), ierr)
    end do
    call mpi_waitall(nreq, req, MPI_STATUSES_IGNORE, ierr)
    mpi_exchange = int(ierr, c_int)
  end function mpi_exchange

  !> omg_host_allgather_fn over MPI
  integer(c_int) function mpi_allgather_dp(user, mine, n, all) bind(C)
    type(c_ptr), value         :: user
    integer(c_int), value      :: n
    real(c_double), intent(in) :: mine(n)
    real(c_double), intent(out) :: all(*)
    integer                    :: ierr
    call mpi_allgather(mine, int(n), MPI_DOUBLE_PRECISION, all, int(n), MPI_DOUBLE_PRECISION, &
         xport_comm, ierr)
    mpi_allgather_dp = int(ierr, c_int)
  end function mpi_allgather_dp

  !> The device's refinement_bnd hand-back (omg_set_refinement_bnd): for
  !> each record, the box's variable iv (reference layout) goes into
  !> mg%boxes(id)%cc for the callback, which the reference calls as
  !> fill_refinement_bnd does (m_ghost_cells.f90:321-325); the ghosts it sets
  !> come back in cc, and the host box keeps what it held before.
  subroutine rb_trampoline(user, lvl, iv, n, ids, nbs, nc, cgc, cc) bind(C)
    type(c_ptr), value            :: user
    integer(c_int), value         :: lvl, iv, n, nc
    integer(c_int), intent(in)    :: ids(n), nbs(n)
    real(c_double), intent(in)    :: cgc(nc, nc, n)
    real(c_double), intent(inout) :: cc(0:nc+1, 0:nc+1, 0:nc+1, n)
    real(dp), allocatable         :: keep(:, :, :)
    integer                       :: k, id, nb

    if (.not. associated(cb_mg)) error stop "octree-mg GPU backend: refinement_bnd outside a call"
    do k = 1, n
       id = ids(k)
       nb = nbs(k)
       keep = cb_mg%boxes(id)%cc(:, :, :, iv)
       cb_mg%boxes(id)%cc(:, :, :, iv) = cc(:, :, :, k)
       call cb_mg%bc(nb, iv)%refinement_bnd(cb_mg%boxes(id), int(nc), int(iv), nb, cgc(:, :, k))
       cc(:, :, :, k) = cb_mg%boxes(id)%cc(:, :, :, iv)
       cb_mg%boxes(id)%cc(:, :, :, iv) = keep
    end do
  end subroutine rb_trampoline

end module m_multigrid
