! TEST INFRASTRUCTURE — golden-vector generator (oracle/_ref build only).
!
! Drives the REFERENCE octree-mg (compiled from /root/reference/src by
! oracle/Makefile) through the same problem set-ups the reference's own tests
! use, and prints every per-iteration scalar as the exact IEEE-754 bit pattern
! so the fixtures in tests/golden/ pin parity bit-for-bit.
!
! Set-ups restated from the reference tests:
!   * manufactured solution u = prod(sin(2*pi*5*x)) and rhs = box_op(u) on
!     every level          (tests/test_uniform_grid.f90:132-170)
!   * callback Dirichlet BC with the solution on the faces
!                          (tests/test_uniform_grid.f90:204-239)
!   * rhs = 1, Dirichlet 0 (tests/test_performance.f90:55-56,102-115)
!   * centre-refined AMR tree (tests/test_refinement.f90:191-247), ghost cells
!     of u via mg_restrict + mg_fill_ghost_cells (:141-144)
!
! Usage (positional):
!   omg_golden box nx ny nz n_its cycle smoother op lambda bc rhs n_levels lb maxres dump
!     cycle    v | f | d1 | d2  (d1/d2: one m_diffusion time step of order
!              1/2 per iteration, dt = the lambda argument; op helm ->
!              diffusion_solve with D = 0.5, vhelm -> diffusion_solve_vcoeff,
!              ahelm -> diffusion_solve_acoeff; max_res 1e-8)
!     smoother gs | gsrb
!     op       lpl | helm | vlpl | vhelm   (v*: coefficient eps in var 5, solution in 6)
!              | ahelm (eps1..3 in vars 5..7, solution in 8; the dump holds rhs)
!     bc       sol (callback Dirichlet u) | d0 (Dirichlet 0) | per (periodic)
!              | n0 (Neumann 0) | c0 (continuous) | mx1, mx2 (per-face types
!              and constant values, tests/mgdriver.py MIXED_BC)
!     rhs      sol (rhs = L u) | one (rhs = 1) | phi (phi = u incl. ghosts,
!              rhs = 0: the initial state of a diffusion run)
!     n_levels 1 = uniform, >1 = test_refinement's AMR tree
!     lb       lb (mg_load_balance) | lbp (+ mg_load_balance_parents);
!              a trailing "rb" (lbrb, lbprb) installs a custom refinement_bnd
!              callback for phi (custom_rb: sides_rb's form with other
!              coefficients, m_ghost_cells.f90:769-861); a trailing "mv"
!              (lbmv, lbpmv) rebuilds the tree after the n_its iterations as
!              AMRVAC's regrid does (coupling_amrvac/mod_multigrid_coupling.t:
!              116-130,272-351): mg_deallocate_storage, the same AMR tree with
!              its refined region moved (+1/4 of the domain in x, -1/4 in y:
!              same box count, other neighbours, children, ranks and ids
!              order), load balance, mg_allocate_storage, the problem set up
!              again and n_its more iterations (a second IT 0.. block)
!     maxres   0 | 1  (request max_res from mg_fas_vcycle/mg_fas_fmg)
!     dump     x, or a file: final phi interior of every box (ids order per
!              level, lowest..highest, i fastest), raw float64; with more
!              than one rank every rank writes <file>.r<rank>: per box it
!              owns, int32 lvl, int32 position in lvls(lvl)%ids, int32 nc,
!              then the nc^3 doubles (tests/golden/make_golden.py reassembles
!              the one-rank order)
#include "cpp_macros.h"
program omg_golden
  use mpi
  use m_octree_mg
  use m_diffusion
  implicit none

  integer, parameter  :: i8k = selected_int_kind(18)
  integer             :: n_modes(NDIM) = 5
  integer             :: box_size, domain_size(NDIM), n_its, n_levels
  real(dp)            :: dr(NDIM), r_min(NDIM) = 0.0_dp, lambda
  logical             :: periodic(NDIM) = .false.
  real(dp), parameter :: pi = acos(-1.0_dp)
  character(len=64)   :: a_cycle, a_smoother, a_op, a_bc, a_rhs, a_lb, a_dump, arg
  integer             :: n, ierr, maxres_flag, i_sol, order, n_tree, n_trees
  real(dp)            :: shift(NDIM) = 0.0_dp
  real(dp)            :: max_res, t0, t1
  real(dp), parameter :: diff_coeff = 0.5_dp, diff_tol = 1.0e-8_dp
  type(mg_t)          :: mg

  if (command_argument_count() < 15) error stop "omg_golden: need 15 args"
  call get_command_argument(1, arg); read(arg, *) box_size
  do n = 1, NDIM
     call get_command_argument(1+n, arg); read(arg, *) domain_size(n)
  end do
  call get_command_argument(5, arg); read(arg, *) n_its
  call get_command_argument(6, a_cycle)
  call get_command_argument(7, a_smoother)
  call get_command_argument(8, a_op)
  call get_command_argument(9, arg); read(arg, *) lambda
  call get_command_argument(10, a_bc)
  call get_command_argument(11, a_rhs)
  call get_command_argument(12, arg); read(arg, *) n_levels
  call get_command_argument(13, a_lb)
  call get_command_argument(14, arg); read(arg, *) maxres_flag
  a_dump = ""
  call get_command_argument(15, arg)
  if (trim(arg) /= "x") a_dump = arg

  dr = 1.0_dp / domain_size
  mg%n_extra_vars = 1
  i_sol = mg_num_vars + 1

  mg%geometry_type = mg_cartesian
  if (trim(a_op) == "helm") then
     mg%operator_type = mg_helmholtz
     call helmholtz_set_lambda(lambda)
  else if (trim(a_op) == "ahelm") then
     ! eps1..3 in vars 5..7 (mg_iveps1..3), the solution in 8; the smoother
     ! box_gs_ahelmh is broken in 3D (a0(4:5), m_ahelmholtz.f90:145), so only
     ! the operator is pinned: run with n_its = 0, the dump holds rhs = L(u)
     mg%n_extra_vars = 4
     i_sol = mg_num_vars + 4
     mg%operator_type = mg_ahelmholtz
     call ahelmholtz_set_lambda(lambda)
  else if (trim(a_op) == "vlpl" .or. trim(a_op) == "vhelm") then
     ! variable coefficient eps in mg_iveps (= 5): the solution moves to 6
     mg%n_extra_vars = 2
     i_sol = mg_num_vars + 2
     if (trim(a_op) == "vlpl") then
        mg%operator_type = mg_vlaplacian
     else
        mg%operator_type = mg_vhelmholtz
        call vhelmholtz_set_lambda(lambda)
     end if
  else
     mg%operator_type = mg_laplacian
  end if
  if (trim(a_smoother) == "gsrb") then
     mg%smoother_type = mg_smoother_gsrb
  else
     mg%smoother_type = mg_smoother_gs
  end if

  select case (trim(a_bc))
  case ("sol")
     do n = 1, mg_num_neighbors
        mg%bc(n, mg_iphi)%boundary_cond => sol_boundary_condition
     end do
  case ("d0")
     mg%bc(:, mg_iphi)%bc_type = mg_bc_dirichlet
     mg%bc(:, mg_iphi)%bc_value = 0.0_dp
  case ("per")
     periodic = .true.
  case ("n0")
     mg%bc(:, mg_iphi)%bc_type = mg_bc_neumann
     mg%bc(:, mg_iphi)%bc_value = 0.0_dp
  case ("c0")
     mg%bc(:, mg_iphi)%bc_type = mg_bc_continuous
     mg%bc(:, mg_iphi)%bc_value = 0.0_dp
  case ("mx1")
     ! per-face types and constant values (tests/mgdriver.py MIXED_BC)
     mg%bc(:, mg_iphi)%bc_type = [mg_bc_dirichlet, mg_bc_dirichlet, mg_bc_neumann, &
          mg_bc_neumann, mg_bc_continuous, mg_bc_continuous]
     mg%bc(:, mg_iphi)%bc_value = [0.5_dp, -1.25_dp, 0.75_dp, -0.3_dp, 0.2_dp, 0.0_dp]
  case ("mx2")
     mg%bc(:, mg_iphi)%bc_type = [mg_bc_continuous, mg_bc_neumann, mg_bc_dirichlet, &
          mg_bc_continuous, mg_bc_neumann, mg_bc_dirichlet]
     mg%bc(:, mg_iphi)%bc_value = [0.0_dp, 1.5_dp, -0.625_dp, 0.0_dp, -2.0_dp, 0.125_dp]
  case default
     error stop "bad bc"
  end select

  call mg_set_methods(mg)
  call mg_comm_init(mg)

  n = len_trim(a_lb)
  n_trees = 1
  if (n > 2) then
     if (a_lb(n-1:n) == "mv") n_trees = 2
  end if

  do n_tree = 1, n_trees
  if (n_tree == 2) then
     ! AMRVAC's regrid: free the storage, build the new tree, balance, allocate
     call mg_deallocate_storage(mg)
     shift = [0.25_dp, -0.25_dp, 0.0_dp]
  end if
  if (n_levels <= 1) then
     call mg_build_rectangle(mg, domain_size, box_size, dr, r_min, periodic, 0)
  else
     call build_amr_tree(mg, n_levels, domain_size, box_size, dr, periodic)
  end if
  call mg_load_balance(mg)
  if (a_lb(1:3) == "lbp") call mg_load_balance_parents(mg)
  n = len_trim(a_lb)
  if (n > 2) then
     if (a_lb(n-1:n) == "rb") then
        do ierr = 1, mg_num_neighbors
           mg%bc(ierr, mg_iphi)%refinement_bnd => custom_rb
        end do
     end if
  end if
  call mg_allocate_storage(mg)
#ifdef OMG_GPU_RESIDENT
  ! GPU drop-in only (octree-mg_amd/fortran): data stays on the GPU between
  ! cycles; the host copy is refreshed before every print_state
  call mg_gpu_set_resident(mg, .true.)
#endif

  if (mg%operator_type == mg_vlaplacian .or. mg%operator_type == mg_vhelmholtz) call set_eps(mg)
  if (mg%operator_type == mg_ahelmholtz) call set_eps3(mg)
  if (trim(a_rhs) == "sol") then
     call set_solution(mg, n_levels > 1)
     call compute_rhs_and_reset(mg)
  else if (trim(a_rhs) == "phi") then
     call set_solution(mg, n_levels > 1)
     call copy_solution_to_phi(mg)
  else
     call set_rhs_one(mg)
  end if

  call print_state(mg, 0, 0.0_dp)
  t0 = mpi_wtime()
  do n = 1, n_its
     max_res = 0.0_dp
     if (a_cycle(1:1) == "d") then
        read(a_cycle(2:2), *) order
        if (mg%operator_type == mg_helmholtz) then
           call diffusion_solve(mg, lambda, diff_coeff, order, diff_tol)
        else if (mg%operator_type == mg_vhelmholtz) then
           call diffusion_solve_vcoeff(mg, lambda, order, diff_tol)
        else
           call diffusion_solve_acoeff(mg, lambda, order, diff_tol)
        end if
     else if (trim(a_cycle) == "f") then
        if (maxres_flag == 1) then
           call mg_fas_fmg(mg, n > 1, max_res)
        else
           call mg_fas_fmg(mg, n > 1)
        end if
     else
        if (maxres_flag == 1) then
           call mg_fas_vcycle(mg, max_res=max_res)
        else
           call mg_fas_vcycle(mg)
        end if
     end if
#ifdef OMG_GPU_RESIDENT
     call mg_gpu_to_host(mg)
#endif
     call print_state(mg, n, max_res)
  end do
  t1 = mpi_wtime()
  if (mg%my_rank == 0) write(*, '(A,ES25.17,A,I0)') "TIME", (t1 - t0) / max(n_its, 1), " NCPU ", mg%n_cpu
  end do

  if (len_trim(a_dump) > 0) then
     if (mg%n_cpu == 1) then
        call dump_phi(mg, trim(a_dump))
     else
        call dump_phi_rank(mg, trim(a_dump))
     end if
  end if

  call mpi_barrier(mpi_comm_world, ierr)
  call mpi_finalize(ierr)

contains

  real(dp) function solution(r)
    real(dp), intent(in) :: r(NDIM)
    solution = product(sin(2 * pi * n_modes * r))
  end function solution

  subroutine set_solution(mg, refined)
    type(mg_t), intent(inout) :: mg
    logical, intent(in)       :: refined
    integer                   :: n, id, lvl, nc, IJK
    real(dp)                  :: r(NDIM)
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(n)
          do KJI_DO(0, nc+1)
             r = mg%boxes(id)%r_min + ([IJK] - 0.5_dp) * mg%dr(:, lvl)
             mg%boxes(id)%cc(IJK, i_sol) = solution(r)
          end do; CLOSE_DO
       end do
    end do
    if (refined) then
       call mg_restrict(mg, i_sol)
       call mg_fill_ghost_cells(mg, i_sol)
    end if
  end subroutine set_solution

  ! eps = (1.5 + sin(2 pi x)) (1.5 + sin(2 pi y)) (1.5 + sin(2 pi z)) on every
  ! cell incl. ghosts of every level (products only: no contraction)
  subroutine set_eps(mg)
    type(mg_t), intent(inout) :: mg
    integer                   :: n, id, lvl, nc, IJK
    real(dp)                  :: r(NDIM)
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(n)
          do KJI_DO(0, nc+1)
             r = mg%boxes(id)%r_min + ([IJK] - 0.5_dp) * mg%dr(:, lvl)
             mg%boxes(id)%cc(IJK, mg_iveps) = (1.5_dp + sin(2 * pi * r(1))) * &
                  (1.5_dp + sin(2 * pi * r(2))) * (1.5_dp + sin(2 * pi * r(3)))
          end do; CLOSE_DO
       end do
    end do
  end subroutine set_eps

  ! aniso: eps_d = eps * d (d = 1, 2, 3) in mg_iveps1..3
  subroutine set_eps3(mg)
    type(mg_t), intent(inout) :: mg
    integer                   :: n, id, lvl, nc, IJK, d
    real(dp)                  :: r(NDIM), e
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(n)
          do KJI_DO(0, nc+1)
             r = mg%boxes(id)%r_min + ([IJK] - 0.5_dp) * mg%dr(:, lvl)
             e = (1.5_dp + sin(2 * pi * r(1))) * (1.5_dp + sin(2 * pi * r(2))) * &
                  (1.5_dp + sin(2 * pi * r(3)))
             do d = 1, NDIM
                mg%boxes(id)%cc(IJK, mg_iveps1 + d - 1) = e * d
             end do
          end do; CLOSE_DO
       end do
    end do
  end subroutine set_eps3

  subroutine compute_rhs_and_reset(mg)
    type(mg_t), intent(inout) :: mg
    integer                   :: n, id, lvl, nc
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(n)
          mg%boxes(id)%cc(DTIMES(:), mg_iphi) = mg%boxes(id)%cc(DTIMES(:), i_sol)
          call mg%box_op(mg, id, nc, mg_irhs)
          mg%boxes(id)%cc(DTIMES(:), mg_iphi) = 0.0_dp
       end do
    end do
  end subroutine compute_rhs_and_reset

  subroutine copy_solution_to_phi(mg)
    type(mg_t), intent(inout) :: mg
    integer                   :: n, id, lvl
    do lvl = mg%lowest_lvl, mg%highest_lvl
       do n = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(n)
          mg%boxes(id)%cc(DTIMES(:), mg_iphi) = mg%boxes(id)%cc(DTIMES(:), i_sol)
       end do
    end do
  end subroutine copy_solution_to_phi

  subroutine set_rhs_one(mg)
    type(mg_t), intent(inout) :: mg
    integer                   :: n, id, lvl, nc, IJK
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(n)
          do KJI_DO(1, nc)
             mg%boxes(id)%cc(IJK, mg_irhs) = 1.0_dp
             mg%boxes(id)%cc(IJK, i_sol) = 0.0_dp
          end do; CLOSE_DO
       end do
    end do
  end subroutine set_rhs_one

  ! max |phi - u| and max |res| over the leaves of levels >= 1, reduced with
  ! MPI_MAX (exact under any order).  Scalars are printed as IEEE bit patterns.
  subroutine print_state(mg, it, mres)
    type(mg_t), intent(inout) :: mg
    integer, intent(in)       :: it
    real(dp), intent(in)      :: mres
    integer                   :: n, nc, id, lvl, IJK, ierr
    real(dp)                  :: err, res, gerr, gres
    err = 0.0_dp
    res = 0.0_dp
    do lvl = 1, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%my_leaves)
          id = mg%lvls(lvl)%my_leaves(n)
          do KJI_DO(1, nc)
             err = max(err, abs(mg%boxes(id)%cc(IJK, mg_iphi) - mg%boxes(id)%cc(IJK, i_sol)))
             res = max(res, abs(mg%boxes(id)%cc(IJK, mg_ires)))
          end do; CLOSE_DO
       end do
    end do
    call mpi_reduce(err, gerr, 1, MPI_DOUBLE_PRECISION, MPI_MAX, 0, mpi_comm_world, ierr)
    call mpi_reduce(res, gres, 1, MPI_DOUBLE_PRECISION, MPI_MAX, 0, mpi_comm_world, ierr)
    if (mg%my_rank == 0) write(*, '(A,I4,3(1X,Z16.16),3(1X,ES25.17))') "IT", it, &
         transfer(gerr, 0_i8k), transfer(gres, 0_i8k), transfer(mres, 0_i8k), gerr, gres, mres
  end subroutine print_state

  subroutine dump_phi(mg, fname)
    type(mg_t), intent(inout) :: mg
    character(len=*), intent(in) :: fname
    integer :: u, n, id, lvl, nc
    open(newunit=u, file=fname, access="stream", form="unformatted", status="replace")
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%ids)
          id = mg%lvls(lvl)%ids(n)
          if (mg%operator_type == mg_ahelmholtz) then
             write(u) mg%boxes(id)%cc(1:nc, 1:nc, 1:nc, mg_irhs)
          else
             write(u) mg%boxes(id)%cc(1:nc, 1:nc, 1:nc, mg_iphi)
          end if
       end do
    end do
    close(u)
  end subroutine dump_phi

  ! multi-rank: this rank's boxes, each tagged with its place in the one-rank order
  subroutine dump_phi_rank(mg, fname)
    type(mg_t), intent(inout) :: mg
    character(len=*), intent(in) :: fname
    character(len=16) :: suffix
    integer :: u, n, id, lvl, nc
    write(suffix, '(A,I0)') ".r", mg%my_rank
    open(newunit=u, file=fname // trim(suffix), access="stream", form="unformatted", status="replace")
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%ids)
          id = mg%lvls(lvl)%ids(n)
          if (mg%boxes(id)%rank /= mg%my_rank) cycle
          write(u) lvl, n, nc
          if (mg%operator_type == mg_ahelmholtz) then
             write(u) mg%boxes(id)%cc(1:nc, 1:nc, 1:nc, mg_irhs)
          else
             write(u) mg%boxes(id)%cc(1:nc, 1:nc, 1:nc, mg_iphi)
          end if
       end do
    end do
    close(u)
  end subroutine dump_phi_rank

  !> A refinement-boundary method of the mg_subr_rb interface
  !> (m_data_structures.f90:364-378): sides_rb's second-order form
  !> 0.5 gc + 0.75 x1 - 0.25 x2 (m_ghost_cells.f90:769-861) with other
  !> coefficients that also sum to one.
  subroutine custom_rb(box, nc, iv, nb, cgc)
    type(mg_box_t), intent(inout) :: box
    integer, intent(in)           :: nc, iv, nb
    real(dp), intent(in)          :: cgc(nc, nc)
    integer                       :: a, c, x1, x2, g
    if (mg_neighb_low(nb)) then
       x1 = 1; x2 = 2; g = 0
    else
       x1 = nc; x2 = nc - 1; g = nc + 1
    end if
    do c = 1, nc
       do a = 1, nc
          select case (mg_neighb_dim(nb))
          case (1)
             box%cc(g, a, c, iv) = 0.4_dp * cgc(a, c) + 0.9_dp * box%cc(x1, a, c, iv) &
                  - 0.3_dp * box%cc(x2, a, c, iv)
          case (2)
             box%cc(a, g, c, iv) = 0.4_dp * cgc(a, c) + 0.9_dp * box%cc(a, x1, c, iv) &
                  - 0.3_dp * box%cc(a, x2, c, iv)
          case default
             box%cc(a, c, g, iv) = 0.4_dp * cgc(a, c) + 0.9_dp * box%cc(a, c, x1, iv) &
                  - 0.3_dp * box%cc(a, c, x2, iv)
          end select
       end do
    end do
  end subroutine custom_rb

  subroutine sol_boundary_condition(box, nc, iv, nb, bc_type, bc)
    type(mg_box_t), intent(in) :: box
    integer, intent(in)        :: nc, iv, nb
    integer, intent(out)       :: bc_type
    real(dp), intent(out)      :: bc(nc, nc)
    real(dp)                   :: x(nc, nc, 3)
    integer                    :: i, j
    call mg_get_face_coords(box, nb, nc, x)
    bc_type = mg_bc_dirichlet
    do j = 1, nc
       do i = 1, nc
          bc(i, j) = solution(x(i, j, :))
       end do
    end do
  end subroutine sol_boundary_condition

  subroutine build_amr_tree(mg, n_amr_levels, lvl1_size, box_size, dr, periodic)
    type(mg_t), intent(inout) :: mg
    integer, intent(in)       :: n_amr_levels, lvl1_size(NDIM), box_size
    real(dp), intent(in)      :: dr(NDIM)
    logical, intent(in)       :: periodic(NDIM)
    integer                   :: lvl, i, id, n_finer
    real(dp)                  :: r_min(NDIM), domain_len(NDIM)
    real(dp)                  :: r0(NDIM), r1(NDIM), box_center(NDIM)
    n_finer    = n_amr_levels * product(lvl1_size / box_size) + 1000
    r_min      = 0.0_dp
    domain_len = lvl1_size * dr
    call mg_build_rectangle(mg, lvl1_size, box_size, dr, r_min, periodic, n_finer)
    do lvl = 1, n_amr_levels-1
       do i = 1, size(mg%lvls(lvl)%ids)
          id = mg%lvls(lvl)%ids(i)
          r0 = (0.5_dp + shift) * domain_len - domain_len * 0.5**(lvl+1)
          r1 = (0.5_dp + shift) * domain_len + domain_len * 0.5**(lvl+1)
          box_center = mg%boxes(id)%r_min + 0.5_dp * box_size * mg%boxes(id)%dr
          if (all(box_center >= r0 .and. box_center <= r1)) call mg_add_children(mg, id)
       end do
       call mg_set_leaves_parents(mg%boxes, mg%lvls(lvl))
       call mg_set_next_level_ids(mg, lvl)
       call mg_set_neighbors_lvl(mg, lvl+1)
    end do
    call mg_set_leaves_parents(mg%boxes, mg%lvls(n_amr_levels))
    mg%highest_lvl = n_amr_levels
    do lvl = 1, mg%highest_lvl
       call mg_set_refinement_boundaries(mg%boxes, mg%lvls(lvl))
    end do
  end subroutine build_amr_tree

end program omg_golden
