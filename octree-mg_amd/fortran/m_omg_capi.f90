!> ISO_C_BINDING interfaces of libomg.so (include/omg.h).
!>
!> This is the reference-side binding of the drop-in boundary: the Fortran
!> m_multigrid of octree-mg_amd/fortran/m_multigrid.f90 reaches the MI355X
!> kernels only through these declarations.  Every function returns 0 on
!> success; omg_error_message() turns omg_last_error() into a Fortran string.
module m_omg_capi
  use iso_c_binding
  implicit none
  private

  integer, parameter, public :: omg_unique_id_bytes = 128

  public :: omg_error_message
  public :: omg_get_unique_id, omg_ctx_create, omg_ctx_destroy
  public :: omg_host_unique_id, omg_set_host_transport, omg_device_count
  public :: omg_tree_setup, omg_set_operator, omg_set_smoother
  public :: omg_set_subtract_mean, omg_set_bc, omg_set_bc_faces
  public :: omg_level_size, omg_upload_level, omg_download_level
  public :: omg_fas_vcycle, omg_fas_fmg, omg_apply_op, omg_phi_bc_store
  public :: omg_synchronize, omg_diffusion_solve
  public :: omg_poisson_free_3d, omg_free_planes
  public :: omg_set_refinement_bnd

  interface
     function omg_last_error() bind(C, name="omg_last_error") result(p)
       import :: c_ptr
       type(c_ptr) :: p
     end function omg_last_error

     function omg_get_unique_id(out) bind(C, name="omg_get_unique_id") result(ierr)
       import :: c_int, c_int8_t
       integer(c_int8_t), intent(out) :: out(*)
       integer(c_int) :: ierr
     end function omg_get_unique_id

     function omg_host_unique_id(out) bind(C, name="omg_host_unique_id") result(ierr)
       import :: c_int, c_int8_t
       integer(c_int8_t), intent(out) :: out(*)
       integer(c_int) :: ierr
     end function omg_host_unique_id

     function omg_set_host_transport(ctx, exchange, allgather, user) &
          bind(C, name="omg_set_host_transport") result(ierr)
       import :: c_ptr, c_int, c_funptr
       type(c_ptr), value    :: ctx
       type(c_funptr), value :: exchange, allgather
       type(c_ptr), value    :: user
       integer(c_int) :: ierr
     end function omg_set_host_transport

     function omg_device_count(n) bind(C, name="omg_device_count") result(ierr)
       import :: c_int
       integer(c_int), intent(out) :: n
       integer(c_int) :: ierr
     end function omg_device_count

     function omg_ctx_create(ctx, device, rank, n_ranks, unique_id) &
          bind(C, name="omg_ctx_create") result(ierr)
       import :: c_ptr, c_int, c_int8_t
       type(c_ptr), intent(out)          :: ctx
       integer(c_int), value             :: device, rank, n_ranks
       integer(c_int8_t), intent(in)     :: unique_id(*)
       integer(c_int) :: ierr
     end function omg_ctx_create

     function omg_ctx_destroy(ctx) bind(C, name="omg_ctx_destroy") result(ierr)
       import :: c_ptr, c_int
       type(c_ptr), value :: ctx
       integer(c_int) :: ierr
     end function omg_ctx_destroy

     function omg_tree_setup(ctx, n_boxes, lvl, parent, children, neighbors, ix, &
          rank, lowest_lvl, highest_lvl, first_normal_lvl, box_size, box_size_lvl, &
          dr, list_off, lists, n_vars) bind(C, name="omg_tree_setup") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value         :: ctx
       integer(c_int), value      :: n_boxes
       integer(c_int), intent(in) :: lvl(*), parent(*), children(*), neighbors(*)
       integer(c_int), intent(in) :: ix(*), rank(*)
       integer(c_int), value      :: lowest_lvl, highest_lvl, first_normal_lvl, box_size
       integer(c_int), intent(in) :: box_size_lvl(*)
       real(c_double), intent(in) :: dr(*)
       integer(c_int), intent(in) :: list_off(*), lists(*)
       integer(c_int), value      :: n_vars
       integer(c_int) :: ierr
     end function omg_tree_setup

     function omg_set_operator(ctx, op, lambda) bind(C, name="omg_set_operator") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value    :: ctx
       integer(c_int), value :: op
       real(c_double), value :: lambda
       integer(c_int) :: ierr
     end function omg_set_operator

     function omg_set_smoother(ctx, smoother, n_cycle_down, n_cycle_up, max_coarse_cycles, &
          residual_coarse_abs, residual_coarse_rel) bind(C, name="omg_set_smoother") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value    :: ctx
       integer(c_int), value :: smoother, n_cycle_down, n_cycle_up, max_coarse_cycles
       real(c_double), value :: residual_coarse_abs, residual_coarse_rel
       integer(c_int) :: ierr
     end function omg_set_smoother

     function omg_set_subtract_mean(ctx, on) bind(C, name="omg_set_subtract_mean") result(ierr)
       import :: c_ptr, c_int
       type(c_ptr), value    :: ctx
       integer(c_int), value :: on
       integer(c_int) :: ierr
     end function omg_set_subtract_mean

     function omg_set_bc(ctx, iv, nb, bc_type, bc_value) bind(C, name="omg_set_bc") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value    :: ctx
       integer(c_int), value :: iv, nb, bc_type
       real(c_double), value :: bc_value
       integer(c_int) :: ierr
     end function omg_set_bc

     function omg_set_refinement_bnd(ctx, iv, nb, fn, user) &
          bind(C, name="omg_set_refinement_bnd") result(ierr)
       import :: c_ptr, c_int, c_funptr
       type(c_ptr), value    :: ctx
       integer(c_int), value :: iv, nb
       type(c_funptr), value :: fn
       type(c_ptr), value    :: user
       integer(c_int) :: ierr
     end function omg_set_refinement_bnd

     function omg_set_bc_faces(ctx, iv, face_off, face_type, data, n_data) &
          bind(C, name="omg_set_bc_faces") result(ierr)
       import :: c_ptr, c_int, c_long_long, c_double
       type(c_ptr), value             :: ctx
       integer(c_int), value          :: iv
       integer(c_long_long), intent(in) :: face_off(*)
       integer(c_int), intent(in)     :: face_type(*)
       real(c_double), intent(in)     :: data(*)
       integer(c_long_long), value    :: n_data
       integer(c_int) :: ierr
     end function omg_set_bc_faces

     function omg_level_size(ctx, lvl, n_boxes, nc) bind(C, name="omg_level_size") result(ierr)
       import :: c_ptr, c_int
       type(c_ptr), value          :: ctx
       integer(c_int), value       :: lvl
       integer(c_int), intent(out) :: n_boxes, nc
       integer(c_int) :: ierr
     end function omg_level_size

     function omg_upload_level(ctx, lvl, iv, host) bind(C, name="omg_upload_level") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value         :: ctx
       integer(c_int), value      :: lvl, iv
       real(c_double), intent(in) :: host(*)
       integer(c_int) :: ierr
     end function omg_upload_level

     function omg_download_level(ctx, lvl, iv, host) bind(C, name="omg_download_level") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value          :: ctx
       integer(c_int), value       :: lvl, iv
       real(c_double), intent(out) :: host(*)
       integer(c_int) :: ierr
     end function omg_download_level

     function omg_fas_vcycle(ctx, highest_lvl, want_max_res, max_res, standalone) &
          bind(C, name="omg_fas_vcycle") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value          :: ctx
       integer(c_int), value       :: highest_lvl, want_max_res, standalone
       real(c_double), intent(out) :: max_res
       integer(c_int) :: ierr
     end function omg_fas_vcycle

     function omg_fas_fmg(ctx, have_guess, want_max_res, max_res) &
          bind(C, name="omg_fas_fmg") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value          :: ctx
       integer(c_int), value       :: have_guess, want_max_res
       real(c_double), intent(out) :: max_res
       integer(c_int) :: ierr
     end function omg_fas_fmg

     function omg_apply_op(ctx, i_out) bind(C, name="omg_apply_op") result(ierr)
       import :: c_ptr, c_int
       type(c_ptr), value    :: ctx
       integer(c_int), value :: i_out
       integer(c_int) :: ierr
     end function omg_apply_op

     function omg_phi_bc_store(ctx) bind(C, name="omg_phi_bc_store") result(ierr)
       import :: c_ptr, c_int
       type(c_ptr), value :: ctx
       integer(c_int) :: ierr
     end function omg_phi_bc_store

     function omg_diffusion_solve(ctx, op, dt, diffusion_coeff, order, max_res, n_vcycles, res) &
          bind(C, name="omg_diffusion_solve") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value          :: ctx
       integer(c_int), value       :: op, order
       real(c_double), value       :: dt, diffusion_coeff, max_res
       integer(c_int), intent(out) :: n_vcycles
       real(c_double), intent(out) :: res
       integer(c_int) :: ierr
     end function omg_diffusion_solve

     function omg_poisson_free_3d(ctx, new_rhs, max_fft_frac, fmgcycle, want_max_res, &
          max_res, r_min, box_r_min) bind(C, name="omg_poisson_free_3d") result(ierr)
       import :: c_ptr, c_int, c_double
       type(c_ptr), value          :: ctx
       integer(c_int), value       :: new_rhs, fmgcycle, want_max_res
       real(c_double), value       :: max_fft_frac
       real(c_double), intent(out) :: max_res
       real(c_double), intent(in)  :: r_min(*), box_r_min(*)
       integer(c_int) :: ierr
     end function omg_poisson_free_3d

     function omg_free_planes(ctx, fft_lvl, nx, planes, cap) bind(C, name="omg_free_planes") &
          result(ierr)
       import :: c_ptr, c_int, c_double, c_long_long
       type(c_ptr), value          :: ctx
       integer(c_int), intent(out) :: fft_lvl, nx(3)
       real(c_double), intent(out) :: planes(*)
       integer(c_long_long), value :: cap
       integer(c_int) :: ierr
     end function omg_free_planes

     function omg_synchronize(ctx) bind(C, name="omg_synchronize") result(ierr)
       import :: c_ptr, c_int
       type(c_ptr), value :: ctx
       integer(c_int) :: ierr
     end function omg_synchronize

     function c_strlen(s) bind(C, name="strlen") result(n)
       import :: c_ptr, c_size_t
       type(c_ptr), value :: s
       integer(c_size_t) :: n
     end function c_strlen
  end interface

contains

  !> omg_last_error() as a Fortran string
  function omg_error_message() result(msg)
    character(len=:), allocatable :: msg
    type(c_ptr)                   :: p
    character(kind=c_char), pointer :: chars(:)
    integer                       :: n, i

    p = omg_last_error()
    if (.not. c_associated(p)) then
       msg = ""
       return
    end if
    n = int(c_strlen(p))
    call c_f_pointer(p, chars, [n])
    allocate(character(len=n) :: msg)
    do i = 1, n
       msg(i:i) = chars(i)
    end do
  end function omg_error_message

end module m_omg_capi
