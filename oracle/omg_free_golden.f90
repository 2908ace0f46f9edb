! TEST INFRASTRUCTURE — golden-vector generator for free-space boundary
! conditions (oracle/_ref build only).
!
! Drives the REFERENCE m_free_space (src/m_free_space.f90, with the reference's
! own poisson_3d_fft package, both compiled from /root/reference by
! oracle/Makefile) through the set-up of the reference's test
! tests/test_free_space.f90: a Gaussian charge of amplitude 1, sigma 0.1 at
! (0.5, 0.5, 0.5) on the unit cube (:9-13, :141-148), its analytic potential
! as the solution (:127-139), rhs and solution on every level (:150-165), and
! mg_poisson_free_3d(mg, n == 1, fft_frac, fmg, max_res) per iteration (:79).
! Per iteration it prints max |phi - sol| and sqrt(mean (phi - sol)^2) over
! the highest level, and max_res, as IEEE bit patterns (the test's print_error,
! :167-195, which reduces over mpi_comm_world the same way).
!
! Usage: omg_free_golden box nx ny nz n_its fft_frac cycle dump
!   cycle f (FMG, as the test) | v (V-cycle)
!   dump  x, or a file: final phi interior of every box (ids order per level,
!         lowest..highest, i fastest), raw float64, 1 rank only
#include "cpp_macros.h"
program omg_free_golden
  use mpi
  use m_octree_mg
  use m_free_space
  implicit none

  integer, parameter  :: i8k = selected_int_kind(18)
  real(dp), parameter :: gauss_ampl  = 1.0d0
  real(dp), parameter :: gauss_r0(3) = [0.5d0, 0.5d0, 0.5d0]
  real(dp), parameter :: gauss_sigma = 0.1d0
  real(dp), parameter :: pi          = acos(-1.0_dp)
  integer             :: box_size, domain_size(NDIM), n_its, n, ierr, i_sol
  real(dp)            :: dr(NDIM), r_min(NDIM) = 0.0_dp, fft_frac, max_res, t0, t1
  logical             :: periodic(NDIM) = .false.
  character(len=64)   :: arg, a_cycle, a_dump
  type(mg_t)          :: mg

  if (command_argument_count() < 8) error stop "omg_free_golden: need 8 args"
  call get_command_argument(1, arg); read(arg, *) box_size
  do n = 1, NDIM
     call get_command_argument(1+n, arg); read(arg, *) domain_size(n)
  end do
  call get_command_argument(5, arg); read(arg, *) n_its
  call get_command_argument(6, arg); read(arg, *) fft_frac
  call get_command_argument(7, a_cycle)
  a_dump = ""
  call get_command_argument(8, arg)
  if (trim(arg) /= "x") a_dump = arg

  dr = 1.0_dp / domain_size
  mg%n_extra_vars = 1
  i_sol = mg_num_vars + 1
  mg%geometry_type = mg_cartesian
  mg%operator_type = mg_laplacian
  mg%smoother_type = mg_smoother_gsrb

  call mg_set_methods(mg)
  call mg_comm_init(mg)
  call mg_build_rectangle(mg, domain_size, box_size, dr, r_min, periodic, 0)
  call mg_load_balance(mg)
  call mg_allocate_storage(mg)
  call set_rhs_and_solution(mg)

  t0 = mpi_wtime()
  do n = 1, n_its
     max_res = 0.0_dp
     call mg_poisson_free_3d(mg, n == 1, fft_frac, a_cycle(1:1) == "f", max_res)
     call print_error(mg, n, max_res)
  end do
  t1 = mpi_wtime()
  if (mg%my_rank == 0) write(*, '(A,ES25.17,A,I0)') "TIME", (t1 - t0) / max(n_its, 1), " NCPU ", mg%n_cpu
  if (len_trim(a_dump) > 0 .and. mg%n_cpu == 1) call dump_phi(mg, trim(a_dump))
  call mpi_barrier(mpi_comm_world, ierr)
  call mpi_finalize(ierr)

contains

  elemental function solution(x, y, z) result(val)
    real(dp), intent(in) :: x, y, z
    real(dp)             :: val, rnorm
    real(dp), parameter  :: fac = 1/(4 * pi)
    rnorm = norm2([ x, y, z ] - gauss_r0)
    if (rnorm < sqrt(epsilon(1.0d0))) then
       val = 2 * fac * gauss_ampl / (sqrt(pi) * gauss_sigma)
    else
       val = fac * gauss_ampl * erf(rnorm / gauss_sigma) / rnorm
    end if
  end function solution

  elemental function rhs(x, y, z) result(val)
    real(dp), intent(in) :: x, y, z
    real(dp)             :: val, r(NDIM)
    r = ([ x, y, z ] - gauss_r0) / gauss_sigma
    val = -gauss_ampl / (gauss_sigma**3 * pi * sqrt(pi)) * exp(-sum(r**2))
  end function rhs

  subroutine set_rhs_and_solution(mg)
    type(mg_t), intent(inout) :: mg
    real(dp)                  :: r(3)
    integer                   :: n, id, lvl, nc, IJK
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(n)
          do KJI_DO(1, nc)
             r = mg%boxes(id)%r_min + ([IJK] - 0.5_dp) * mg%dr(:, lvl)
             mg%boxes(id)%cc(IJK, mg_irhs) = rhs(r(1), r(2), r(3))
             mg%boxes(id)%cc(IJK, i_sol) = solution(r(1), r(2), r(3))
          end do; CLOSE_DO
       end do
    end do
  end subroutine set_rhs_and_solution

  subroutine print_error(mg, it, mres)
    type(mg_t), intent(inout) :: mg
    integer, intent(in)       :: it
    real(dp), intent(in)      :: mres
    integer                   :: n, nc, id, lvl, IJK, ierr
    real(dp)                  :: err, max_err, err2_sum, err2
    max_err  = 0.0_dp
    err2_sum = 0.0_dp
    lvl = mg%highest_lvl
    nc = mg%box_size_lvl(lvl)
    do n = 1, size(mg%lvls(lvl)%my_ids)
       id = mg%lvls(lvl)%my_ids(n)
       do KJI_DO(1, nc)
          err      = abs(mg%boxes(id)%cc(IJK, mg_iphi) - mg%boxes(id)%cc(IJK, i_sol))
          max_err  = max(max_err, err)
          err2_sum = err2_sum + err**2
       end do; CLOSE_DO
    end do
    call mpi_allreduce(MPI_IN_PLACE, max_err, 1, MPI_DOUBLE, MPI_MAX, mpi_comm_world, ierr)
    call mpi_allreduce(MPI_IN_PLACE, err2_sum, 1, MPI_DOUBLE, MPI_SUM, mpi_comm_world, ierr)
    err2 = sqrt(err2_sum / mg_number_of_unknowns(mg))
    if (mg%my_rank == 0) write(*, '(A,I4,3(1X,Z16.16),3(1X,ES25.17))') "IT", it, &
         transfer(max_err, 0_i8k), transfer(err2, 0_i8k), transfer(mres, 0_i8k), max_err, err2, mres
  end subroutine print_error

  subroutine dump_phi(mg, fname)
    type(mg_t), intent(inout) :: mg
    character(len=*), intent(in) :: fname
    integer :: u, n, id, lvl, nc
    open(newunit=u, file=fname, access="stream", form="unformatted", status="replace")
    do lvl = mg%lowest_lvl, mg%highest_lvl
       nc = mg%box_size_lvl(lvl)
       do n = 1, size(mg%lvls(lvl)%ids)
          id = mg%lvls(lvl)%ids(n)
          write(u) mg%boxes(id)%cc(1:nc, 1:nc, 1:nc, mg_iphi)
       end do
    end do
    close(u)
  end subroutine dump_phi

end program omg_free_golden
