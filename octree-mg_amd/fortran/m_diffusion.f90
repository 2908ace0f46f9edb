!> Drop-in m_diffusion for octree-mg, backed by the MI355X kernels of libomg.so.
!>
!> Same module name and public API as the reference's src/m_diffusion.f90:
!> diffusion_solve (:19-57), diffusion_solve_vcoeff (:63-101) and
!> diffusion_solve_acoeff (:108-142).  One implicit time step of phi (order 1
!> = backward Euler, 2 = Crank-Nicolson) solved as a Helmholtz problem.  The
!> whole step (set_rhs, FMG, the V-cycle loop until max_res) runs on the GPU
!> in one omg_diffusion_solve call, so it also works in resident mode
!> (mg_gpu_set_resident), where mg%boxes(:)%cc is not current.  The host
!> state the reference leaves behind (mg%operator_type, the methods, the
!> operator's lambda) is set the same way; the error stops are the same.
module m_diffusion
  use m_data_structures
  use m_multigrid

  implicit none
  private

  public :: diffusion_solve
  public :: diffusion_solve_vcoeff
  public :: diffusion_solve_acoeff

contains

  !> Constant diffusion coefficient (m_diffusion.f90:19-57): lambda = order/(dt*D).
  subroutine diffusion_solve(mg, dt, diffusion_coeff, order, max_res)
    use m_helmholtz
    type(mg_t), intent(inout) :: mg
    real(dp), intent(in)      :: dt
    real(dp), intent(in)      :: diffusion_coeff
    integer, intent(in)       :: order
    real(dp), intent(in)      :: max_res
    logical                   :: ok

    mg%operator_type = mg_helmholtz
    call mg_set_methods(mg)
    call check_order(order)
    call helmholtz_set_lambda(order/(dt * diffusion_coeff))
    call mg_gpu_diffusion_solve(mg, dt, diffusion_coeff, order, max_res, ok)
    if (.not. ok) call no_convergence(mg, .false.)
  end subroutine diffusion_solve

  !> Variable coefficient in mg_iveps (m_diffusion.f90:63-101): lambda = order/dt.
  subroutine diffusion_solve_vcoeff(mg, dt, order, max_res)
    use m_vhelmholtz
    type(mg_t), intent(inout) :: mg
    real(dp), intent(in)      :: dt
    integer, intent(in)       :: order
    real(dp), intent(in)      :: max_res
    logical                   :: ok

    mg%operator_type = mg_vhelmholtz
    call mg_set_methods(mg)
    call check_order(order)
    call vhelmholtz_set_lambda(order/dt)
    call mg_gpu_diffusion_solve(mg, dt, 1.0_dp, order, max_res, ok)
    if (.not. ok) call no_convergence(mg, .true.)
  end subroutine diffusion_solve_vcoeff

  !> Anisotropic coefficients in mg_iveps1..3 (m_diffusion.f90:108-142).
  subroutine diffusion_solve_acoeff(mg, dt, order, max_res)
    use m_ahelmholtz
    type(mg_t), intent(inout) :: mg
    real(dp), intent(in)      :: dt
    integer, intent(in)       :: order
    real(dp), intent(in)      :: max_res
    logical                   :: ok

    mg%operator_type = mg_ahelmholtz
    call mg_set_methods(mg)
    call check_order(order)
    call ahelmholtz_set_lambda(order/dt)
    call mg_gpu_diffusion_solve(mg, dt, 1.0_dp, order, max_res, ok)
    if (.not. ok) call no_convergence(mg, .true.)
  end subroutine diffusion_solve_acoeff

  subroutine check_order(order)
    integer, intent(in) :: order
    if (order /= 1 .and. order /= 2) error stop "diffusion_solve: order should be 1 or 2"
  end subroutine check_order

  subroutine no_convergence(mg, variable)
    type(mg_t), intent(in) :: mg
    logical, intent(in)    :: variable
    if (mg%my_rank == 0) then
       print *, "Did you specify boundary conditions correctly?"
       if (variable) print *, "Or is the variation in diffusion too large?"
    end if
    error stop "diffusion_solve: no convergence"
  end subroutine no_convergence

end module m_diffusion
