!> Drop-in m_free_space for octree-mg, backed by the MI355X kernels of libomg.so.
!>
!> Same module name and public API as the reference's src/m_free_space.f90
!> (mg_poisson_free_3d :36-214), so the reference's tests/test_free_space.f90
!> compiles unchanged against it.  Where the reference restricts rhs, builds
!> the Green's function and solves with its bundled BigDFT PSolver
!> (poisson_3d_fft/) on the host, all of it runs on the GPU here
!> (omg_poisson_free_3d: kernel tables, hipFFT convolution, boundary planes,
!> boundary table of every level, the initial guess, FMG or V-cycle), through
!> mg_gpu_poisson_free_3d of the drop-in m_multigrid.
!>
!> Afterwards mg is left as the reference leaves it: phi's boundary callback
!> interpolates the six boundary planes the device hands back (the
!> reference's ghost_cells_free_bc / interp_bc, :216-268, same arithmetic
!> order), and the boundary data is stored (mg%phi_bc_data_stored, the bc type
!> in the neighbour slots of physical faces).
module m_free_space
  use m_data_structures

  implicit none
  private

  !> Host copy of the device's free-space state: the six boundary planes
  !> (bc_x0, bc_x1 of nx2*nx3, bc_y0, bc_y1 of nx1*nx3, bc_z0, bc_z1 of
  !> nx1*nx2, first index fastest) in one array, and where each starts.
  logical               :: have_planes = .false.
  integer               :: plane_nx(3) = 0
  integer               :: plane_first(mg_num_neighbors) = 0
  integer               :: plane_rows(mg_num_neighbors) = 0
  real(dp), allocatable :: plane_data(:)
  real(dp)              :: plane_x0(2, mg_num_neighbors) = 0   ! first point of each plane
  real(dp)              :: plane_idr(2, mg_num_neighbors) = 0  ! 1 / its spacing

  public :: mg_poisson_free_3d

contains

  !> mg_poisson_free_3d (m_free_space.f90:36-214) on the GPU.
  subroutine mg_poisson_free_3d(mg, new_rhs, max_fft_frac, fmgcycle, max_res)
    use m_multigrid, only: mg_gpu_poisson_free_3d
    type(mg_t), intent(inout)       :: mg
    logical, intent(in)             :: new_rhs
    real(dp), intent(in)            :: max_fft_frac
    logical, intent(in)             :: fmgcycle
    real(dp), intent(out), optional :: max_res
    real(dp)                        :: res, h(3)
    integer                         :: fft_lvl, nb, d, q, tang(2), pos, lvl, i, id

    if (.not. have_planes .and. .not. new_rhs) &
         error stop "mg_poisson_free_3d: first call requires new_rhs = .true."
    if (mg%geometry_type /= mg_cartesian) &
         error stop "mg_poisson_free_3d: Cartesian 3D geometry required"
    if (mg%operator_type /= mg_laplacian) &
         error stop "mg_poisson_free_3d: laplacian operator required"

    call mg_gpu_poisson_free_3d(mg, new_rhs, max_fft_frac, fmgcycle, present(max_res), res, &
         fft_lvl, plane_nx, plane_data)
    have_planes = .true.

    ! where each plane starts, its row length and its geometry: cell-centred
    ! points of the FFT level's grid, one ghost layer out (:128-139)
    h = mg%dr(:, fft_lvl)
    pos = 0
    do nb = 1, mg_num_neighbors
       d = mg_neighb_dim(nb)
       tang = pack([1, 2, 3], [1, 2, 3] /= d)
       plane_first(nb) = pos
       plane_rows(nb) = plane_nx(tang(1))
       pos = pos + plane_nx(tang(1)) * plane_nx(tang(2))
       do q = 1, 2
          plane_idr(q, nb) = 1 / h(tang(q))
          plane_x0(q, nb)  = mg%r_min(tang(q)) - 0.5_dp * h(tang(q))
       end do
    end do

    ! the reference's side effects on mg (:102-104, mg_phi_bc_store :174)
    do nb = 1, mg_num_neighbors
       mg%bc(nb, mg_iphi)%boundary_cond => free_space_bc
    end do
    do lvl = mg%lowest_lvl, mg%highest_lvl
       do i = 1, size(mg%lvls(lvl)%my_ids)
          id = mg%lvls(lvl)%my_ids(i)
          where (mg%boxes(id)%neighbors < mg_no_box) mg%boxes(id)%neighbors = mg_bc_dirichlet
       end do
    end do
    mg%phi_bc_data_stored = .true.

    if (present(max_res) .and. fft_lvl < mg%highest_lvl) max_res = res
  end subroutine mg_poisson_free_3d

  !> Boundary callback of phi: the face's cell-centre coordinates
  !> (mg_get_face_coords), then bilinear interpolation in the stored plane,
  !> weights and sum in the order of the reference's interp_bc.
  subroutine free_space_bc(box, nc, iv, nb, bc_type, bc)
    type(mg_box_t), intent(in)    :: box
    integer, intent(in)           :: nc
    integer, intent(in)           :: iv
    integer, intent(in)           :: nb
    integer, intent(out)          :: bc_type
    double precision, intent(out) :: bc(nc, nc)
    double precision              :: rr(nc, nc, 3), f(2), lo(2)
    integer                       :: tang(2), i, j, k(2), base, m

    bc_type = mg_bc_dirichlet
    tang = pack([1, 2, 3], [1, 2, 3] /= mg_neighb_dim(nb))
    call mg_get_face_coords(box, nb, nc, rr)
    base = plane_first(nb)
    m = plane_rows(nb)
    do j = 1, nc
       do i = 1, nc
          f(1) = (rr(i, j, tang(1)) - plane_x0(1, nb)) * plane_idr(1, nb)
          f(2) = (rr(i, j, tang(2)) - plane_x0(2, nb)) * plane_idr(2, nb)
          k = ceiling(f)
          lo = k - f
          bc(i, j) = (lo(1) * lo(2)) * at(k(1), k(2))
          bc(i, j) = bc(i, j) + ((1 - lo(1)) * lo(2)) * at(k(1) + 1, k(2))
          bc(i, j) = bc(i, j) + (lo(1) * (1 - lo(2))) * at(k(1), k(2) + 1)
          bc(i, j) = bc(i, j) + ((1 - lo(1)) * (1 - lo(2))) * at(k(1) + 1, k(2) + 1)
       end do
    end do

  contains

    real(dp) function at(a, b)
      integer, intent(in) :: a, b
      at = plane_data(base + a + m * (b - 1))
    end function at
  end subroutine free_space_bc

end module m_free_space
