!> `use mpi` for amdflang: the image's conda MPICH ships a gfortran-format
!> mpi.mod, so this module includes its mpif.h instead.
module mpi
  implicit none
  include 'mpif.h'
end module mpi
