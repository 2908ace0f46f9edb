! TEST INFRASTRUCTURE (oracle/_ref build only).
! The image's conda MPICH 3.3.2 ships a gfortran-format mpi.mod that amdflang
! cannot read; this module exposes the same real MPICH interface by including
! the image's own mpif.h.  Nothing is stubbed: every symbol resolves to
! /opt/conda/lib/libmpi(fort).so at link time.
module mpi
  implicit none
  include 'mpif.h'
end module mpi
