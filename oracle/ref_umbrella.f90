! TEST INFRASTRUCTURE (oracle/_ref build only).
! Umbrella module with the name the reference's tests `use`
! (reference: src/m_octree_mg.f90:2-19).  It re-exports the reference modules
! compiled from /root/reference/src, minus m_free_space, whose BigDFT FFT
! dependency (poisson_3d_fft/) is out of scope (SURVEY.md §2, OUT rows).
module m_octree_mg
  use m_data_structures
  use m_build_tree
  use m_load_balance
  use m_ghost_cells
  use m_allocate_storage
  use m_restrict
  use m_communication
  use m_prolong
  use m_multigrid
  use m_helmholtz
  use m_vhelmholtz
  use m_ahelmholtz
  implicit none
  public
end module m_octree_mg
