!> Umbrella module with the name the reference's programs `use`
!> (reference: src/m_octree_mg.f90:2-19), re-exporting the kept host modules
!> of the reference and the GPU-backed m_multigrid and m_free_space of this
!> directory.
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
  use m_free_space
  implicit none
  public
end module m_octree_mg
