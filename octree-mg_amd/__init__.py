"""octree-mg_amd — MI355X-native hot path of the octree-mg FAS V-cycle.

libomg.so (csrc/, HIP for gfx950) implements the per-level box loops of the
reference's m_multigrid / m_laplacian / m_helmholtz / m_restrict / m_prolong /
m_ghost_cells behind the C-ABI in include/omg.h; this package is the Python
host mirror of the reference's Fortran API (mg.py) and its tree bookkeeping
(tree.py), m_diffusion's implicit time step (diffusion.py) and m_free_space's
free-space boundary conditions (free_space.py).  The Fortran drop-in modules
live in fortran/.
"""
from . import device, problems, tree  # noqa: F401
from .mg import (BC, MG, Loopback, helmholtz_set_lambda, mg_add_children, mg_allocate_storage,  # noqa: F401
                 mg_apply_op, mg_build_rectangle, mg_comm_init, mg_deallocate_storage,
                 mg_fas_fmg, mg_fas_vcycle, mg_fill_ghost_cells, mg_fill_ghost_cells_lvl,
                 mg_load_balance, mg_load_balance_parents, mg_load_balance_simple,
                 mg_phi_bc_store, mg_prolong, mg_restrict, mg_restrict_lvl, mg_set_methods)
from .diffusion import diffusion_solve, diffusion_solve_acoeff, diffusion_solve_vcoeff  # noqa: F401
from .free_space import mg_poisson_free_3d  # noqa: F401
from .tree import *  # noqa: F401,F403
