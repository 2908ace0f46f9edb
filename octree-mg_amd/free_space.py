"""Python mirror of the reference's m_free_space (src/m_free_space.f90).

    mg_poisson_free_3d(mg, new_rhs, max_fft_frac, fmgcycle, max_res=False)   # :36-214

Free-space boundary conditions for the 3D Poisson problem: the problem is
solved once by FFT convolution with the free-space Green's function on the
highest uniform level holding at most max_fft_frac of the unknowns, that
solution gives the Dirichlet values of phi on every physical face of every
level and the initial guess, and one FMG (fmgcycle) or V-cycle follows.  All
of it runs on the GPU (omg_poisson_free_3d in libomg.so: the Green's
function, hipFFT transforms, boundary interpolation and the multigrid cycle).

Same names, argument meaning and error behaviour as the reference: the first
call needs new_rhs = True ("mg_poisson_free_3d: first call requires new_rhs =
.true."), the geometry must be Cartesian and the operator the Laplacian.
Afterwards mg.bc[nb][MG_IPHI] holds the boundary callback
(ghost_cells_free_bc, :216-270) backed by host copies of the six boundary
planes, and mg.phi_bc_data_stored is set, as the reference leaves mg.
Returns the max residual when max_res is requested (None otherwise, and
0.0 when the FFT level is the highest and no cycle runs).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from .mg import BC, MG
from .tree import MG_BC_DIRICHLET, MG_CARTESIAN, MG_IPHI, MG_LAPLACIAN, NEIGHB_DIM, NEIGHB_LOW


class FreeBoundary:
    """ghost_cells_free_bc + interp_bc (m_free_space.f90:216-270) over host
    copies of the six boundary planes; a boundary_cond callback of mg.bc."""

    def __init__(self, mg: MG, fft_lvl: int, nx, planes: np.ndarray):
        self.nx = [int(v) for v in nx]
        n1, n2, n3 = self.nx
        sizes = [n2 * n3, n2 * n3, n1 * n3, n1 * n3, n1 * n2, n1 * n2]
        shapes = [(n3, n2), (n3, n2), (n3, n1), (n3, n1), (n2, n1), (n2, n1)]
        self.planes, pos = [], 0
        for s, sh in zip(sizes, shapes):
            # first index fastest in memory -> [second, first] here
            self.planes.append(planes[pos:pos + s].reshape(sh))
            pos += s
        dr = np.asarray(mg.dr[fft_lvl], dtype=np.float64)
        self.inv_dr, self.r_min = {}, {}
        for nb in range(1, 7):
            ixs = [d for d in range(3) if d != NEIGHB_DIM[nb - 1] - 1]
            self.inv_dr[nb] = [1.0 / dr[d] for d in ixs]
            self.r_min[nb] = [mg.r_min[d] - 0.5 * dr[d] for d in ixs]

    def __call__(self, mg: MG, id_: int, nc: int, iv: int, nb: int):
        rr = mg.get_face_coords(id_, nb, nc)          # [nc, nc, 3], rr[i, j]
        ixs = [d for d in range(3) if d != NEIGHB_DIM[nb - 1] - 1]
        x1 = rr[:, :, ixs[0]]
        x2 = rr[:, :, ixs[1]]
        f1 = (x1 - self.r_min[nb][0]) * self.inv_dr[nb][0]
        f2 = (x2 - self.r_min[nb][1]) * self.inv_dr[nb][1]
        i1 = np.ceil(f1).astype(np.int64)
        i2 = np.ceil(f2).astype(np.int64)
        l1 = i1 - f1
        l2 = i2 - f2
        P = self.planes[nb - 1]   # P[b - 1, a - 1] = plane(a, b), 1-based
        v = (l1 * l2) * P[i2 - 1, i1 - 1]
        v = v + ((1 - l1) * l2) * P[i2 - 1, i1]
        v = v + (l1 * (1 - l2)) * P[i2, i1 - 1]
        v = v + ((1 - l1) * (1 - l2)) * P[i2, i1]
        # values[nc*nc] with the first tangential index fastest
        return MG_BC_DIRICHLET, np.ascontiguousarray(v.T).reshape(-1)


def mg_poisson_free_3d(mg: MG, new_rhs: bool, max_fft_frac: float, fmgcycle: bool, max_res=False):
    """mg_poisson_free_3d (reference: src/m_free_space.f90:36-214)."""
    if mg.geometry_type != MG_CARTESIAN:
        raise RuntimeError("mg_poisson_free_3d: Cartesian 3D geometry required")
    if mg.operator_type != MG_LAPLACIAN:
        raise RuntimeError("mg_poisson_free_3d: laplacian operator required")
    mg._require_alloc()
    r = C.c_double(0.0)
    r_min = np.ascontiguousarray(mg.r_min, dtype=np.float64)
    box_r_min = np.ascontiguousarray(mg.box_r_min[1:mg.n_boxes + 1], dtype=np.float64).reshape(-1)
    mg.ctx.call("poisson_free_3d", int(bool(new_rhs)), float(max_fft_frac), int(bool(fmgcycle)),
                int(bool(max_res)), C.byref(r), r_min, box_r_min.ctypes.data_as(C.c_void_p))
    # the reference's side effects on mg: phi's boundary callback (:102-104)
    # and the stored boundary data (:174)
    lvl, nx = C.c_int(0), np.zeros(3, np.int32)
    mg.ctx.call("free_planes", C.byref(lvl), nx, None, 0)
    n1, n2, n3 = (int(v) for v in nx)
    planes = np.empty(2 * (n2 * n3 + n1 * n3 + n1 * n2))
    mg.ctx.call("free_planes", C.byref(lvl), nx, planes.ctypes.data_as(C.c_void_p), planes.size)
    cb = FreeBoundary(mg, lvl.value, nx, planes)
    for nb in range(1, 7):
        mg.bc[nb][MG_IPHI] = BC(MG_BC_DIRICHLET, 0.0, boundary_cond=cb)
    mg.phi_bc_data_stored = True
    return r.value if max_res else None


def fft_level(mg: MG, max_fft_frac: float) -> int:
    """The level mg_poisson_free_3d solves by FFT (m_free_space.f90:80-93):
    the highest uniform level with at most max_fft_frac of the unknowns."""
    n_total = mg.number_of_unknowns()
    lvl = mg.first_normal_lvl
    while lvl <= mg.highest_lvl - 1:
        L = mg.lvls[lvl]
        if len(L.leaves) != 0 and len(L.parents) != 0:
            break
        lvl += 1
    while lvl >= mg.lowest_lvl + 1:
        if float(len(mg.lvls[lvl].ids) * mg.box_size ** 3) <= max_fft_frac * float(n_total):
            break
        lvl -= 1
    return lvl


def fft_length(m: int) -> int:
    """Transform length of one padded axis (omg_api.cpp fft_length): the
    smallest even n >= m with prime factors 2, 3, 5, 7."""
    n = max(m, 2)
    while True:
        if n % 2 == 0:
            r = n
            for f in (2, 3, 5, 7):
                while r % f == 0:
                    r //= f
            if r == 1:
                return n
        n += 1


RHS_FAC = -1.0 / (4.0 * math.acos(-1.0))   # m_free_space.f90:67
__all__ = ["mg_poisson_free_3d", "FreeBoundary", "fft_level", "fft_length", "RHS_FAC", "NEIGHB_LOW"]
