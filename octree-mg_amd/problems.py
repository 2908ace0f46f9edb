"""Problem set-ups used by the reference's own test drivers, restated on the host.

These produce INPUT data (solution u, callback boundary values) exactly as the
reference tests compute them, so that the device path and the checker start
from bit-identical inputs:

* u = prod(sin(2*pi*n_modes*r)) at cell centres of every cell incl. ghosts
  (reference: tests/test_uniform_grid.f90:132-153)
* Dirichlet callback with u on the boundary faces
  (reference: tests/test_uniform_grid.f90:204-239, mg_get_face_coords
  src/m_data_structures.f90:495-539)
"""
from __future__ import annotations

import math

import numpy as np

from .tree import MG_BC_DIRICHLET, MG_NO_BOX

PI = math.acos(-1.0)
TWO_PI_N = 2.0 * PI * 5.0  # (2*pi)*real(n_modes) with n_modes = 5


def solution_at(r: np.ndarray) -> np.ndarray:
    """product(sin(2*pi*n_modes*r)) over the last axis (3 components)."""
    s = np.sin(TWO_PI_N * r)
    return (s[..., 0] * s[..., 1]) * s[..., 2]


def box_solution(tree, id_: int) -> np.ndarray:
    """u on the full (nc+2)^3 box incl. ghosts, array index [k, j, i]."""
    lvl = int(tree.lvl[id_])
    nc = tree.box_size_lvl[lvl]
    dr = tree.dr[lvl]
    idx = np.arange(0, nc + 2, dtype=np.float64) - 0.5
    rmin = tree.box_r_min[id_]
    r = np.empty((nc + 2, nc + 2, nc + 2, 3))
    r[..., 0] = rmin[0] + idx[None, None, :] * dr[0]
    r[..., 1] = rmin[1] + idx[None, :, None] * dr[1]
    r[..., 2] = rmin[2] + idx[:, None, None] * dr[2]
    return solution_at(r)


def level_solution(tree, lvl: int, ids=None) -> np.ndarray:
    """u on every box of a level, [box, k, j, i].  u is separable, so the three
    sines are evaluated per box row and multiplied as (s_x*s_y)*s_z — the
    same roundings as box_solution() cell by cell."""
    ids = np.asarray(tree.lvls[lvl].ids if ids is None else ids, dtype=np.int64)
    nc = tree.box_size_lvl[lvl]
    if len(ids) == 0:
        return np.zeros((0, nc + 2, nc + 2, nc + 2))
    dr = tree.dr[lvl]
    idx = np.arange(0, nc + 2, dtype=np.float64) - 0.5
    rmin = tree.box_r_min[ids]                                   # [b, 3]
    s = [np.sin(TWO_PI_N * (rmin[:, d:d + 1] + idx[None, :] * dr[d])) for d in range(3)]
    return (s[0][:, None, None, :] * s[1][:, None, :, None]) * s[2][:, :, None, None]


TWO_PI = 2.0 * PI


def level_eps(tree, lvl: int, ids=None) -> np.ndarray:
    """The coefficient of the golden v-operator runs on every box of a level,
    incl. ghosts: eps = (1.5 + sin(2 pi x)) * (1.5 + sin(2 pi y)) * (1.5 +
    sin(2 pi z)) (oracle/omg_golden.f90 set_eps), [box, k, j, i]."""
    ids = np.asarray(tree.lvls[lvl].ids if ids is None else ids, dtype=np.int64)
    nc = tree.box_size_lvl[lvl]
    if len(ids) == 0:
        return np.zeros((0, nc + 2, nc + 2, nc + 2))
    dr = tree.dr[lvl]
    idx = np.arange(0, nc + 2, dtype=np.float64) - 0.5
    rmin = tree.box_r_min[ids]
    f = [1.5 + np.sin(TWO_PI * (rmin[:, d:d + 1] + idx[None, :] * dr[d])) for d in range(3)]
    return (f[0][:, None, None, :] * f[1][:, None, :, None]) * f[2][:, :, None, None]


def callback_bc_faces(tree, boxes=None):
    """Tabulate the Dirichlet-u callback for every physical face of every box.

    Returns (face_off[int64, n_boxes*6], face_type[int32, n_boxes*6], data)
    with face_off[(id-1)*6 + nb-1] the offset of nc*nc values (first
    tangential index fastest), or -1 where the face is not physical."""
    n = tree.n_boxes
    face_off = np.full(n * 6, -1, dtype=np.int64)
    face_type = np.zeros(n * 6, dtype=np.int32)
    chunks, pos = [], 0
    ids = range(1, n + 1) if boxes is None else boxes
    for id_ in ids:
        id_ = int(id_)
        nc = tree.box_size_lvl[int(tree.lvl[id_])]
        for nb in range(1, 7):
            if tree.neighbors[id_, nb - 1] < MG_NO_BOX:
                x = tree.get_face_coords(id_, nb, nc)          # [i, j, :]
                vals = solution_at(x).T.reshape(-1)            # i fastest
                face_off[(id_ - 1) * 6 + nb - 1] = pos
                face_type[(id_ - 1) * 6 + nb - 1] = MG_BC_DIRICHLET
                chunks.append(vals)
                pos += vals.size
    data = np.concatenate(chunks) if chunks else np.zeros(1)
    return face_off, face_type, data
