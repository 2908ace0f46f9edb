"""ctypes binding of the C oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker.  The product path (octree-mg_amd/libomg.so) never loads it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_P = C.c_void_p
_I = C.c_int
_D = C.c_double
_IP = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_DP = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_LP = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")

LAPLACIAN, VLAPLACIAN, HELMHOLTZ, VHELMHOLTZ, AHELMHOLTZ = 1, 2, 3, 4, 5
GS, GSRB = 1, 2


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run `make -C oracle`)")
        L = C.CDLL(path)
        L.orc_create.restype = _P
        L.orc_create.argtypes = [_I, _IP, _IP, _IP, _IP, _IP, _I, _I, _I, _I, _IP, _DP,
                                 _IP, _IP, _I, _IP, _I]
        L.orc_destroy.argtypes = [_P]
        L.orc_set_operator.argtypes = [_P, _I, _D, _I]
        L.orc_set_smoother.argtypes = [_P, _I, _I, _I, _I, _D, _D]
        L.orc_set_subtract_mean.argtypes = [_P, _I]
        L.orc_set_bc.argtypes = [_P, _I, _I, _I, _D]
        L.orc_set_bc_faces.argtypes = [_P, _I, _LP, _IP, _DP, C.c_longlong]
        L.orc_get_box.argtypes = [_P, _I, _I, _DP]
        L.orc_set_box.argtypes = [_P, _I, _I, _DP]
        L.orc_fas_vcycle.argtypes = [_P, _I, _I, C.POINTER(_D), _I]
        L.orc_fas_fmg.argtypes = [_P, _I, _I, C.POINTER(_D)]
        for f in ("orc_apply_op",):
            getattr(L, f).argtypes = [_P, _I]
        L.orc_box_op.argtypes = [_P, _I, _I]
        L.orc_set_rhs.argtypes = [_P, _D, _D]
        L.orc_diffusion_solve.restype = _I
        L.orc_diffusion_solve.argtypes = [_P, _I, _D, _D, _I, _D, C.POINTER(_I), C.POINTER(_D)]
        L.orc_restrict.argtypes = [_P, _I]
        L.orc_restrict_lvl.argtypes = [_P, _I, _I]
        L.orc_fill_ghost_cells.argtypes = [_P, _I]
        L.orc_fill_ghost_cells_lvl.argtypes = [_P, _I, _I]
        L.orc_smooth_boxes.argtypes = [_P, _I, _I]
        L.orc_box_smoother.argtypes = [_P, _I, _I]
        L.orc_update_coarse.argtypes = [_P, _I]
        L.orc_correct_children.argtypes = [_P, _I]
        L.orc_prolong.argtypes = [_P, _I, _I, _I, _I]
        L.orc_residual_lvl.argtypes = [_P, _I]
        L.orc_max_residual_lvl.argtypes = [_P, _I]
        L.orc_max_residual_lvl.restype = _D
        L.orc_subtract_mean.argtypes = [_P, _I, _I]
        L.orc_get_sum.argtypes = [_P, _I]
        L.orc_get_sum.restype = _D
        L.orc_phi_bc_store.argtypes = [_P]
        _LIB = L
    return _LIB


def tree_lists(tree):
    """Flatten per-level id lists (ids, leaves, parents, ref_bnds)."""
    off, data = [0], []
    for l in range(tree.lowest_lvl, tree.highest_lvl + 1):
        L = tree.lvls[l]
        for arr in (L.ids, L.leaves, L.parents, L.ref_bnds):
            data.extend(int(x) for x in arr)
            off.append(len(data))
    return np.array(off, dtype=np.int32), np.array(data if data else [0], dtype=np.int32)


class Oracle:
    """The whole tree on one CPU process (the reference with all boxes local)."""

    def __init__(self, tree, n_vars, n_ranks=1):
        L = lib()
        n = tree.n_boxes
        self.tree = tree
        self.n_vars = n_vars
        i32 = lambda a: np.ascontiguousarray(np.asarray(a)[1:n + 1], dtype=np.int32).reshape(-1)
        nlev = tree.highest_lvl - tree.lowest_lvl + 1
        bsl = np.array([tree.box_size_lvl[l] for l in range(tree.lowest_lvl, tree.highest_lvl + 1)],
                       dtype=np.int32)
        dr = np.ascontiguousarray(np.array([tree.dr[l] for l in range(tree.lowest_lvl,
                                                                      tree.highest_lvl + 1)],
                                           dtype=np.float64).reshape(nlev * 3))
        off, data = tree_lists(tree)
        self._keep = [i32(tree.lvl), i32(tree.parent), i32(tree.children), i32(tree.neighbors),
                      i32(tree.ix), bsl, dr, off, data, i32(tree.rank)]
        self.h = L.orc_create(n, self._keep[0], self._keep[1], self._keep[2], self._keep[3],
                              self._keep[4], tree.lowest_lvl, tree.highest_lvl,
                              tree.first_normal_lvl, tree.box_size, bsl, dr, off, data, n_vars,
                              self._keep[9], n_ranks)
        self.L = L

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_destroy(self.h)
            self.h = None

    def configure(self, op=LAPLACIAN, lam=0.0, smoother=GS, n_cycle_down=2, n_cycle_up=2,
                  max_coarse_cycles=1000, res_abs=1e-8, res_rel=1e-8, subtract_mean=False):
        self.L.orc_set_operator(self.h, op, lam, 1)
        self.L.orc_set_smoother(self.h, smoother, n_cycle_down, n_cycle_up, max_coarse_cycles,
                                res_abs, res_rel)
        self.L.orc_set_subtract_mean(self.h, int(subtract_mean))

    def set_bc(self, iv, nb, bc_type, value):
        self.L.orc_set_bc(self.h, iv, nb, bc_type, value)

    def set_bc_faces(self, iv, face_off, face_type, data):
        self.L.orc_set_bc_faces(self.h, iv, np.ascontiguousarray(face_off, dtype=np.int64),
                                np.ascontiguousarray(face_type, dtype=np.int32),
                                np.ascontiguousarray(data, dtype=np.float64), len(data))

    def get_box(self, id_, iv):
        nc = self.tree.box_size_lvl[int(self.tree.lvl[id_])]
        out = np.empty((nc + 2) ** 3)
        self.L.orc_get_box(self.h, int(id_), iv, out)
        return out.reshape((nc + 2,) * 3)  # [k][j][i]

    def set_box(self, id_, iv, arr):
        self.L.orc_set_box(self.h, int(id_), iv, np.ascontiguousarray(arr, dtype=np.float64).reshape(-1))

    def get_level(self, lvl, iv, ids=None):
        ids = self.tree.lvls[lvl].ids if ids is None else ids
        return np.stack([self.get_box(i, iv) for i in ids]) if len(ids) else None

    def set_level(self, lvl, iv, data, ids=None):
        ids = self.tree.lvls[lvl].ids if ids is None else ids
        for n, i in enumerate(ids):
            self.set_box(i, iv, data[n])

    def fas_vcycle(self, highest_lvl=None, want_max_res=False, standalone=True):
        r = C.c_double(0.0)
        hl = self.tree.lowest_lvl - 1 if highest_lvl is None else highest_lvl
        self.L.orc_fas_vcycle(self.h, hl, int(want_max_res), C.byref(r), int(standalone))
        return r.value

    def fas_fmg(self, have_guess, want_max_res=False):
        r = C.c_double(0.0)
        self.L.orc_fas_fmg(self.h, int(have_guess), int(want_max_res), C.byref(r))
        return r.value

    def diffusion_solve(self, op, dt, coeff, order, max_res):
        """m_diffusion's time step (orc_diffusion_solve): (status, n_vcycles, res)."""
        n, r = C.c_int(0), C.c_double(0.0)
        rc = self.L.orc_diffusion_solve(self.h, op, dt, coeff, order, max_res, C.byref(n), C.byref(r))
        return rc, n.value, r.value

    def __getattr__(self, name):
        # thin pass-through: orc.<fn>(args) -> liboracle.orc_<fn>(h, args)
        f = getattr(lib(), "orc_" + name)
        return lambda *a: f(self.h, *a)
