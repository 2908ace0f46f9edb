"""Host-side octree bookkeeping: the ``mg_t`` tree type and its set-up routines.

This is the Python host mirror of the reference's kept host modules
(``m_data_structures`` types, ``m_build_tree``, ``m_load_balance``); it runs
once at set-up and produces the tree every rank holds in full.  Box ids are
1-based, id 0 is ``mg_no_box`` and negative neighbour ids are physical
boundaries, exactly as in the reference, so the tree can be compared entry by
entry with the Fortran one and handed to the device plan builder unchanged.

Citations are ``path:line`` in the reference repository.
"""
from __future__ import annotations

import numpy as np

# Constants (reference: src/m_data_structures.f90:14-84)
MG_LAPLACIAN, MG_VLAPLACIAN, MG_HELMHOLTZ, MG_VHELMHOLTZ, MG_AHELMHOLTZ = 1, 2, 3, 4, 5
MG_CARTESIAN = 1
MG_SMOOTHER_GS, MG_SMOOTHER_GSRB, MG_SMOOTHER_JACOBI = 1, 2, 3
MG_NUM_VARS = 4
MG_IPHI, MG_IRHS, MG_IOLD, MG_IRES = 1, 2, 3, 4
MG_IVEPS, MG_IVEPS1, MG_IVEPS2, MG_IVEPS3 = 5, 5, 6, 7
MG_LVL_LO, MG_LVL_HI = -20, 20
MG_BC_DIRICHLET, MG_BC_NEUMANN, MG_BC_CONTINUOUS = -10, -11, -12
MG_NO_BOX, MG_PHYSICAL_BOUNDARY = 0, -1
MG_NUM_CHILDREN, MG_NUM_NEIGHBORS = 8, 6

# 3D topology tables (reference: src/m_data_structures.f90:155-190), 0-based
# child/neighbour slots here; values as in the reference.
CHILD_DIX = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0],
                      [0, 0, 1], [1, 0, 1], [0, 1, 1], [1, 1, 1]], dtype=np.int64)
# children (1-based child index) adjacent to neighbour direction nb
CHILD_ADJ_NB = np.array([[1, 3, 5, 7], [2, 4, 6, 8], [1, 2, 5, 6],
                         [3, 4, 7, 8], [1, 2, 3, 4], [5, 6, 7, 8]], dtype=np.int64)
NEIGHB_REV = np.array([2, 1, 4, 3, 6, 5], dtype=np.int64)      # 1-based values
NEIGHB_DIM = np.array([1, 1, 2, 2, 3, 3], dtype=np.int64)
NEIGHB_LOW = np.array([True, False, True, False, True, False])
NEIGHB_HIGH_PM = np.array([-1, 1, -1, 1, -1, 1], dtype=np.int64)


def ix_to_ichild(ix) -> int:
    """mg_ix_to_ichild (reference: src/m_data_structures.f90:440-451)."""
    return 8 - 4 * (int(ix[2]) & 1) - 2 * (int(ix[1]) & 1) - (int(ix[0]) & 1)


def child_low(d: int, c_ix: int) -> bool:
    """mg_child_low(d, c_ix) (reference: src/m_data_structures.f90:165-169)."""
    return CHILD_DIX[c_ix - 1, d - 1] == 0


# mg_child_rev (reference: src/m_data_structures.f90:159-160)
_CHILD_REV = [[2, 1, 4, 3, 6, 5, 8, 7], [3, 4, 1, 2, 7, 8, 5, 6], [5, 6, 7, 8, 1, 2, 3, 4]]


class MGLevel:
    """mg_lvl_t (reference: src/m_data_structures.f90:194-203)."""

    def __init__(self):
        e = np.zeros(0, dtype=np.int64)
        self.ids, self.leaves, self.parents, self.ref_bnds = e, e, e, e
        self.my_ids, self.my_leaves, self.my_parents, self.my_ref_bnds = e, e, e, e


class MGTree:
    """The tree part of mg_t (reference: src/m_data_structures.f90:250-342)."""

    def __init__(self):
        self.tree_created = False
        self.n_cpu = 1
        self.my_rank = 0
        self.box_size = -1
        self.highest_lvl = -1
        self.lowest_lvl = -1
        self.first_normal_lvl = -1
        self.n_boxes = 0
        self.box_size_lvl = {}
        self.domain_size_lvl = {}
        self.dr = {}
        self.r_min = np.zeros(3)
        self.periodic = np.zeros(3, dtype=bool)
        self.smoother_type = MG_SMOOTHER_GS
        self.coarsest_grid = np.array([2, 2, 2], dtype=np.int64)
        self.subtract_mean = False
        self.lvls = {l: MGLevel() for l in range(MG_LVL_LO, MG_LVL_HI + 1)}
        # per-box arrays, index = id (0 unused)
        self._cap = 0

    # -- storage -----------------------------------------------------------
    def _alloc(self, n: int):
        self._cap = n
        self.rank = np.zeros(n + 1, dtype=np.int64)
        self.lvl = np.zeros(n + 1, dtype=np.int64)
        self.ix = np.zeros((n + 1, 3), dtype=np.int64)
        self.parent = np.zeros(n + 1, dtype=np.int64)
        self.children = np.zeros((n + 1, 8), dtype=np.int64)
        self.neighbors = np.zeros((n + 1, 6), dtype=np.int64)
        self.box_r_min = np.zeros((n + 1, 3))
        self.box_dr = np.zeros((n + 1, 3))

    def has_children(self, ids):
        """mg_has_children (reference: src/m_data_structures.f90:430-436)."""
        return self.children[ids, 0] != MG_NO_BOX

    def get_child_offset(self, id_: int) -> np.ndarray:
        """mg_get_child_offset (reference: src/m_data_structures.f90:456-467)."""
        if self.lvl[id_] <= self.first_normal_lvl:
            return np.zeros(3, dtype=np.int64)
        return ((self.ix[id_] - 1) & 1) * (self.box_size >> 1)

    # -- m_build_tree ------------------------------------------------------
    def build_rectangle(self, domain_size, box_size, dx, r_min, periodic, n_finer=0):
        """mg_build_rectangle (reference: src/m_build_tree.f90:18-174)."""
        domain_size = np.asarray(domain_size, dtype=np.int64)
        dx = np.asarray(dx, dtype=np.float64)
        r_min = np.asarray(r_min, dtype=np.float64)
        periodic = np.asarray(periodic, dtype=bool)
        if box_size % 2 != 0:
            raise RuntimeError("box_size should be even")
        if np.any(domain_size % box_size != 0):
            raise RuntimeError("box_size does not divide domain_size")
        if np.all(periodic):
            self.subtract_mean = True

        nx = domain_size.copy()
        self.box_size = int(box_size)
        self.box_size_lvl = {1: int(box_size)}
        self.domain_size_lvl = {1: domain_size.copy()}
        self.first_normal_lvl = 1
        self.dr = {1: dx.copy()}
        self.r_min = r_min.copy()
        self.periodic = periodic.copy()
        bpd = {1: domain_size // box_size}

        lvl = 1
        while lvl >= MG_LVL_LO + 1:
            if (np.any((nx % 2 == 1) | (nx == self.coarsest_grid)) or
                    (self.box_size_lvl[lvl] == self.coarsest_grid[0] and
                     self.smoother_type == MG_SMOOTHER_GS)):
                break
            if np.all((nx // self.box_size_lvl[lvl]) % 2 == 0):
                self.box_size_lvl[lvl - 1] = self.box_size_lvl[lvl]
                bpd[lvl - 1] = bpd[lvl] // 2
                self.first_normal_lvl = lvl - 1
            else:
                self.box_size_lvl[lvl - 1] = self.box_size_lvl[lvl] // 2
                bpd[lvl - 1] = bpd[lvl].copy()
            self.dr[lvl - 1] = self.dr[lvl] * 2
            nx = nx // 2
            self.domain_size_lvl[lvl - 1] = nx.copy()
            lvl -= 1
        self.lowest_lvl = lvl
        self.highest_lvl = 1
        for l in range(2, MG_LVL_HI + 1):
            self.dr[l] = self.dr[l - 1] * 0.5
            self.box_size_lvl[l] = int(box_size)
            self.domain_size_lvl[l] = 2 * self.domain_size_lvl[l - 1]

        n = int(sum(int(np.prod(bpd[l])) for l in bpd)) + int(n_finer)
        self._alloc(n)
        self.n_boxes = 0

        # lowest level, i fastest (KJI_DO_VEC: k outer), reference :95-138
        nxb = bpd[self.lowest_lvl]
        periodic_offset = np.array([nxb[0] - 1, (nxb[1] - 1) * nxb[0],
                                    (nxb[2] - 1) * nxb[1] * nxb[0]], dtype=np.int64)
        bsl = self.box_size_lvl[self.lowest_lvl]
        drl = self.dr[self.lowest_lvl]
        for k in range(1, nxb[2] + 1):
            for j in range(1, nxb[1] + 1):
                for i in range(1, nxb[0] + 1):
                    self.n_boxes += 1
                    n = self.n_boxes
                    ijk = np.array([i, j, k], dtype=np.int64)
                    self.rank[n] = 0
                    self.lvl[n] = self.lowest_lvl
                    self.ix[n] = ijk
                    self.box_r_min[n] = r_min + ((ijk - 1) * bsl).astype(np.float64) * drl
                    self.box_dr[n] = drl
                    self.parent[n] = MG_NO_BOX
                    self.children[n] = MG_NO_BOX
                    self.neighbors[n] = [n - 1, n + 1, n - nxb[0], n + nxb[0],
                                         n - nxb[0] * nxb[1], n + nxb[0] * nxb[1]]
                    for d in range(3):
                        if ijk[d] == 1:
                            self.neighbors[n, 2 * d] = (n + periodic_offset[d] if periodic[d]
                                                        else MG_PHYSICAL_BOUNDARY)
                        if ijk[d] == nxb[d]:
                            self.neighbors[n, 2 * d + 1] = (n - periodic_offset[d] if periodic[d]
                                                            else MG_PHYSICAL_BOUNDARY)
        self.lvls[self.lowest_lvl].ids = np.arange(1, self.n_boxes + 1, dtype=np.int64)

        for l in range(self.lowest_lvl, 1):
            ids = self.lvls[l].ids
            if self.box_size_lvl[l + 1] == self.box_size_lvl[l]:
                for id_ in ids:
                    self.add_children(int(id_))
                self.set_leaves_parents(l)
                self.set_next_level_ids(l)
                self.set_neighbors_lvl(l + 1)
            else:
                for id_ in ids:
                    self._add_single_child(int(id_), len(ids))
                self.set_leaves_parents(l)
                self.set_next_level_ids(l)
        self.set_leaves_parents(1)
        for l in range(self.lowest_lvl, 2):
            self.lvls[l].ref_bnds = np.zeros(0, dtype=np.int64)
        self.tree_created = True

    def set_neighbors_lvl(self, lvl):
        """mg_set_neighbors_lvl (reference: src/m_build_tree.f90:176-185)."""
        for id_ in self.lvls[lvl].ids:
            self._set_neighbs(int(id_))

    def set_next_level_ids(self, lvl):
        """mg_set_next_level_ids (reference: src/m_build_tree.f90:187-216)."""
        parents = self.lvls[lvl].parents
        if self.box_size_lvl[lvl + 1] == self.box_size_lvl[lvl]:
            self.lvls[lvl + 1].ids = self.children[parents].reshape(-1).copy()
        else:
            self.lvls[lvl + 1].ids = self.children[parents, 0].copy()

    def _set_neighbs(self, id_):
        """set_neighbs (reference: src/m_build_tree.f90:219-233)."""
        for nb in range(1, 7):
            if self.neighbors[id_, nb - 1] == MG_NO_BOX:
                nb_id = self._find_neighb(id_, nb)
                if nb_id > MG_NO_BOX:
                    self.neighbors[id_, nb - 1] = nb_id
                    self.neighbors[nb_id, NEIGHB_REV[nb - 1] - 1] = id_

    def _find_neighb(self, id_, nb):
        """find_neighb (reference: src/m_build_tree.f90:236-255)."""
        p_id = int(self.parent[id_])
        c_ix = ix_to_ichild(self.ix[id_])
        d = int(NEIGHB_DIM[nb - 1])
        if child_low(d, c_ix) == bool(NEIGHB_LOW[nb - 1]):
            p_id = int(self.neighbors[p_id, nb - 1])
        return int(self.children[p_id, _CHILD_REV[d - 1][c_ix - 1] - 1])

    def set_leaves_parents(self, lvl):
        """mg_set_leaves_parents (reference: src/m_build_tree.f90:258-293)."""
        ids = self.lvls[lvl].ids
        hc = self.has_children(ids)
        self.lvls[lvl].parents = ids[hc].copy()
        self.lvls[lvl].leaves = ids[~hc].copy()

    def set_refinement_boundaries(self, lvl):
        """mg_set_refinement_boundaries (reference: src/m_build_tree.f90:296-328)."""
        L = self.lvls[lvl]
        if len(L.parents) == 0:
            L.ref_bnds = np.zeros(0, dtype=np.int64)
            return
        out = []
        for id_ in L.leaves:
            for nb in range(6):
                nb_id = self.neighbors[id_, nb]
                if nb_id > MG_NO_BOX and self.children[nb_id, 0] != MG_NO_BOX:
                    out.append(int(id_))
                    break
        L.ref_bnds = np.array(out, dtype=np.int64)

    def add_children(self, id_):
        """mg_add_children (reference: src/m_build_tree.f90:330-367)."""
        if self.n_boxes + 8 > self._cap:
            raise RuntimeError("mg_add_children: not enough space")
        c_ids = np.arange(self.n_boxes + 1, self.n_boxes + 9, dtype=np.int64)
        self.n_boxes += 8
        self.children[id_] = c_ids
        c_ix_base = 2 * self.ix[id_] - 1
        lvl = int(self.lvl[id_]) + 1
        drl = self.dr[lvl]
        for i in range(8):
            c = c_ids[i]
            self.rank[c] = self.rank[id_]
            self.ix[c] = c_ix_base + CHILD_DIX[i]
            self.lvl[c] = lvl
            self.parent[c] = id_
            self.children[c] = MG_NO_BOX
            self.neighbors[c] = MG_NO_BOX
            self.box_r_min[c] = (self.box_r_min[id_] +
                                 drl * CHILD_DIX[i].astype(np.float64) * float(self.box_size))
            self.box_dr[c] = drl
        for nb in range(6):
            if self.neighbors[id_, nb] < MG_NO_BOX:
                child_nb = c_ids[CHILD_ADJ_NB[nb] - 1]
                self.neighbors[child_nb, nb] = self.neighbors[id_, nb]

    def _add_single_child(self, id_, n_boxes_lvl):
        """add_single_child (reference: src/m_build_tree.f90:369-393)."""
        self.n_boxes += 1
        c = self.n_boxes
        self.children[id_, 0] = c
        lvl = int(self.lvl[id_]) + 1
        self.rank[c] = self.rank[id_]
        self.ix[c] = self.ix[id_]
        self.lvl[c] = lvl
        self.parent[c] = id_
        self.children[c] = MG_NO_BOX
        nbs = self.neighbors[id_]
        self.neighbors[c] = np.where(nbs == MG_PHYSICAL_BOUNDARY, nbs, nbs + n_boxes_lvl)
        self.box_r_min[c] = self.box_r_min[id_]
        self.box_dr[c] = self.dr[lvl]

    # -- m_load_balance ----------------------------------------------------
    @staticmethod
    def _most_popular(lst, work, n_cpu):
        """most_popular (reference: src/m_load_balance.f90:197-221)."""
        best_count, best_work, best = 0, 0, -1
        for r in lst:
            r = int(r)
            cnt = int(np.count_nonzero(lst == r))
            w = int(work[r])
            if cnt > best_count or (cnt == best_count and w < best_work):
                best_count, best_work, best = cnt, w, r
        return best

    def load_balance(self):
        """mg_load_balance (reference: src/m_load_balance.f90:71-136)."""
        n_cpu = self.n_cpu
        single = max(self.first_normal_lvl - 1, self.lowest_lvl)
        my_work = np.zeros(n_cpu + 1, dtype=np.int64)
        for lvl in range(self.highest_lvl, single, -1):
            my_work[:] = 0
            for id_ in self.lvls[lvl].parents:
                i_cpu = self._most_popular(self.rank[self.children[id_]], my_work, n_cpu)
                self.rank[id_] = i_cpu
                my_work[i_cpu] += 1
            leaves = self.lvls[lvl].leaves
            work_left = len(leaves)
            i_cpu = 0
            for id_ in leaves:
                if (n_cpu - i_cpu - 1) * my_work[i_cpu] >= work_left + my_work[i_cpu + 1:].sum():
                    i_cpu += 1
                my_work[i_cpu] += 1
                work_left -= 1
                self.rank[id_] = i_cpu
        if single < self.highest_lvl:
            coarse_rank = self._most_popular(self.rank[self.lvls[single + 1].ids], my_work, n_cpu)
        else:
            coarse_rank = 0
        for lvl in range(self.lowest_lvl, single + 1):
            self.rank[self.lvls[lvl].ids] = coarse_rank
        for lvl in range(self.lowest_lvl, self.highest_lvl + 1):
            self._update_lvl_info(lvl)

    def load_balance_parents(self):
        """mg_load_balance_parents (reference: src/m_load_balance.f90:140-193)."""
        n_cpu = self.n_cpu
        single = max(self.first_normal_lvl - 1, self.lowest_lvl)
        my_work = np.zeros(n_cpu + 1, dtype=np.int64)
        for lvl in range(self.highest_lvl - 1, single, -1):
            my_work[:] = 0
            for id_ in self.lvls[lvl].leaves:
                my_work[self.rank[id_]] += 1
            for id_ in self.lvls[lvl].parents:
                i_cpu = self._most_popular(self.rank[self.children[id_]], my_work, n_cpu)
                self.rank[id_] = i_cpu
                my_work[i_cpu] += 1
        if single < self.highest_lvl:
            coarse_rank = self._most_popular(self.rank[self.lvls[single + 1].ids], my_work, n_cpu)
        else:
            coarse_rank = 0
        for lvl in range(self.lowest_lvl, single + 1):
            self.rank[self.lvls[lvl].ids] = coarse_rank
        for lvl in range(self.lowest_lvl, self.highest_lvl + 1):
            self._update_lvl_info(lvl)

    def load_balance_simple(self):
        """mg_load_balance_simple (reference: src/m_load_balance.f90:22-63)."""
        n_cpu = self.n_cpu
        single = max(self.first_normal_lvl - 1, self.lowest_lvl)
        for lvl in range(self.lowest_lvl, single + 1):
            self.rank[self.lvls[lvl].ids] = 0
        for lvl in range(single + 1, self.highest_lvl + 1):
            ids = self.lvls[lvl].ids
            work_left, my_work, i_cpu = len(ids), 0, 0
            for id_ in ids:
                if (n_cpu - i_cpu - 1) * my_work >= work_left:
                    i_cpu += 1
                    my_work = 0
                my_work += 1
                work_left -= 1
                self.rank[id_] = i_cpu
        for lvl in range(self.lowest_lvl, self.highest_lvl + 1):
            self._update_lvl_info(lvl)

    def _update_lvl_info(self, lvl):
        """update_lvl_info (reference: src/m_load_balance.f90:223-235)."""
        L = self.lvls[lvl]
        r = self.my_rank
        L.my_ids = L.ids[self.rank[L.ids] == r]
        L.my_leaves = L.leaves[self.rank[L.leaves] == r]
        L.my_parents = L.parents[self.rank[L.parents] == r]
        L.my_ref_bnds = L.ref_bnds[self.rank[L.ref_bnds] == r]

    # -- geometry helpers --------------------------------------------------
    def get_face_coords(self, id_, nb, nc):
        """mg_get_face_coords, 3D (reference: src/m_data_structures.f90:495-539).

        Returns x(nc, nc, 3) as an array indexed [i-1, j-1, :] (i along the
        first tangential dimension)."""
        nb_dim = int(NEIGHB_DIM[nb - 1])
        ixs = [d for d in (1, 2, 3) if d != nb_dim]
        rmin = self.box_r_min[id_].copy()
        dr = self.box_dr[id_]
        if not NEIGHB_LOW[nb - 1]:
            rmin[nb_dim - 1] = rmin[nb_dim - 1] + dr[nb_dim - 1] * nc
        x = np.empty((nc, nc, 3))
        x[:, :, :] = rmin
        ii = (np.arange(1, nc + 1) - 0.5)
        x[:, :, ixs[0] - 1] = rmin[ixs[0] - 1] + ii[:, None] * dr[ixs[0] - 1]
        x[:, :, ixs[1] - 1] = rmin[ixs[1] - 1] + ii[None, :] * dr[ixs[1] - 1]
        return x

    def number_of_unknowns(self):
        """mg_number_of_unknowns (reference: src/m_data_structures.f90:482-492)."""
        n = sum(len(self.lvls[l].leaves) for l in range(self.first_normal_lvl, self.highest_lvl + 1))
        return n * self.box_size ** 3
