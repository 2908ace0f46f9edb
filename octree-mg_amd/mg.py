"""Python host mirror of the reference octree-mg API (``m_octree_mg``).

Same names, argument meaning and error behaviour as the Fortran library the
reference's tests call (tests/test_uniform_grid.f90:77-105):

    mg = MG()                                # type(mg_t) :: mg
    mg.smoother_type = MG_SMOOTHER_GSRB
    mg.bc[nb][MG_IPHI] = BC(MG_BC_DIRICHLET, 0.0)   # or .boundary_cond = f
    mg_set_methods(mg)
    mg_comm_init(mg)
    mg_build_rectangle(mg, domain_size, box_size, dr, r_min, periodic, n_finer)
    mg_load_balance(mg)
    mg_allocate_storage(mg)                  # device arenas live here
    mg_fas_vcycle(mg) / mg_fas_fmg(mg, have_guess, max_res=True)

Host-side tree bookkeeping runs in tree.py; every per-level step runs as HIP
kernels in libomg.so through the C-ABI (device.py).  Box data is exchanged
per level as arrays [box, k, j, i] of the reference's cc(0:nc+1,...) layout.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import device
from .tree import (MG_AHELMHOLTZ, MG_VHELMHOLTZ, MG_VLAPLACIAN, MG_BC_DIRICHLET, MG_CARTESIAN, MG_HELMHOLTZ,
                   MG_IPHI, MG_LAPLACIAN, MG_NO_BOX, MG_NUM_VARS,
                   MG_SMOOTHER_GS, MG_SMOOTHER_GSRB, MGLevel, MGTree)


class BC:
    """mg_bc_t (reference: src/m_data_structures.f90:235-242)."""

    def __init__(self, bc_type=MG_BC_DIRICHLET, bc_value=0.0, boundary_cond=None, refinement_bnd=None):
        self.bc_type = bc_type
        self.bc_value = bc_value
        # boundary_cond(mg, id, nc, iv, nb) -> (bc_type, values[nc*nc], first index fastest)
        self.boundary_cond = boundary_cond
        # refinement_bnd(mg, id, nc, iv, nb, cgc, cc): mg_subr_rb (:364-378);
        # cgc [c-1, a-1] the coarse face (box_gc_for_fine_neighbor), cc
        # [k, j, i] (0..nc+1) the box's variable iv, whose face-nb ghosts it
        # sets in place (omg_set_refinement_bnd: called after every ghost fill)
        self.refinement_bnd = refinement_bnd


# omg_rb_fn (include/omg.h)
_RB_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                     C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double))


class MG(MGTree):
    """mg_t: tree (host) + device context (HIP)."""

    def __init__(self):
        super().__init__()
        self.is_allocated = False
        self.n_extra_vars = 0
        self.comm = None
        self.operator_type = MG_LAPLACIAN
        self.geometry_type = MG_CARTESIAN
        self.n_smoother_substeps = 1
        self.n_cycle_down = 2
        self.n_cycle_up = 2
        self.max_coarse_cycles = 1000
        self.residual_coarse_abs = 1e-8
        self.residual_coarse_rel = 1e-8
        self.helmholtz_lambda = 0.0
        self.methods_set = False
        self.bc = [[BC() for _ in range(17)] for _ in range(7)]   # bc[nb][iv], 1-based
        self.ctx: device.Context | None = None
        self.device_index = 0
        self._uid = None
        # replicate coarse levels of up to this many cells on every rank
        # (omg_set_coarse_replication; 0 = split them like the reference)
        self.coarse_replication_cells = 0

    # -- data access -------------------------------------------------------
    @property
    def n_vars(self):
        return MG_NUM_VARS + self.n_extra_vars

    def set_level(self, lvl, iv, data):
        """Upload variable iv of all my_ids boxes at lvl ([box, k, j, i])."""
        self._require_alloc()
        self.ctx.upload_level(lvl, iv, data)

    def get_level(self, lvl, iv):
        self._require_alloc()
        return self.ctx.download_level(lvl, iv)

    def _require_alloc(self):
        if not self.is_allocated:
            raise RuntimeError("allocate_storage: tree is not allocated")

    # -- device configuration (mg_set_methods) ---------------------------
    def _push_methods(self):
        c = self.ctx
        c.call("set_operator", self.operator_type, float(self.helmholtz_lambda))
        c.call("set_smoother", self.smoother_type, self.n_cycle_down, self.n_cycle_up,
               self.max_coarse_cycles, self.residual_coarse_abs, self.residual_coarse_rel)
        c.call("set_subtract_mean", int(self.subtract_mean))

    def _rb_trampoline(self, iv, nb, cb):
        def fn(user, lvl, iv_, n, ids, nbs, nc, cgc, cc):
            try:
                s = nc + 2
                g = np.ctypeslib.as_array(cgc, shape=(n, nc, nc))
                a = np.ctypeslib.as_array(cc, shape=(n, s, s, s))
                for q in range(n):
                    cb(self, int(ids[q]), nc, iv_, int(nbs[q]), g[q], a[q])
            except BaseException as ex:  # noqa: BLE001  (no exception may cross the C frame)
                self._rb_error = ex
        return _RB_FN(fn)

    def _raise_rb_error(self):
        ex = getattr(self, "_rb_error", None)
        if ex is not None:
            self._rb_error = None
            raise ex

    def push_bc(self, ivs=None):
        """Send mg%bc to the device; boundary_cond callbacks are tabulated per
        physical face of my boxes (they are pure functions of box geometry);
        refinement_bnd callbacks are handed to omg_set_refinement_bnd."""
        c = self.ctx
        ivs = range(1, self.n_vars + 1) if ivs is None else ivs
        if not hasattr(self, "_rb_keep"):
            self._rb_keep = {}
            c.after_call = self._raise_rb_error
        for iv in ivs:
            for nb in range(1, 7):
                cb = self.bc[nb][iv].refinement_bnd
                had = self._rb_keep.get((iv, nb)) is not None
                fp = self._rb_keep[(iv, nb)] = self._rb_trampoline(iv, nb, cb) if cb else None
                if fp or had:   # (nothing to clear otherwise: older libraries lack the entry)
                    c.call("set_refinement_bnd", iv, nb, C.cast(fp, C.c_void_p) if fp else None, None)
            cbs = [self.bc[nb][iv].boundary_cond for nb in range(1, 7)]
            for nb in range(1, 7):
                b = self.bc[nb][iv]
                c.call("set_bc", iv, nb, int(b.bc_type), float(b.bc_value))
            if any(cb is not None for cb in cbs):
                n = self.n_boxes
                face_off = np.full(n * 6, -1, dtype=np.int64)
                face_type = np.zeros(n * 6, dtype=np.int32)
                chunks, pos = [], 0
                rep = c.replicated_level()
                for lvl in range(self.lowest_lvl, self.highest_lvl + 1):
                    nc = self.box_size_lvl[lvl]
                    # a replicated level needs the table of every box
                    for id_ in (self.lvls[lvl].ids if lvl <= rep else self.lvls[lvl].my_ids):
                        for nb in range(1, 7):
                            if self.neighbors[id_, nb - 1] < MG_NO_BOX and cbs[nb - 1] is not None:
                                t, vals = cbs[nb - 1](self, int(id_), nc, iv, nb)
                                vals = np.ascontiguousarray(vals, dtype=np.float64).reshape(-1)
                                face_off[(id_ - 1) * 6 + nb - 1] = pos
                                face_type[(id_ - 1) * 6 + nb - 1] = t
                                chunks.append(vals)
                                pos += vals.size
                data = np.concatenate(chunks) if chunks else np.zeros(1)
                c.call("set_bc_faces", iv, face_off, face_type, data, len(data))


# ---------------------------------------------------------------------------
# The public procedures (names as in the reference's m_octree_mg)

class Loopback:
    """Communicator of an in-process loopback group: n_ranks MG objects of one
    process, one host thread each, sharing a GPU (include/omg.h,
    omg_loopback_unique_id).  Used to run the multi-rank path on one GPU."""

    def __init__(self, tag: int, rank: int, n_ranks: int):
        self.tag, self.rank, self.n_ranks = int(tag), int(rank), int(n_ranks)


def mg_comm_init(mg: MG, comm=None):
    """mg_comm_init (reference: src/m_communication.f90:14-35).  Ranks come
    from torch.distributed when it is initialised (or from a Loopback
    communicator), else a single rank."""
    if isinstance(comm, Loopback):
        mg.comm, mg.my_rank, mg.n_cpu = comm, comm.rank, comm.n_ranks
        return
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            mg.comm = comm or dist.group.WORLD
            mg.my_rank = dist.get_rank()
            mg.n_cpu = dist.get_world_size()
            return
    except ImportError:
        pass
    mg.comm = None
    mg.my_rank = 0
    mg.n_cpu = 1


def mg_set_methods(mg: MG):
    """mg_set_methods (reference: src/m_multigrid.f90:27-60)."""
    if mg.operator_type == MG_LAPLACIAN:
        if np.all(mg.periodic):
            mg.subtract_mean = True
    elif mg.operator_type == MG_HELMHOLTZ:
        mg.subtract_mean = False
    elif mg.operator_type in (MG_VLAPLACIAN, MG_VHELMHOLTZ):
        # vlaplacian_set_methods / vhelmholtz_set_methods (m_vlaplacian.f90:13-49,
        # m_vhelmholtz.f90:19-49): eps in var 5 with Neumann-0 ghosts
        mg.n_extra_vars = max(1, mg.n_extra_vars)
        mg.subtract_mean = False
        for nb in range(1, 7):
            mg.bc[nb][5] = BC(-11, 0.0)
    elif mg.operator_type == MG_AHELMHOLTZ:
        mg.n_extra_vars = max(3, mg.n_extra_vars)
        for nb in range(1, 7):
            for iv in (5, 6, 7):
                mg.bc[nb][iv] = BC(-11, 0.0)
    else:
        raise RuntimeError("mg_set_methods: unknown operator")
    if mg.smoother_type not in (MG_SMOOTHER_GS, MG_SMOOTHER_GSRB):
        raise RuntimeError("unsupported smoother type")
    mg.n_smoother_substeps = 2 if mg.smoother_type == MG_SMOOTHER_GSRB else 1
    mg.methods_set = True
    if mg.ctx is not None:
        mg._push_methods()


def helmholtz_set_lambda(mg: MG, lam: float):
    """helmholtz_set_lambda (reference: src/m_helmholtz.f90:39-46)."""
    if lam < 0:
        raise RuntimeError("helmholtz_set_lambda: lambda < 0 not allowed")
    mg.helmholtz_lambda = float(lam)
    if mg.ctx is not None:
        mg._push_methods()


def mg_build_rectangle(mg: MG, domain_size, box_size, dx, r_min, periodic, n_finer=0):
    mg.build_rectangle(domain_size, box_size, dx, r_min, periodic, n_finer)


def mg_load_balance(mg: MG):
    mg.load_balance()


def mg_load_balance_parents(mg: MG):
    mg.load_balance_parents()


def mg_load_balance_simple(mg: MG):
    mg.load_balance_simple()


def mg_add_children(mg: MG, id_):
    mg.add_children(id_)


def _tree_arrays(mg: MG):
    n = mg.n_boxes
    i32 = lambda a: np.ascontiguousarray(np.asarray(a)[1:n + 1], dtype=np.int32).reshape(-1)
    lo, hi = mg.lowest_lvl, mg.highest_lvl
    bsl = np.array([mg.box_size_lvl[l] for l in range(lo, hi + 1)], dtype=np.int32)
    dr = np.ascontiguousarray(np.array([mg.dr[l] for l in range(lo, hi + 1)],
                                       dtype=np.float64).reshape(-1))
    off, data = [0], []
    for l in range(lo, hi + 1):
        L = mg.lvls[l]
        for arr in (L.ids, L.leaves, L.parents, L.ref_bnds):
            data.extend(int(x) for x in arr)
            off.append(len(data))
    return (i32(mg.lvl), i32(mg.parent), i32(mg.children), i32(mg.neighbors), i32(mg.ix),
            i32(mg.rank), bsl, dr, np.array(off, dtype=np.int32),
            np.array(data if data else [0], dtype=np.int32))


def mg_allocate_storage(mg: MG, device_index=None):
    """mg_allocate_storage (reference: src/m_allocate_storage.f90:51-99): the
    device arenas of every level this rank owns boxes on, zero-initialised."""
    if not mg.tree_created:
        raise RuntimeError("allocate_storage: tree is not yet created")
    if mg.is_allocated:
        raise RuntimeError("allocate_storage: tree is already allocated")
    if device_index is None:
        device_index = int(os.environ.get("LOCAL_RANK", mg.device_index if mg.n_cpu == 1 else 0))
    uid = None
    host = False
    if isinstance(mg.comm, Loopback):
        uid = device.loopback_unique_id(mg.comm.tag) if mg.comm.n_ranks > 1 else None
        device_index = 0
    elif mg.n_cpu > 1:
        import torch.distributed as dist
        host = _use_host_transport(mg)
        if host:
            # ranks share a GPU (RCCL refuses that): the host transport over
            # the torch.distributed group, rank r on GPU r mod ndev
            uid = device.host_unique_id()
            device_index = mg.my_rank % max(device.device_count(), 1)
        else:
            obj = [device.unique_id() if mg.my_rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            uid = obj[0]
    mg.ctx = device.Context(device_index, mg.my_rank, mg.n_cpu, uid)
    if host:
        mg.ctx.set_host_transport(mg.comm)
    if mg.coarse_replication_cells:
        mg.ctx.call("set_coarse_replication", int(mg.coarse_replication_cells))
    arrs = _tree_arrays(mg)
    mg.ctx.call("tree_setup", mg.n_boxes, *arrs[:6], mg.lowest_lvl, mg.highest_lvl,
                mg.first_normal_lvl, mg.box_size, arrs[6], arrs[7], arrs[8], arrs[9], mg.n_vars)
    mg.is_allocated = True
    mg._push_methods()
    mg.push_bc()


def _use_host_transport(mg: MG) -> bool:
    """The host transport when this node's ranks outnumber its visible GPUs
    or OMG_TRANSPORT=host; agreed over the group (as the Fortran drop-in
    does).  The node's ranks: LOCAL_WORLD_SIZE (torchrun, bench.py's own
    launcher), else every rank of the group (one node)."""
    import torch
    import torch.distributed as dist
    n_node = int(os.environ.get("LOCAL_WORLD_SIZE", mg.n_cpu))
    want = os.environ.get("OMG_TRANSPORT") == "host" or device.device_count() < n_node
    t = torch.tensor([1 if want else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=mg.comm)
    return bool(t[0])


def mg_deallocate_storage(mg: MG):
    if not mg.is_allocated:
        raise RuntimeError("deallocate_storage: tree is not allocated")
    mg.ctx.close()
    mg.ctx = None
    # as src/m_allocate_storage.f90:14-47: the level lists go, the tree is empty
    for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
        mg.lvls[lvl] = MGLevel()
    mg.n_boxes = 0
    mg.is_allocated = False


def _check_methods(mg):
    if not mg.methods_set:
        mg_set_methods(mg)


def mg_fas_vcycle(mg: MG, highest_lvl=None, max_res=False, standalone=True):
    """mg_fas_vcycle (reference: src/m_multigrid.f90:150-243).  Returns the
    max residual when max_res is requested, else None."""
    _check_methods(mg)
    mg._require_alloc()
    hl = mg.lowest_lvl - 1 if highest_lvl is None else int(highest_lvl)
    r = C.c_double(0.0)
    mg.ctx.call("fas_vcycle", hl, int(bool(max_res)), C.byref(r), int(bool(standalone)))
    return r.value if max_res else None


def mg_fas_fmg(mg: MG, have_guess, max_res=False):
    """mg_fas_fmg (reference: src/m_multigrid.f90:84-147)."""
    _check_methods(mg)
    mg._require_alloc()
    r = C.c_double(0.0)
    mg.ctx.call("fas_fmg", int(bool(have_guess)), int(bool(max_res)), C.byref(r))
    return r.value if max_res else None


def mg_apply_op(mg: MG, i_out):
    """mg_apply_op (reference: src/m_multigrid.f90:439-456)."""
    mg.ctx.call("apply_op", i_out)


def mg_restrict(mg: MG, iv):
    mg.ctx.call("restrict", iv)


def mg_restrict_lvl(mg: MG, iv, lvl):
    mg.ctx.call("restrict_lvl", iv, lvl)


def mg_fill_ghost_cells(mg: MG, iv):
    mg.ctx.call("fill_ghost_cells", iv)


def mg_fill_ghost_cells_lvl(mg: MG, lvl, iv):
    mg.ctx.call("fill_ghost_cells_lvl", lvl, iv)


def mg_prolong(mg: MG, lvl, iv, iv_to, add):
    mg.ctx.call("prolong", lvl, iv, iv_to, int(bool(add)))


def mg_phi_bc_store(mg: MG):
    """mg_phi_bc_store (reference: src/m_ghost_cells.f90:66-117): phi's bc
    values move into the rhs ghost cells on the device."""
    mg.ctx.call("phi_bc_store")
    mg.phi_bc_data_stored = True
