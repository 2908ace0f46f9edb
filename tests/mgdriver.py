"""Problem runner shared by the parity tests, smoke() and bench.py.

It replays oracle/omg_golden.f90 (the golden-vector driver that runs the
reference itself) on either backend:

* ``device`` — the product: the Python host mirror (octree_mg_amd.MG) driving
  libomg.so on the GPU through the C-ABI;
* ``oracle`` — the C restatement (oracle/liboracle.so), the checker.

Both start from bit-identical inputs, so their per-iteration histories (and
the sha256 of the final phi of every box) must agree exactly with each other
and with tests/golden/golden.json.
"""
from __future__ import annotations

import hashlib
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__  # noqa: E402

omg = __graft_entry__.load_package()
T = omg.tree
P = omg.problems


def hexbits(x: float) -> str:
    return "%016X" % struct.unpack("<Q", struct.pack("<d", float(x)))[0]


def parse(args: str) -> dict:
    f = args.split()
    return dict(box=int(f[0]), domain=[int(f[1]), int(f[2]), int(f[3])], n_its=int(f[4]),
                cycle=f[5], smoother=f[6], op=f[7], lam=float(f[8]), bc=f[9], rhs=f[10],
                n_levels=int(f[11]), lb=f[12], maxres=int(f[13]))


def regrids(cfg: dict) -> bool:
    """omg_golden's lb suffix "mv": after n_its iterations the tree is rebuilt
    with its refined region moved (AMRVAC's regrid) and n_its more run."""
    return cfg["lb"].endswith("mv")


REGRID_SHIFT = (0.25, -0.25, 0.0)   # omg_golden.f90: the second tree's shift


def build_tree(cfg: dict, tree, n_ranks=1, my_rank=0, shift=(0.0, 0.0, 0.0)):
    """The tree set-up of omg_golden (reference tests' mg_build_rectangle or
    build_amr_tree, tests/test_refinement.f90:191-247, with the refined region
    centred at 0.5 + shift, then load balance)."""
    tree.smoother_type = T.MG_SMOOTHER_GSRB if cfg["smoother"] == "gsrb" else T.MG_SMOOTHER_GS
    tree.n_cpu, tree.my_rank = n_ranks, my_rank
    dom = np.array(cfg["domain"], dtype=np.int64)
    dr = 1.0 / dom.astype(np.float64)
    periodic = [cfg["bc"] == "per"] * 3
    box = cfg["box"]
    if cfg["n_levels"] <= 1:
        tree.build_rectangle(dom, box, dr, [0.0, 0.0, 0.0], periodic, 0)
    else:
        nl = cfg["n_levels"]
        n_finer = nl * int(np.prod(dom // box)) + 1000
        domain_len = dom * dr
        ctr = 0.5 + np.asarray(shift, dtype=np.float64)
        tree.build_rectangle(dom, box, dr, [0.0, 0.0, 0.0], periodic, n_finer)
        for lvl in range(1, nl):
            for id_ in tree.lvls[lvl].ids:
                r0 = ctr * domain_len - domain_len * 0.5 ** (lvl + 1)
                r1 = ctr * domain_len + domain_len * 0.5 ** (lvl + 1)
                center = tree.box_r_min[id_] + 0.5 * box * tree.box_dr[id_]
                if np.all((center >= r0) & (center <= r1)):
                    tree.add_children(int(id_))
            tree.set_leaves_parents(lvl)
            tree.set_next_level_ids(lvl)
            tree.set_neighbors_lvl(lvl + 1)
        tree.set_leaves_parents(nl)
        tree.highest_lvl = nl
        for lvl in range(1, nl + 1):
            tree.set_refinement_boundaries(lvl)
    tree.load_balance()
    if cfg["lb"].startswith("lbp"):
        tree.load_balance_parents()
    return tree


def custom_rb(mg, id_, nc, iv, nb, cgc, cc, k=(0.4, 0.9, -0.3)):
    """omg_golden.f90's custom_rb (a refinement_bnd callback: sides_rb's form
    0.5 gc + 0.75 x1 - 0.25 x2, m_ghost_cells.f90:769-861, with other
    coefficients); k = (0.5, 0.75, -0.25) restates sides_rb itself.
    cgc[c-1, a-1], cc[k, j, i]."""
    low = nb % 2 == 1
    x1, x2, g = (1, 2, 0) if low else (nc, nc - 1, nc + 1)
    d = (nb + 1) // 2
    s = slice(1, nc + 1)
    if d == 1:
        cc[s, s, g] = k[0] * cgc + k[1] * cc[s, s, x1] + k[2] * cc[s, s, x2]
    elif d == 2:
        cc[s, g, s] = k[0] * cgc + k[1] * cc[s, x1, s] + k[2] * cc[s, x2, s]
    else:
        cc[g, s, s] = k[0] * cgc + k[1] * cc[x1, s, s] + k[2] * cc[x2, s, s]


I_EPS = 5   # mg_iveps: the coefficient of the v-operators (vlpl / vhelm)


def is_vop(cfg):
    return cfg["op"] in ("vlpl", "vhelm")


def i_sol(cfg):
    """omg_golden's solution variable: 5, or 6 when var 5 holds eps, or 8
    after the three aniso coefficients."""
    return 8 if cfg["op"] == "ahelm" else 6 if is_vop(cfg) else 5


def n_vars(cfg):
    return i_sol(cfg)


OPS = {"lpl": 1, "vlpl": 2, "helm": 3, "vhelm": 4, "ahelm": 5}

# omg_golden's diffusion runs (cycle d1 / d2): max_res of every step, and the
# coefficient D of diffusion_solve (the v/a forms take none: 1)
DIFF_TOL = 1.0e-8


def diffusion_coeff(cfg):
    return 0.5 if cfg["op"] == "helm" else 1.0


class OracleBackend:
    def __init__(self, cfg, n_ranks=1, shift=(0.0, 0.0, 0.0)):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle  # checker only
        self.cfg = cfg
        if cfg["lb"].endswith("rb"):
            raise NotImplementedError("the oracle has no custom refinement_bnd (its goldens pin the drop-in)")
        self.n_ranks = n_ranks
        self.tree = build_tree(cfg, T.MGTree(), n_ranks, shift=shift)
        self.o = pyoracle.Oracle(self.tree, n_vars(cfg), n_ranks)
        op = OPS[cfg["op"]]
        sm = pyoracle.GSRB if cfg["smoother"] == "gsrb" else pyoracle.GS
        # omg_golden calls mg_set_methods before building the tree, and
        # mg_build_rectangle sets subtract_mean for a fully periodic domain
        # (m_build_tree.f90:36-38) whatever the operator's set_methods cleared
        sub = cfg["bc"] == "per"
        self.o.configure(op=op, lam=cfg["lam"], smoother=sm, subtract_mean=sub)
        _apply_bc(cfg, self.tree, lambda iv, nb, t, v: self.o.set_bc(iv, nb, t, v),
                  lambda iv, a, b, c: self.o.set_bc_faces(iv, a, b, c))

    def levels(self):
        return range(self.tree.lowest_lvl, self.tree.highest_lvl + 1)

    def my_ids(self, lvl):
        return self.tree.lvls[lvl].ids

    def regrid(self, shift):
        """A new oracle over the moved tree (the checker has no storage to free)."""
        self.__init__(self.cfg, self.n_ranks, shift)

    def collective(self, lvl, iv=None):
        return False

    def set_level(self, lvl, iv, data):
        self.o.set_level(lvl, iv, data)

    def get_level(self, lvl, iv):
        return self.o.get_level(lvl, iv)

    def restrict(self, iv):
        self.o.restrict(iv)

    def fill_ghost_cells(self, iv):
        self.o.fill_ghost_cells(iv)

    def apply_op(self, iv):
        self.o.apply_op(iv)

    def vcycle(self, want):
        return self.o.fas_vcycle(want_max_res=bool(want))

    def fmg(self, have_guess, want):
        return self.o.fas_fmg(have_guess, bool(want))

    def diffusion(self, order, dt):
        op = OPS[self.cfg["op"]]
        rc, n, res = self.o.diffusion_solve(op, dt, diffusion_coeff(self.cfg), order, DIFF_TOL)
        if rc == 2:
            raise RuntimeError("diffusion_solve: order should be 1 or 2")
        if rc == 1:
            raise RuntimeError("diffusion_solve: no convergence")
        return res


class DeviceBackend:
    def __init__(self, cfg, comm=None, rep_cells=0):
        self.cfg = cfg
        mg = omg.MG()
        mg.coarse_replication_cells = rep_cells
        mg.n_extra_vars = n_vars(cfg) - 4
        mg.operator_type = OPS[cfg["op"]]
        mg.helmholtz_lambda = cfg["lam"]
        mg.smoother_type = T.MG_SMOOTHER_GSRB if cfg["smoother"] == "gsrb" else T.MG_SMOOTHER_GS
        omg.mg_set_methods(mg)
        omg.mg_comm_init(mg, comm)
        self.mg = mg
        self._build((0.0, 0.0, 0.0))

    def _build(self, shift):
        cfg, mg = self.cfg, self.mg
        # set_methods ran in __init__, before the build, as in omg_golden: the
        # build's subtract_mean for a fully periodic domain stands
        build_tree(cfg, mg, mg.n_cpu, mg.my_rank, shift)

        def set_bc(iv, nb, t, v):
            mg.bc[nb][iv] = omg.BC(t, v)

        faces = {}

        def set_faces(iv, off, typ, data):
            faces[iv] = (off, typ, data)

        _apply_bc(cfg, mg, set_bc, set_faces)
        if cfg["lb"].endswith("rb"):   # omg_golden's custom_rb on phi
            for nb in range(1, 7):
                mg.bc[nb][T.MG_IPHI].refinement_bnd = custom_rb
        omg.mg_allocate_storage(mg)
        for iv, (off, typ, data) in faces.items():
            mg.ctx.call("set_bc_faces", iv, off, typ, data, len(data))
        self.tree = mg
        self.rep_lvl = mg.ctx.replicated_level()

    def regrid(self, shift):
        """omg_golden's "mv" step on the same mg: mg_deallocate_storage, the
        moved tree, load balance, mg_allocate_storage."""
        self.mg.ctx.call("synchronize")
        omg.mg_deallocate_storage(self.mg)
        self._build(shift)

    def levels(self):
        return range(self.mg.lowest_lvl, self.mg.highest_lvl + 1)

    def my_ids(self, lvl):
        return self.mg.lvls[lvl].my_ids

    def collective(self, lvl, iv=None):
        # uploads to a replicated level: every rank calls (omg_set_coarse_replication);
        # so do uploads of phi (the stand-alone fill decision, include/omg.h)
        return lvl <= self.rep_lvl or iv == T.MG_IPHI

    def set_level(self, lvl, iv, data):
        if len(self.my_ids(lvl)) or self.collective(lvl, iv):
            self.mg.set_level(lvl, iv, data)

    def get_level(self, lvl, iv):
        return self.mg.get_level(lvl, iv) if len(self.my_ids(lvl)) else None

    def restrict(self, iv):
        omg.mg_restrict(self.mg, iv)

    def fill_ghost_cells(self, iv):
        omg.mg_fill_ghost_cells(self.mg, iv)

    def apply_op(self, iv):
        omg.mg_apply_op(self.mg, iv)

    def vcycle(self, want):
        return omg.mg_fas_vcycle(self.mg, max_res=bool(want)) or 0.0

    def fmg(self, have_guess, want):
        return omg.mg_fas_fmg(self.mg, have_guess, max_res=bool(want)) or 0.0

    def diffusion(self, order, dt):
        op = self.cfg["op"]
        if op == "helm":
            return omg.diffusion_solve(self.mg, dt, diffusion_coeff(self.cfg), order, DIFF_TOL)
        if op == "vhelm":
            return omg.diffusion_solve_vcoeff(self.mg, dt, order, DIFF_TOL)
        return omg.diffusion_solve_acoeff(self.mg, dt, order, DIFF_TOL)


# per face x-, x+, y-, y+, z-, z+: (type, constant value)
MIXED_BC = {
    "mx1": [(T.MG_BC_DIRICHLET, 0.5), (T.MG_BC_DIRICHLET, -1.25), (T.MG_BC_NEUMANN, 0.75),
            (T.MG_BC_NEUMANN, -0.3), (T.MG_BC_CONTINUOUS, 0.2), (T.MG_BC_CONTINUOUS, 0.0)],
    "mx2": [(T.MG_BC_CONTINUOUS, 0.0), (T.MG_BC_NEUMANN, 1.5), (T.MG_BC_DIRICHLET, -0.625),
            (T.MG_BC_CONTINUOUS, 0.0), (T.MG_BC_NEUMANN, -2.0), (T.MG_BC_DIRICHLET, 0.125)],
}


def _apply_bc(cfg, tree, set_bc, set_faces):
    bc = cfg["bc"]
    if bc == "sol":
        off, typ, data = P.callback_bc_faces(tree)
        set_faces(T.MG_IPHI, off, typ, data)
    elif bc in ("d0", "n0", "c0"):
        t = {"d0": T.MG_BC_DIRICHLET, "n0": T.MG_BC_NEUMANN, "c0": T.MG_BC_CONTINUOUS}[bc]
        for nb in range(1, 7):
            set_bc(T.MG_IPHI, nb, t, 0.0)
    elif bc in MIXED_BC:
        # (not omg_golden's: per-face types and nonzero constant values, for
        # the block passes' physical faces)
        for nb, (t, v) in enumerate(MIXED_BC[bc], start=1):
            set_bc(T.MG_IPHI, nb, t, v)


def setup_problem(be):
    """set_solution + compute_rhs_and_reset (tests/test_uniform_grid.f90:
    137-170), or set_rhs (tests/test_performance.f90:102-115)."""
    cfg, tree = be.cfg, be.tree
    I_SOL = i_sol(cfg)

    def empty(lvl):
        nc = tree.box_size_lvl[lvl]
        return np.zeros((0, nc + 2, nc + 2, nc + 2))

    def put(lvl, iv, make):
        # a rank without boxes still calls when the upload is collective
        ids = be.my_ids(lvl)
        if len(ids):
            be.set_level(lvl, iv, make(ids))
        elif be.collective(lvl, iv):
            be.set_level(lvl, iv, empty(lvl))

    if is_vop(cfg) or cfg["op"] == "ahelm":
        for lvl in be.levels():
            e = P.level_eps(tree, lvl, be.my_ids(lvl)) if len(be.my_ids(lvl)) else empty(lvl)
            if cfg["op"] == "ahelm":
                for d in (1, 2, 3):                 # eps_d = eps * d, vars 5..7
                    put(lvl, I_EPS + d - 1, lambda ids: e * float(d))
            else:
                put(lvl, I_EPS, lambda ids: e)
    if cfg["rhs"] == "phi":
        # copy_solution_to_phi: phi = u incl. ghosts, rhs stays 0
        for lvl in be.levels():
            put(lvl, I_SOL, lambda ids: P.level_solution(tree, lvl, ids))
        if cfg["n_levels"] > 1:
            be.restrict(I_SOL)
            be.fill_ghost_cells(I_SOL)
        for lvl in be.levels():
            put(lvl, T.MG_IPHI, lambda ids: be.get_level(lvl, I_SOL))
    elif cfg["rhs"] == "sol":
        for lvl in be.levels():
            put(lvl, I_SOL, lambda ids: P.level_solution(tree, lvl, ids))
        if cfg["n_levels"] > 1:
            be.restrict(I_SOL)
            be.fill_ghost_cells(I_SOL)
        for lvl in be.levels():
            put(lvl, T.MG_IPHI, lambda ids: be.get_level(lvl, I_SOL))
        be.apply_op(T.MG_IRHS)
        for lvl in be.levels():
            nc = tree.box_size_lvl[lvl]
            put(lvl, T.MG_IPHI, lambda ids: np.zeros((len(ids), nc + 2, nc + 2, nc + 2)))
    else:
        def ones(ids):
            a = np.zeros((len(ids), nc + 2, nc + 2, nc + 2))
            a[:, 1:nc + 1, 1:nc + 1, 1:nc + 1] = 1.0
            return a
        for lvl in be.levels():
            nc = tree.box_size_lvl[lvl]
            put(lvl, T.MG_IRHS, ones)


def measure(be):
    """print_state of omg_golden: max |phi-u| and max |res| over the leaves of
    levels >= 1 (this rank's boxes)."""
    tree = be.tree
    err = res = 0.0
    for lvl in range(1, tree.highest_lvl + 1):
        ids = list(be.my_ids(lvl))
        if not ids:
            continue
        nc = tree.box_size_lvl[lvl]
        leaves = set(int(x) for x in tree.lvls[lvl].leaves)
        sel = [n for n, i in enumerate(ids) if int(i) in leaves]
        if not sel:
            continue
        phi = be.get_level(lvl, T.MG_IPHI)[sel, 1:nc + 1, 1:nc + 1, 1:nc + 1]
        sol = be.get_level(lvl, i_sol(be.cfg))[sel, 1:nc + 1, 1:nc + 1, 1:nc + 1]
        r = be.get_level(lvl, T.MG_IRES)[sel, 1:nc + 1, 1:nc + 1, 1:nc + 1]
        err = max(err, float(np.max(np.abs(phi - sol))))
        res = max(res, float(np.max(np.abs(r))))
    return err, res


def phi_digest(be, iv=None):
    iv = T.MG_IPHI if iv is None else iv
    h = hashlib.sha256()
    for lvl in be.levels():
        ids = be.my_ids(lvl)
        if not len(ids):
            continue
        nc = be.tree.box_size_lvl[lvl]
        phi = be.get_level(lvl, iv)[:, 1:nc + 1, 1:nc + 1, 1:nc + 1]
        h.update(np.ascontiguousarray(phi).tobytes())
    return h.hexdigest()


class StepError(RuntimeError):
    """A step that failed the way the reference's error stop does; .history
    holds what was printed before it."""

    def __init__(self, msg, history):
        super().__init__(msg)
        self.history = history


def _cycles(be, cfg, reduce=None):
    """The iterations of omg_golden; with "mv" the second tree's set-up and
    iterations follow (its IT 0.. block appended)."""
    hist = _tree_cycles(be, cfg, reduce)
    if regrids(cfg):
        be.regrid(REGRID_SHIFT)
        setup_problem(be)
        hist += _tree_cycles(be, cfg, reduce)
    return hist


def _tree_cycles(be, cfg, reduce=None):
    hist = []

    def record(it, mres):
        e, r = measure(be)
        if reduce is not None:
            e, r = reduce(e, r)
        hist.append({"it": it, "err": hexbits(e), "res": hexbits(r), "max_res": hexbits(mres)})

    record(0, 0.0)
    for n in range(1, cfg["n_its"] + 1):
        if cfg["cycle"] in ("d1", "d2"):
            # one m_diffusion time step; omg_golden prints max_res = 0
            try:
                be.diffusion(int(cfg["cycle"][1]), cfg["lam"])
            except RuntimeError as ex:
                raise StepError(str(ex), hist) from ex
            record(n, 0.0)
            continue
        if cfg["cycle"] == "f":
            m = be.fmg(n > 1, cfg["maxres"])
        else:
            m = be.vcycle(cfg["maxres"])
        record(n, m if cfg["maxres"] else 0.0)
    return hist


def run_problem(args: str, backend="device", n_ranks=1, n_its=None, reduce=None):
    """Run one omg_golden configuration; returns {'history': [...], 'phi_sha256'}.

    reduce(err, res) -> (err, res) combines per-rank maxima for multi-rank runs."""
    cfg = parse(args)
    if n_its is not None:
        cfg["n_its"] = n_its
    be = OracleBackend(cfg, n_ranks) if backend == "oracle" else DeviceBackend(cfg)
    setup_problem(be)
    try:
        hist = _cycles(be, cfg, reduce)
    except StepError as ex:   # the reference's error stop: what it printed + the message
        return {"history": ex.history, "error": str(ex), "backend": be}
    out = {"history": hist, "phi_sha256": phi_digest(be), "backend": be}
    if cfg["op"] == "ahelm":
        out["rhs_sha256"] = phi_digest(be, T.MG_IRHS)
    return out


def _owned_phi(be):
    """{(lvl, id): interior phi bytes} of the boxes this rank owns (a
    replicated coarse level: every box, each rank holds them all)."""
    out = {}
    for lvl in be.levels():
        ids = be.my_ids(lvl)
        n, nc = be.mg.ctx.level_size(lvl)
        if lvl <= be.rep_lvl and n == len(be.tree.lvls[lvl].ids):
            ids = be.tree.lvls[lvl].ids
        if not n:
            continue
        phi = be.mg.get_level(lvl, T.MG_IPHI)[:, 1:nc + 1, 1:nc + 1, 1:nc + 1]
        for q, id_ in enumerate(ids):
            out[(lvl, int(id_))] = np.ascontiguousarray(phi[q]).tobytes()
    return out


def run_loopback(args: str, n_ranks: int, body, n_its=None, timeout=600, rep_cells=0):
    """Run body(be, rank, reduce) on n_ranks device contexts of this process
    (one thread per rank, all on GPU 0) exchanging through the loopback
    transport (omg_loopback_unique_id), each with the configuration's tree and
    problem set up; reduce(e, r) is omg_golden's MPI_Reduce(MAX) of a pair.
    Returns the per-rank results; the first rank error is raised."""
    import threading
    cfg = parse(args)
    if n_its is not None:
        cfg["n_its"] = n_its
    tag = int.from_bytes(os.urandom(6), "little")
    bar = threading.Barrier(n_ranks)
    slots = [None] * n_ranks
    out = [None] * n_ranks
    errors = []

    def worker(rank):
        def reduce(e, r):
            slots[rank] = (e, r)
            bar.wait()
            E = max(x[0] for x in slots)
            R = max(x[1] for x in slots)
            bar.wait()
            return E, R
        try:
            be = DeviceBackend(cfg, omg.Loopback(tag, rank, n_ranks), rep_cells)
            setup_problem(be)
            out[rank] = body(be, rank, reduce)
            be.mg.ctx.call("synchronize")
            omg.mg_deallocate_storage(be.mg)
        except BaseException as ex:  # noqa: BLE001  (re-raised in the caller)
            errors.append((rank, ex))
            bar.abort()

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n_ranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    if errors:
        msg = "; ".join(f"rank {r}: {type(e).__name__}: {e}" for r, e in sorted(errors, key=lambda x: x[0])
                        if not isinstance(e, threading.BrokenBarrierError))
        raise RuntimeError(msg or str(errors[0][1]))
    if any(t.is_alive() for t in th):
        raise TimeoutError("loopback run did not finish")
    return out


def run_problem_loopback(args: str, n_ranks: int, n_its=None, timeout=600, rep_cells=0, stats=(), cycles=None):
    """The same configuration on n_ranks device contexts of this process,
    exchanging through the loopback transport (run_loopback): the multi-rank
    path of libomg.so (plans, packing, MPICH-order reductions) on a single
    GPU.  Returns the history with err / res reduced by max over ranks, as
    omg_golden's MPI_Reduce(MAX), and the sha256 of the final phi of every box
    gathered from its owner, in the order phi_digest uses for a one-rank run
    (ids per level, lowest first).  stats: kernel-family names (omg_kernel_stats)
    whose launch counts every rank returns under "stats" (the cycles then run
    with profiling on); cycles = (n_cycle_down, n_cycle_up) other than the
    reference's 2, 2."""
    cfg = parse(args)
    if n_its is not None:
        cfg["n_its"] = n_its

    def body(be, rank, reduce):
        if cycles:
            be.mg.n_cycle_down, be.mg.n_cycle_up = cycles
            be.mg._push_methods()
        if stats:
            be.mg.ctx.call("set_profiling", 1)
        hist = _cycles(be, cfg, reduce)
        be.mg.ctx.call("synchronize")
        st = {name: be.mg.ctx.kernel_stats(name)[0] for name in stats}
        t = be.tree   # (copied: run_loopback frees the storage, which empties the level lists)
        order = [(lvl, [int(i) for i in t.lvls[lvl].ids]) for lvl in range(t.lowest_lvl, t.highest_lvl + 1)]
        return hist, _owned_phi(be), (order, t.rank.copy()), st

    res = run_loopback(args, n_ranks, body, n_its, timeout, rep_cells)
    out = [r[0] for r in res]
    phis = [r[1] for r in res]
    order, owners = res[0][2]
    assert all(h == out[0] for h in out)
    h = hashlib.sha256()
    for lvl, ids in order:
        for id_ in ids:
            key = (lvl, id_)
            owner = int(owners[id_])
            h.update(phis[owner][key] if key in phis[owner] else phis[0][key])
    return {"history": out[0], "phi_sha256": h.hexdigest(), "stats": [r[3] for r in res]}
