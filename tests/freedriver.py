"""Problem runner of the free-space tests: replays oracle/omg_free_golden.f90
(the reference's tests/test_free_space.f90 set-up) on

* ``device`` — the product: octree_mg_amd.MG + free_space.mg_poisson_free_3d
  driving libomg.so (Green's function, hipFFT solve, boundary table, FMG) on
  the GPU, one rank or several through the loopback transport;
* ``oracle`` — the checker: the C restatement of the multigrid
  (oracle/liboracle.so) with oracle/free_space_oracle.py's direct-convolution
  restatement of PSolver.

Both start from the same inputs.  The Green's-function solve sums in another
order on each (and in the reference), so results agree at round-off, which
the tests state as tolerances (see tolerances()).
"""
from __future__ import annotations

import math
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__  # noqa: E402

omg = __graft_entry__.load_package()
T = omg.tree

GAUSS_AMPL, GAUSS_SIGMA = 1.0, 0.1        # tests/test_free_space.f90:9-13
GAUSS_R0 = np.array([0.5, 0.5, 0.5])
I_SOL = 5


def parse(args: str) -> dict:
    f = args.split()
    return dict(box=int(f[0]), domain=[int(f[1]), int(f[2]), int(f[3])], n_its=int(f[4]),
                frac=float(f[5]), cycle=f[6])


def build_tree(cfg, tree, n_ranks=1, my_rank=0):
    tree.smoother_type = T.MG_SMOOTHER_GSRB
    tree.n_cpu, tree.my_rank = n_ranks, my_rank
    dom = np.array(cfg["domain"], dtype=np.int64)
    tree.build_rectangle(dom, cfg["box"], 1.0 / dom.astype(np.float64), [0.0, 0.0, 0.0], [False] * 3, 0)
    tree.load_balance()
    return tree


def _erf(x):
    return np.vectorize(math.erf, otypes=[np.float64])(x)


def level_fields(tree, lvl, ids):
    """rhs and solution of test_free_space (:127-165) on boxes ids, as
    [box, k, j, i] arrays of (nc+2)^3 with zero ghosts."""
    nc = tree.box_size_lvl[lvl]
    dr = np.asarray(tree.dr[lvl])
    rhs = np.zeros((len(ids), nc + 2, nc + 2, nc + 2))
    sol = np.zeros_like(rhs)
    c = np.arange(1, nc + 1) - 0.5
    pi = math.acos(-1.0)
    for n, id_ in enumerate(ids):
        r0 = tree.box_r_min[id_]
        x = r0[0] + c * dr[0]
        y = r0[1] + c * dr[1]
        z = r0[2] + c * dr[2]
        Z, Y, X = np.meshgrid(z, y, x, indexing="ij")
        s2 = ((X - GAUSS_R0[0]) / GAUSS_SIGMA) ** 2 + ((Y - GAUSS_R0[1]) / GAUSS_SIGMA) ** 2 + \
            ((Z - GAUSS_R0[2]) / GAUSS_SIGMA) ** 2
        rhs[n, 1:-1, 1:-1, 1:-1] = -GAUSS_AMPL / (GAUSS_SIGMA ** 3 * pi * math.sqrt(pi)) * np.exp(-s2)
        rn = np.sqrt((X - GAUSS_R0[0]) ** 2 + (Y - GAUSS_R0[1]) ** 2 + (Z - GAUSS_R0[2]) ** 2)
        fac = 1.0 / (4.0 * pi)
        with np.errstate(divide="ignore", invalid="ignore"):
            v = fac * GAUSS_AMPL * _erf(rn / GAUSS_SIGMA) / rn
        v = np.where(rn < math.sqrt(np.finfo(np.float64).eps),
                     2.0 * fac * GAUSS_AMPL / (math.sqrt(pi) * GAUSS_SIGMA), v)
        sol[n, 1:-1, 1:-1, 1:-1] = v
    return rhs, sol


def _errors(tree, phi, sol):
    """print_error (:167-195): max |phi - sol| and the squared-error sum over
    the highest level (this rank's boxes)."""
    d = np.abs(phi[:, 1:-1, 1:-1, 1:-1] - sol[:, 1:-1, 1:-1, 1:-1])
    return float(d.max()) if d.size else 0.0, float(np.sum(d ** 2))


def _history_entry(it, e, e2sum, n_unknowns, mres):
    return {"it": it, "err": e, "err2": math.sqrt(e2sum / n_unknowns), "max_res": mres}


def run_oracle(args: str):
    """The configuration on the CPU oracle; returns history and the final
    phi of the highest level [box, k, j, i] (ids order)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import free_space_oracle as F   # checker only
    import pyoracle
    cfg = parse(args)
    tree = build_tree(cfg, T.MGTree())
    o = pyoracle.Oracle(tree, I_SOL)
    o.configure(op=pyoracle.LAPLACIAN, smoother=pyoracle.GSRB)
    for lvl in range(tree.lowest_lvl, tree.highest_lvl + 1):
        rhs, sol = level_fields(tree, lvl, tree.lvls[lvl].ids)
        o.set_level(lvl, T.MG_IRHS, rhs)
        o.set_level(lvl, I_SOL, sol)
    S = F.FreeState()
    hl = tree.highest_lvl
    sol_h = o.get_level(hl, I_SOL)
    hist = []
    for n in range(1, cfg["n_its"] + 1):
        m = F.poisson_free_3d(o, tree, S, n == 1, cfg["frac"], cfg["cycle"] == "f", True)
        e, e2 = _errors(tree, o.get_level(hl, T.MG_IPHI), sol_h)
        hist.append(_history_entry(n, e, e2, tree.number_of_unknowns(), m))
    return {"history": hist, "phi": o.get_level(hl, T.MG_IPHI), "tree": tree}


class _Device:
    def __init__(self, cfg, comm=None, rep_cells=0):
        mg = omg.MG()
        mg.coarse_replication_cells = rep_cells
        mg.n_extra_vars = 1
        mg.operator_type = T.MG_LAPLACIAN
        mg.smoother_type = T.MG_SMOOTHER_GSRB
        omg.mg_set_methods(mg)
        omg.mg_comm_init(mg, comm)
        build_tree(cfg, mg, mg.n_cpu, mg.my_rank)
        omg.mg_allocate_storage(mg)
        self.mg = mg
        rep = mg.ctx.replicated_level()
        for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
            ids = mg.lvls[lvl].my_ids
            if len(ids) or lvl <= rep:
                rhs, sol = level_fields(mg, lvl, ids)
                mg.set_level(lvl, T.MG_IRHS, rhs)
                mg.set_level(lvl, I_SOL, sol)
        hl = mg.highest_lvl
        self.sol_h = mg.get_level(hl, I_SOL) if len(mg.lvls[hl].my_ids) else None

    def step(self, cfg, n):
        return omg.mg_poisson_free_3d(self.mg, n == 1, cfg["frac"], cfg["cycle"] == "f", max_res=True)

    def errors(self):
        hl = self.mg.highest_lvl
        if self.sol_h is None:
            return 0.0, 0.0
        return _errors(self.mg, self.mg.get_level(hl, T.MG_IPHI), self.sol_h)


def run_device(args: str):
    """The configuration on one GPU rank."""
    cfg = parse(args)
    d = _Device(cfg)
    hist = []
    for n in range(1, cfg["n_its"] + 1):
        m = d.step(cfg, n)
        e, e2 = d.errors()
        hist.append(_history_entry(n, e, e2, d.mg.number_of_unknowns(), m))
    out = {"history": hist, "phi": d.mg.get_level(d.mg.highest_lvl, T.MG_IPHI), "mg": d.mg}
    return out


def run_device_loopback(args: str, n_ranks: int, timeout=600, rep_cells=0):
    """n_ranks device contexts of this process (one thread each, loopback
    transport, all on GPU 0); err by max and the squared errors summed over
    ranks, as print_error's MPI_Allreduce."""
    cfg = parse(args)
    tag = int.from_bytes(os.urandom(6), "little")
    bar = threading.Barrier(n_ranks)
    slots = [None] * n_ranks
    hists = [None] * n_ranks
    errors = []

    def worker(rank):
        try:
            d = _Device(cfg, omg.Loopback(tag, rank, n_ranks), rep_cells)
            hist = []
            for n in range(1, cfg["n_its"] + 1):
                m = d.step(cfg, n)
                slots[rank] = d.errors()
                bar.wait()
                e = max(s[0] for s in slots)
                e2 = sum(s[1] for s in slots)
                bar.wait()
                hist.append(_history_entry(n, e, e2, d.mg.number_of_unknowns(), m))
            hists[rank] = hist
            d.mg.ctx.call("synchronize")
            omg.mg_deallocate_storage(d.mg)
        except BaseException as ex:  # noqa: BLE001  (re-raised below)
            errors.append((rank, ex))
            bar.abort()

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n_ranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    if errors:
        real = [(r, e) for r, e in errors if not isinstance(e, threading.BrokenBarrierError)]
        r, e = (real or errors)[0]
        raise RuntimeError(f"rank {r}: {type(e).__name__}: {e}")
    if any(t.is_alive() for t in th):
        raise TimeoutError("loopback run did not finish")
    return {"history": hists[0], "all": hists}


def golden_history(entry, ranks=1):
    """The reference's history of a free_golden.json entry as floats."""
    import struct
    f = lambda h: struct.unpack(">d", bytes.fromhex(h))[0]
    return [{"it": h["it"], "err": f(h["err"]), "err2": f(h["err2"]), "max_res": f(h["max_res"])}
            for h in entry["runs"][str(ranks)]["history"]]


def tolerances(cfg):
    """Agreement stated for free-space results.  The Green's-function solve
    is exact up to summation order, so phi agrees to a few ulps of its scale
    (max |phi| < 1); errors against the analytic solution (~1e-3) inherit
    that absolutely; residuals are second differences of phi, so a phi
    difference of delta moves them by up to delta * 2*sum(1/dr^2)."""
    dr = 1.0 / np.asarray(cfg["domain"], dtype=np.float64)
    op_norm = 2.0 * float(np.sum(1.0 / dr ** 2))
    phi_abs = 2e-14
    return {"phi_abs": phi_abs, "err_abs": phi_abs, "res_abs": 4 * phi_abs * op_norm}


def compare_history(got, ref, cfg, what=""):
    tol = tolerances(cfg)
    assert len(got) == len(ref), (what, len(got), len(ref))
    for g, r in zip(got, ref):
        assert abs(g["err"] - r["err"]) <= tol["err_abs"], (what, g, r)
        assert abs(g["err2"] - r["err2"]) <= tol["err_abs"], (what, g, r)
        assert abs(g["max_res"] - r["max_res"]) <= tol["res_abs"], (what, g, r)
