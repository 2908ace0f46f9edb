"""Parity of the HIP path (libomg.so on the GPU, through the C-ABI) with the
reference: bit-for-bit against the golden vectors the reference itself
produced (tests/golden/golden.json), and against the C oracle per operation
on random inputs."""
import json
import os

import numpy as np
import pytest

from tests.mgdriver import (DeviceBackend, OracleBackend, T, parse, run_problem,
                            setup_problem)

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["configs"]
ONE_RANK = [n for n, e in GOLDEN.items() if "1" in e["runs"]]

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ONE_RANK)
def test_device_matches_reference_golden(name):
    e = GOLDEN[name]
    run = e["runs"]["1"]
    out = run_problem(e["args"], backend="device")
    assert out["history"] == run["history"]
    assert out.get("error") == run.get("error")
    if "phi_sha256" in run:
        assert out["phi_sha256"] == run["phi_sha256"]
    if "rhs_sha256" in run:   # aniso operator pinned through rhs = L(u)
        assert out["rhs_sha256"] == run["rhs_sha256"]


def _random_fill(be, rng, ivs=(1, 2, 5)):
    for lvl in be.levels():
        ids = be.my_ids(lvl)
        if not len(ids):
            continue
        nc = be.tree.box_size_lvl[lvl]
        for iv in ivs:
            be.set_level(lvl, iv, rng.standard_normal((len(ids), nc + 2, nc + 2, nc + 2)))


def _stored_mask(nc):
    """Interior + face ghosts of a (nc+2)^3 box: the cells any operator of the
    reference reads.  Edge/corner ghosts are dead data (never read, never
    written by a fill) and the device layout does not store them."""
    s = nc + 2
    ix = np.arange(s)
    bnd = ((ix == 0) | (ix == s - 1)).astype(int)
    nb = bnd[:, None, None] + bnd[None, :, None] + bnd[None, None, :]
    return nb < 2


def _assert_same(dev, orc, ivs=(1, 2, 3, 4, 5)):
    for lvl in dev.levels():
        if not len(dev.my_ids(lvl)):
            continue
        m = _stored_mask(dev.tree.box_size_lvl[lvl])
        for iv in ivs:
            a, b = dev.get_level(lvl, iv), orc.get_level(lvl, iv)
            assert np.array_equal(a[:, m].view(np.uint64), b[:, m].view(np.uint64)), (lvl, iv)


OPS_CASES = [
    "8 32 32 32 1 v gsrb lpl 0 sol sol 1 lb 0",
    "8 32 32 32 1 v gs helm 3.5 n0 sol 1 lb 0",
    "8 32 32 32 1 v gsrb lpl 0 per sol 1 lb 0",
    "8 32 32 32 1 v gs lpl 0 c0 sol 3 lb 0",
    "4 24 16 8 1 v gsrb lpl 0 d0 sol 1 lb 0",
    # per-face types with nonzero constant values (tests/mgdriver.py MIXED_BC)
    "16 96 128 64 1 v gsrb lpl 0 mx1 sol 1 lb 0",
    "8 32 32 32 1 v gs helm 3.5 mx2 sol 1 lb 0",
    "16 64 64 64 1 v gsrb helm 2 mx2 sol 1 lb 0",
]


@pytest.mark.parametrize("args", OPS_CASES)
def test_per_operation_bitwise(args):
    cfg = parse(args)
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    for be in (dev, orc):
        _random_fill(be, np.random.default_rng(7))
    _assert_same(dev, orc)
    lo, hi = dev.tree.lowest_lvl, dev.tree.highest_lvl
    # ghost cells on every level (physical, periodic, refinement boundaries)
    dev.fill_ghost_cells(1); orc.fill_ghost_cells(1)
    _assert_same(dev, orc)
    import octree_mg_amd as omg
    c = dev.mg.ctx
    for lvl in range(hi, lo, -1):
        c.call("smooth_boxes", lvl, 1); orc.o.smooth_boxes(lvl, 1)
        _assert_same(dev, orc)
        c.call("update_coarse", lvl); orc.o.update_coarse(lvl)
        _assert_same(dev, orc)
    for lvl in range(lo, hi):
        c.call("correct_children", lvl); orc.o.correct_children(lvl)
        _assert_same(dev, orc)
    dev.apply_op(4); orc.apply_op(4)
    _assert_same(dev, orc)
    for lvl in range(lo, hi + 1):
        assert c.scalar("max_residual_lvl", lvl) == orc.o.max_residual_lvl(lvl)
    assert c.scalar("get_sum", 1) == orc.o.get_sum(1)
    c.call("subtract_mean", 1, 1); orc.o.subtract_mean(1, 1)
    _assert_same(dev, orc)
    c.call("set_rhs", 0.3, -1.7); orc.o.set_rhs(0.3, -1.7)   # m_diffusion's set_rhs
    _assert_same(dev, orc)


@pytest.mark.parametrize("args", [OPS_CASES[0], OPS_CASES[1], "16 64 64 64 1 v gsrb helm 2 d0 sol 1 lb 0",
                                  # the register ring with two ghost sets (the first sweep reads the stale set)
                                  "16 256 256 256 1 v gs lpl 0 d0 sol 1 lb 0"])
def test_smoother_with_stale_ghosts(args):
    """smooth_boxes right after phi was overwritten (ghosts not refilled): the
    reference reads the stale ghosts in the first substep; so must we."""
    cfg = parse(args)
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    for be in (dev, orc):
        _random_fill(be, np.random.default_rng(11))
    hi = dev.tree.highest_lvl
    for n_cycle in (1, 2, 3):
        dev.mg.ctx.call("smooth_boxes", hi, n_cycle)
        orc.o.smooth_boxes(hi, n_cycle)
        _assert_same(dev, orc)


@pytest.mark.parametrize("args", ["8 32 32 32 3 v gsrb ahelm 10 sol sol 1 lb 0",
                                  "8 32 32 32 2 v gs ahelm 5 d0 sol 2 lb 0",
                                  # box 16 (the tiled aniso kernels C5-aniso runs)
                                  "16 128 128 128 2 v gsrb ahelm 10 sol sol 1 lb 0"])
def test_ahelm_smoother_matches_oracle(args):
    """The aniso-Helmholtz V-cycle: the reference's 3D box_gs_ahelmh is broken
    (a0(4:5), m_ahelmholtz.f90:145 -> NaN), so the device is held bit for bit
    to the oracle's restatement with a0(5:6); parity unpinned against the
    reference (its operator box_ahelmh is pinned: ahelm*_op goldens)."""
    dev = run_problem(args, backend="device")
    orc = run_problem(args, backend="oracle")
    assert dev["history"] == orc["history"]
    assert dev["phi_sha256"] == orc["phi_sha256"]


@pytest.mark.parametrize("args", ["8 32 32 32 2 d1 gsrb ahelm 0.01 n0 phi 1 lb 0",
                                  "8 32 32 32 2 d2 gs ahelm 0.001 d0 phi 2 lb 0"])
def test_ahelm_diffusion_matches_oracle(args):
    """diffusion_solve_acoeff (m_diffusion.f90:108-142): like the aniso
    V-cycle, held to the oracle's restatement (reference NaN, unpinned)."""
    dev = run_problem(args, backend="device")
    orc = run_problem(args, backend="oracle")
    assert dev.get("error") == orc.get("error")
    assert dev["history"] == orc["history"]
    if "phi_sha256" in orc:
        assert dev["phi_sha256"] == orc["phi_sha256"]


def test_diffusion_bad_order_fails_like_reference():
    """order 3: the reference's error stop (m_diffusion.f90:42-43) as an error,
    with phi untouched."""
    from tests.mgdriver import omg, phi_digest
    cfg = parse("8 16 16 16 1 d1 gsrb helm 0.01 n0 phi 1 lb 0")
    be = DeviceBackend(cfg)
    setup_problem(be)
    before = phi_digest(be)
    with pytest.raises(omg.device.OmgError, match="order should be 1 or 2"):
        be.mg.ctx.call("diffusion_solve", 3, 0.01, 1.0, 3, 1e-8, None, None)
    assert phi_digest(be) == before


@pytest.mark.parametrize("args", ["16 64 64 64 2 v gsrb lpl 0 per sol 1 lb 0",
                                  "16 64 64 64 2 f gsrb lpl 0 per sol 1 lb 0",
                                  "16 64 64 64 2 v gsrb helm 2 per sol 1 lb 0",
                                  "8 64 64 64 2 v gsrb helm 2 per sol 1 lb 0"])
def test_fused_down_substep_matches_oracle(args):
    """Levels whose faces are all same-GPU boxes end their down-smoothing in
    k_smooth_resid (last substep + residual + restriction, the neighbours'
    new boundary cells recomputed): box sizes 16 and 8, Laplacian (with the
    periodic subtract_mean) and Helmholtz, V-cycles and FMG, bit for bit
    against the oracle."""
    dev = run_problem(args, backend="device")
    orc = run_problem(args, backend="oracle")
    assert dev["history"] == orc["history"]
    assert dev["phi_sha256"] == orc["phi_sha256"]


@pytest.mark.parametrize("down,up", [(1, 1), (3, 2)])
def test_fused_down_substep_other_cycle_counts(down, up):
    """k_smooth_resid with n_cycle_down 1 (the pending mean shift is absorbed
    by the only unfused substep) and 3: V-cycles bit for bit against the
    oracle, every stored variable."""
    from tests.mgdriver import setup_problem
    cfg = parse("16 64 64 64 3 v gsrb lpl 0 per sol 1 lb 0")
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    import pyoracle  # on sys.path once OracleBackend exists (checker only)
    dev.mg.n_cycle_down, dev.mg.n_cycle_up = down, up
    dev.mg._push_methods()
    orc.o.configure(op=pyoracle.LAPLACIAN, lam=0.0, smoother=pyoracle.GSRB, n_cycle_down=down,
                    n_cycle_up=up, subtract_mean=True)
    for be in (dev, orc):
        setup_problem(be)
    for _ in range(3):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc, ivs=(1, 2, 3, 4))


# the cycles captured as HIP graphs (OMG_GRAPH=1, read at context creation):
# the same bits as the direct launches, on non-periodic one-GPU goldens (the
# cases the graph path takes) with V-cycles, FMG and max-residual readbacks
GRAPH_CASES = [n for n in ONE_RANK if " per " not in GOLDEN[n]["args"]][:6]


@pytest.mark.parametrize("name", GRAPH_CASES)
def test_graph_cycles_match_golden(name, monkeypatch):
    monkeypatch.setenv("OMG_GRAPH", "1")
    e = GOLDEN[name]
    run = e["runs"]["1"]
    out = run_problem(e["args"], backend="device")
    assert out["history"] == run["history"]
    if "phi_sha256" in run:
        assert out["phi_sha256"] == run["phi_sha256"]


@pytest.mark.parametrize("args", ["8 32 32 32 1 f gsrb lpl 0 sol sol 1 lb 0",
                                  "16 64 64 64 1 f gsrb lpl 0 sol sol 1 lb 0",
                                  "8 32 32 32 1 f gs helm 3.5 n0 sol 1 lb 0",
                                  "8 32 32 32 1 f gsrb lpl 0 per sol 1 lb 0"])
@pytest.mark.parametrize("have_guess", [False, True])
def test_fmg_full_state_matches_oracle(args, have_guess):
    """Every stored cell of phi, rhs, old and res after FMG calls: FMG's
    old = phi (m_multigrid.f90:127-129) is partly fused into the correction
    kernel and partly skipped where update_coarse left old = phi already."""
    cfg = parse(args)
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    for be in (dev, orc):
        setup_problem(be)
    for _ in range(2):
        assert dev.fmg(have_guess, True) == orc.fmg(have_guess, True)
        _assert_same(dev, orc, ivs=(1, 2, 3, 4))


def test_refinement_bnd_callback_restating_sides_rb():
    """omg_set_refinement_bnd through the Python mirror: a host callback that
    restates sides_rb (0.5 gc + 0.75 x1 - 0.25 x2, m_ghost_cells.f90:769-861)
    must give the reference's own history and phi of the bench's refined
    GSRB tree bit for bit (coarse faces, box copies, the ghosts coming back,
    once per fill); the custom_rb goldens pin other coefficients."""
    import functools

    from tests.mgdriver import T, _cycles, custom_rb, phi_digest
    e = GOLDEN["c4_ref2_box16_gsrb"]
    cfg = parse(e["args"])
    be = DeviceBackend(cfg)
    calls = []

    def sides_rb(mg, id_, nc, iv, nb, cgc, cc):
        calls.append(nb)
        custom_rb(mg, id_, nc, iv, nb, cgc, cc, k=(0.5, 0.75, -0.25))

    for nb in range(1, 7):
        be.mg.bc[nb][T.MG_IPHI].refinement_bnd = sides_rb
    be.mg.push_bc([T.MG_IPHI])
    setup_problem(be)
    assert _cycles(be, cfg) == e["runs"]["1"]["history"]
    assert phi_digest(be) == e["runs"]["1"]["phi_sha256"]
    assert calls and set(calls) == set(range(1, 7))


# Every runtime switch of the library (omg_ctx_create reads them; DESIGN.md
# §12 lists them) selects another, unfused or older, path through the same
# arithmetic: each must reproduce the reference's goldens bit for bit.  The
# configurations cover what the switches change: a refined GSRB tree at box
# 16 (fused down-step with refinement-boundary faces, stored coarse parts,
# fused correction + fill on the refined level), physical faces at box 16,
# a periodic tree (pending mean shift, skip-1 correction) and GS with FMG.
SWITCHES = ["OMG_NO_TAIL", "OMG_NO_FUSE_UP", "OMG_NO_SKIP1", "OMG_NO_FILL_TILE", "OMG_NO_FILL_CRHS",
            "OMG_NO_TAIL_CRHS", "OMG_NO_RBGV", "OMG_NO_FUSE_DOWN", "OMG_NO_RB_FUSE", "OMG_NO_FUSE_DOWN_BC",
            "OMG_NO_REV"]
SWITCH_GOLDENS = ["c4_ref2_box16_gsrb", "u64_box16_gsrb_d0_one", "per32_gsrb_v", "ref3_gs_f"]


@pytest.mark.parametrize("name", SWITCH_GOLDENS)
@pytest.mark.parametrize("switch", SWITCHES)
def test_runtime_switches_match_golden(switch, name, monkeypatch):
    monkeypatch.setenv(switch, "1")
    e = GOLDEN[name]
    run = e["runs"]["1"]
    out = run_problem(e["args"], backend="device")
    assert out["history"] == run["history"]
    assert out["phi_sha256"] == run["phi_sha256"]


# the coarse tail forming its top level's fill and coarse rhs itself (the
# default) against update_coarse doing it in its own launch
# (OMG_NO_TAIL_CRHS=1): every stored cell of phi, rhs, old and res after each
# cycle equals the oracle's either way; the 16^3 top over the 8/4/2 chain
# (tabulated faces, lexicographic GS with Helmholtz), an LDS-resident top
# (box 8, periodic) and FMG
TAIL_CRHS_CASES = ["16 128 128 128 2 v gsrb lpl 0 sol sol 2 lb 0",
                   "16 64 64 64 2 v gs helm 2 d0 sol 1 lb 0",
                   "8 64 64 64 2 v gsrb lpl 0 per sol 1 lb 0",
                   "8 32 32 32 2 f gs lpl 0 n0 sol 1 lb 1"]


def _coarse_fill_launches(dev):
    n = 0
    for lvl in dev.levels():
        for fam in ("fill_crhs", "fill_gc", "coarse_rhs"):
            n += dev.mg.ctx.kernel_stats(f"{fam}@{lvl}")[0]
    return n


@pytest.mark.parametrize("args", TAIL_CRHS_CASES)
def test_tail_top_coarse_rhs_matches_oracle(args, monkeypatch):
    launches = {}
    for switch in ("0", "1"):
        if switch == "1":
            monkeypatch.setenv("OMG_NO_TAIL_CRHS", "1")
        cfg = parse(args)
        dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
        for be in (dev, orc):
            setup_problem(be)
        c = dev.mg.ctx
        c.call("reset_stats")
        c.call("set_profiling", 1)
        for _ in range(2):
            if cfg["cycle"] == "f":
                assert dev.fmg(True, True) == orc.fmg(True, True)
            else:
                assert dev.vcycle(True) == orc.vcycle(True)
            _assert_same(dev, orc, ivs=(1, 2, 3, 4))
        c.call("set_profiling", 0)
        launches[switch] = _coarse_fill_launches(dev)
    assert launches["0"] < launches["1"], launches
