"""Three red-black substeps per pass (k_gsrb3, octree-mg_amd/csrc/omg_block.hip)
against the C oracle, every stored cell of every variable after each cycle.

The pass runs on levels of at least kB3MinBoxes boxes of 16^3 whose
faces are all same-GPU boxes (periodic uniform levels), for runs of three
consecutive substeps of smooth_boxes (m_multigrid.f90:404-424), and writes
phi into the level's second buffer.  The cases cover what changes around it:
odd and even numbers of passes per cycle (phi left in either buffer between
cycles and across FMG), the pending mean shift absorbed by its first substep
(periodic Laplacian), Helmholtz, FMG with and without a guess, and the level
with the pass switched off (OMG_NO_BLOCK3) in the same process.  The
up-smoothing's first pass on the 512-box level is the correct_children form
(its coarse level is the 64-box level below): the correction, substeps 1-3 and
the coarse level's res in one pass; OMG_NO_BLOCK3P switches that form off."""
import numpy as np
import pytest

from tests.mgdriver import OPS, DeviceBackend, OracleBackend, parse, setup_problem

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["512", "64", "64-col8"])
def _small_levels(monkeypatch, request):
    """The 128^3 trees here have a 512-box finest level; the pass serves
    levels of 4096 boxes and up by default (kB3MinBoxes), so lower the bound
    for these tests (read at context creation); the full-size golden
    c3_per512_box16 runs the default bound.  At 512 the finest level's
    correct_children form forms the coarse phi - old itself and stores the
    coarse res; at 64 the 64-box level runs the pass too, and its last
    up-smoothing pass stores its res for the form above it to read (C3's
    arrangement on levels 0 and 1).  64-col8: columns of 8 boxes (C3's level
    1 takes them; here the 128^3 tree's 512-box level, its whole z extent)."""
    bound, _, col = request.param.partition("-col")
    monkeypatch.setenv("OMG_BLOCK3_MIN_BOXES", bound)
    if col:
        monkeypatch.setenv("OMG_BLOCK3_COLUMN", col)


def _stored_mask(nc):
    s = nc + 2
    ix = np.arange(s)
    bnd = ((ix == 0) | (ix == s - 1)).astype(int)
    return (bnd[:, None, None] + bnd[None, :, None] + bnd[None, None, :]) < 2


def _assert_same(dev, orc, ivs=(1, 2, 3, 4)):
    for lvl in dev.levels():
        if not len(dev.my_ids(lvl)):
            continue
        m = _stored_mask(dev.tree.box_size_lvl[lvl])
        for iv in ivs:
            a, b = dev.get_level(lvl, iv), orc.get_level(lvl, iv)
            assert np.array_equal(a[:, m].view(np.uint64), b[:, m].view(np.uint64)), (lvl, iv)


def _pair(args, down, up, subtract_mean=None):
    cfg = parse(args)
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    import pyoracle  # on sys.path once OracleBackend exists (checker only)
    sub = cfg["bc"] == "per" if subtract_mean is None else subtract_mean
    dev.mg.n_cycle_down, dev.mg.n_cycle_up = down, up
    dev.mg.subtract_mean = sub
    dev.mg._push_methods()
    op = OPS[cfg["op"]]
    orc.o.configure(op=op, lam=cfg["lam"], smoother=pyoracle.GSRB, n_cycle_down=down, n_cycle_up=up,
                    subtract_mean=sub)
    for be in (dev, orc):
        setup_problem(be)
    return dev, orc


# (n_cycle_down, n_cycle_up): down-smoothing runs 2*down-1 substeps before the
# fused last one, up-smoothing 2*up-1 after the fused first one
@pytest.mark.parametrize("down,up", [(2, 2), (3, 1), (1, 3), (4, 4)])
@pytest.mark.parametrize("args", ["16 128 128 128 3 v gsrb lpl 0 per sol 1 lb 0",
                                  "16 128 128 128 3 v gsrb helm 2 per sol 1 lb 0"])
def test_block3_vcycles_match_oracle(args, down, up):
    dev, orc = _pair(args, down, up)
    for _ in range(3):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc)


@pytest.mark.parametrize("have_guess", [False, True])
def test_block3_fmg_matches_oracle(have_guess):
    dev, orc = _pair("16 128 128 128 2 f gsrb lpl 0 per sol 1 lb 0", 2, 2)
    for _ in range(2):
        assert dev.fmg(have_guess, True) == orc.fmg(have_guess, True)
        _assert_same(dev, orc)


@pytest.mark.parametrize("switch", ["OMG_NO_BLOCK3", "OMG_NO_BLOCK3P", "OMG_NO_BLOCK3R", "OMG_NO_BLOCK4P",
                                    "OMG_NO_DEFER_GC"])
def test_block3_switch_off_same_bits(monkeypatch, switch):
    """OMG_NO_BLOCK3=1 (one substep per launch) / OMG_NO_BLOCK3P=1 (the
    correction by k_prolong_smooth) / OMG_NO_BLOCK3R=1 (no res from the coarse
    level's last pass) / OMG_NO_BLOCK4P=1 (the correction form with three
    substeps, k_gsrb3, instead of k_gsrb4's four) and the default give the
    same state after each cycle."""
    args = "16 128 128 128 2 v gsrb lpl 0 per sol 1 lb 0"
    dev, orc = _pair(args, 3, 2)
    monkeypatch.setenv(switch, "1")
    ref = DeviceBackend(parse(args))
    ref.mg.n_cycle_down, ref.mg.n_cycle_up = 3, 2
    ref.mg._push_methods()
    setup_problem(ref)
    for _ in range(2):
        assert dev.vcycle(True) == ref.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, ref)


# The down-smoothing's four substeps as one k_gsrb4 pass, then the unfused
# residual + restriction (k_resid_restrict; the default where the substep count
# is a multiple of 4), and with OMG_NO_BLOCK4 k_gsrb3 + k_smooth_resid: every
# variable bitwise
@pytest.mark.parametrize("switch", [None, "OMG_NO_BLOCK4"])
@pytest.mark.parametrize("down,up", [(2, 2), (4, 1)])
@pytest.mark.parametrize("args", ["16 128 128 128 3 v gsrb lpl 0 per sol 1 lb 0",
                                  "16 128 128 128 3 v gsrb helm 2 per sol 1 lb 0"])
def test_block4_vcycles_match_oracle(monkeypatch, args, down, up, switch):
    if switch:
        monkeypatch.setenv(switch, "1")
    dev, orc = _pair(args, down, up)
    for _ in range(3):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc)


# the passes swap a level's phi buffer on the host as a captured
# cycle is recorded; a capture (1) or an instantiation / launch (2) that fails
# leaves phi where it was (graph_rollback restores the buffers).  The graph
# path needs a cycle that never waits for the host: no subtract_mean here (on
# both sides), so periodic Helmholtz with the level bound lowered.
@pytest.mark.parametrize("fail_at", [1, 2])
def test_block3_graph_failure_keeps_phi(monkeypatch, fail_at):
    from tests.mgdriver import omg
    monkeypatch.setenv("OMG_GRAPH", "1")
    monkeypatch.setenv("OMG_GRAPH_FAIL", str(fail_at))
    dev, orc = _pair("16 128 128 128 3 v gsrb helm 2 per sol 1 lb 0", 2, 2, subtract_mean=False)
    with pytest.raises(omg.device.OmgError, match="injected failure"):
        dev.vcycle(True)
    _assert_same(dev, orc)
    for _ in range(3):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc)


# Physical faces in the passes (round 6): a column with a
# Dirichlet / Neumann / continuous face (bc_to_gc, m_ghost_cells.f90:665-766)
# loads the ghosts there as they are on entry for its first substep and forms
# them from the cells next to the face for the later ones; its store wave
# writes them from the final cells.  Constant values: zero (omg_golden's d0 /
# n0 / c0) and per-face types and nonzero values (mx1 / mx2).  Non-cubic
# domains: columns shorter than the column length (both z faces physical in
# one column at col8), x extents of 6 boxes.  The passes' launch counts show
# that they ran on the finest level.
PHYS_CASES = ["16 128 128 128 3 v gsrb lpl 0 d0 sol 1 lb 0",
              "16 128 96 64 3 v gsrb helm 2 n0 sol 1 lb 0",
              "16 128 128 128 3 v gsrb lpl 0 c0 sol 1 lb 0",
              "16 96 128 64 3 v gsrb lpl 0 mx1 sol 1 lb 0",
              "16 128 64 96 3 v gsrb helm 2 mx2 sol 1 lb 0"]


def _block_launches(dev, lvl):
    return {f: dev.mg.ctx.kernel_stats(f"{f}@{lvl}")[0] for f in ("smoother_gsrb3", "smoother_gsrb4")}


@pytest.mark.parametrize("four", [False, True])
@pytest.mark.parametrize("down,up", [(2, 2), (3, 1), (1, 3)])
@pytest.mark.parametrize("args", PHYS_CASES)
def test_block3_physical_faces_match_oracle(monkeypatch, args, down, up, four):
    if four:
        monkeypatch.setenv("OMG_BLOCK4_PHYS", "1")
    dev, orc = _pair(args, down, up)
    dev.mg.ctx.call("set_profiling", 1)
    for _ in range(3):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc)
    dev.mg.ctx.call("synchronize")
    top = dev.tree.highest_lvl
    n = _block_launches(dev, top)
    if len(dev.my_ids(top)) >= int(__import__("os").environ["OMG_BLOCK3_MIN_BOXES"]):
        assert n["smoother_gsrb3"] + n["smoother_gsrb4"] > 0, n
        if four and down % 2 == 0:
            assert n["smoother_gsrb4"] > 0, n


@pytest.mark.parametrize("have_guess", [False, True])
def test_block3_physical_faces_fmg_matches_oracle(have_guess):
    dev, orc = _pair("16 128 128 128 2 f gsrb helm 2 mx1 sol 1 lb 0", 2, 2)
    for _ in range(2):
        assert dev.fmg(have_guess, True) == orc.fmg(have_guess, True)
        _assert_same(dev, orc)


def test_block3_physical_faces_switch_off_same_bits(monkeypatch):
    """OMG_NO_BLOCK3_PHYS=1 (levels with physical faces take one substep per
    launch) and the default give the same state after each cycle; an odd
    number of boxes in x (5) declines the columns, the same bits again."""
    for args in ("16 128 128 128 2 v gsrb lpl 0 mx2 sol 1 lb 0", "16 80 128 64 2 v gsrb lpl 0 mx1 sol 1 lb 0"):
        monkeypatch.delenv("OMG_NO_BLOCK3_PHYS", raising=False)
        dev, orc = _pair(args, 2, 2)
        monkeypatch.setenv("OMG_NO_BLOCK3_PHYS", "1")
        ref = DeviceBackend(parse(args))
        ref.mg.n_cycle_down, ref.mg.n_cycle_up = 2, 2
        ref.mg._push_methods()
        setup_problem(ref)
        for _ in range(2):
            assert dev.vcycle(True) == ref.vcycle(True) == orc.vcycle(True)
            _assert_same(dev, ref)


# Deferred ghosts (round 6): the stand-alone V-cycle without the max residual
# ends with k_gsrb4's correction form writing the top level's interior only;
# the next cycle's first pass reads no ghosts and writes them all, and every
# other reader fills them first (Level::gc_deferred).  Cycles without the
# max residual back to back, then each other reader in turn: the download
# (every stored cell, here after each step), the max-residual cycle, FMG,
# mg_apply_op, a fill, and the stand-alone fill decision after an upload.
def test_block3_deferred_ghosts_match_oracle():
    dev, orc = _pair("16 128 128 128 3 v gsrb lpl 0 per sol 1 lb 0", 2, 2)
    for _ in range(2):
        dev.vcycle(False); orc.vcycle(False)
    _assert_same(dev, orc)
    for want in (False, True, False):
        assert dev.vcycle(want) == orc.vcycle(want)
        _assert_same(dev, orc)
    dev.vcycle(False); orc.vcycle(False)
    assert dev.fmg(True, True) == orc.fmg(True, True)
    _assert_same(dev, orc)
    dev.vcycle(False); orc.vcycle(False)
    dev.apply_op(4); orc.apply_op(4)
    _assert_same(dev, orc)
    dev.vcycle(False); orc.vcycle(False)
    dev.fill_ghost_cells(1); orc.fill_ghost_cells(1)
    for lvl in dev.levels():   # an upload of phi (interior and ghosts) between cycles
        if len(dev.my_ids(lvl)):
            dev.set_level(lvl, 1, orc.get_level(lvl, 1))
    for _ in range(2):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc)
    # a cycle whose first substeps on the top level are one-substep launches
    # (one down-smoothing cycle: no block pass) right after a deferring cycle
    import pyoracle
    dev.vcycle(False); orc.vcycle(False)
    dev.mg.n_cycle_down, dev.mg.n_cycle_up = 1, 1
    dev.mg._push_methods()
    orc.o.configure(op=OPS["lpl"], lam=0.0, smoother=pyoracle.GSRB, n_cycle_down=1, n_cycle_up=1,
                    subtract_mean=True)
    for _ in range(2):
        dev.vcycle(False); orc.vcycle(False)
        _assert_same(dev, orc)


# The full-size goldens with physical faces take the passes at the default
# level bound (their 4096-box finest level): each configuration's history and
# final phi against the reference's run, with the launch counts showing that
# the finest level's substeps ran as k_gsrb3 passes
@pytest.mark.parametrize("name", ["c2_256_box16_gsrb_d0", "c5_helm256_box16_gsrb_d0", "mx1_256_box16"])
def test_block3_physical_goldens_take_the_passes(monkeypatch, name):
    import json
    import os
    from tests.mgdriver import _cycles, phi_digest
    monkeypatch.delenv("OMG_BLOCK3_MIN_BOXES", raising=False)
    monkeypatch.delenv("OMG_BLOCK3_COLUMN", raising=False)
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["configs"][name]
    cfg = parse(g["args"])
    dev = DeviceBackend(cfg)
    setup_problem(dev)
    dev.mg.ctx.call("set_profiling", 1)
    hist = _cycles(dev, cfg, None)
    dev.mg.ctx.call("synchronize")
    run = g["runs"]["1"]
    assert hist == run["history"]
    assert phi_digest(dev) == run["phi_sha256"]
    top = dev.tree.highest_lvl
    n = dev.mg.ctx.kernel_stats(f"smoother_gsrb3@{top}")[0]
    assert n >= 2 * cfg["n_its"], n   # (down and up, every cycle)
