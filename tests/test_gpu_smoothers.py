"""Lexicographic GS with the box in a register ring (k_gs_lex_reg), bit for
bit against the C oracle on every stored cell.  It reads rhs from a copy in
ring order, so the copy must follow every change of rhs: between cycles
through the API, and inside a cycle (update_coarse rewrites the rhs of the
levels below).  It serves 16^3 levels of at least 2048 boxes, hence the
256^3 cases; OMG_NO_GS_PLANE=1 selects the line-per-thread kernel (read when
a context is created), which must agree as well.  The ring runs an even number of sweeps with two ghost-face
sets and no fill in between (round 4; each sweep pushes its boundary layers
into the neighbours' other set, physical ghosts formed at load, k_phys_gc
after the last sweep); OMG_NO_GS_DBL=1 keeps the fill after every sweep."""
import numpy as np
import pytest

from tests.mgdriver import DeviceBackend, OracleBackend, parse, setup_problem
from tests.test_gpu_parity import _assert_same, _random_fill

pytestmark = pytest.mark.gpu


def _pair(args, monkeypatch, env=()):
    for k in env:
        monkeypatch.setenv(k, "1")
    cfg = parse(args)
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    for be in (dev, orc):
        setup_problem(be)
    return dev, orc


GS_CASES = ["16 256 256 256 1 v gs lpl 0 d0 sol 1 lb 0",
            "16 256 256 256 1 v gs helm 2.5 n0 sol 1 lb 0",
            "16 256 256 256 1 v gs lpl 0 sol sol 2 lb 0",
            "16 64 64 64 2 v gs lpl 0 d0 sol 1 lb 0"]


@pytest.mark.parametrize("env", [(), ("OMG_NO_GS_DBL",), ("OMG_NO_FILL_XL",), ("OMG_NO_GS_PLANE",)],
                         ids=["ring", "ring-fill", "ring-plainfill", "lines"])
@pytest.mark.parametrize("args", GS_CASES)
def test_gs_rhs_changes_between_cycles(args, env, monkeypatch):
    """V-cycles, then a new rhs on the finest level (upload) and on a level
    below (overwritten again by the next cycle's update_coarse), then more
    cycles and an FMG: every stored cell equal to the oracle's after each."""
    dev, orc = _pair(args, monkeypatch, env)
    for _ in range(2):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc, ivs=(1, 2, 3, 4))
    rng = np.random.default_rng(5)
    hi = dev.tree.highest_lvl
    for lvl in (hi, hi - 1):
        nc = dev.tree.box_size_lvl[lvl]
        new = rng.standard_normal((len(dev.my_ids(lvl)), nc + 2, nc + 2, nc + 2))
        dev.set_level(lvl, 2, new)
        orc.set_level(lvl, 2, new)
    for _ in range(2):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc, ivs=(1, 2, 3, 4))
    assert dev.fmg(True, True) == orc.fmg(True, True)
    _assert_same(dev, orc, ivs=(1, 2, 3, 4))


# two ghost sets with the other physical kinds: continuous (c0) and
# mg_phi_bc_store's stored values (the physical ghost reads rhs's ghost slot)
@pytest.mark.parametrize("args", ["16 256 256 256 1 v gs lpl 0 c0 sol 1 lb 0",
                                  "16 256 256 256 1 v gs helm 1.5 sol sol 1 lb 0"])
@pytest.mark.parametrize("stored", [False, True])
def test_gs_ghost_sets_physical_kinds(args, stored, monkeypatch):
    dev, orc = _pair(args, monkeypatch)
    if stored:
        dev.mg.ctx.call("phi_bc_store")
        orc.o.phi_bc_store()
    for n_cycle in (2, 1, 4):   # even: ghost sets, odd: a fill after every sweep
        hi = dev.tree.highest_lvl
        dev.mg.ctx.call("smooth_boxes", hi, n_cycle)
        orc.o.smooth_boxes(hi, n_cycle)
        _assert_same(dev, orc, ivs=(1, 2))
    assert dev.vcycle(True) == orc.vcycle(True)
    _assert_same(dev, orc, ivs=(1, 2, 3, 4))


@pytest.mark.parametrize("args", GS_CASES[:2])
def test_gs_per_operation_with_rhs_writes(args, monkeypatch):
    """smooth_boxes through the API between other rhs writers (apply_op into
    rhs, set_rhs, subtract_mean), on random data."""
    cfg = parse(args)
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    for be in (dev, orc):
        _random_fill(be, np.random.default_rng(3))
    c = dev.mg.ctx
    hi = dev.tree.highest_lvl
    dev.fill_ghost_cells(1); orc.fill_ghost_cells(1)
    c.call("smooth_boxes", hi, 1); orc.o.smooth_boxes(hi, 1)
    _assert_same(dev, orc)
    dev.apply_op(2); orc.apply_op(2)
    c.call("smooth_boxes", hi, 2); orc.o.smooth_boxes(hi, 2)
    _assert_same(dev, orc)
    c.call("set_rhs", 0.5, -1.25); orc.o.set_rhs(0.5, -1.25)
    c.call("smooth_boxes", hi, 1); orc.o.smooth_boxes(hi, 1)
    _assert_same(dev, orc)
    c.call("subtract_mean", 2, 0); orc.o.subtract_mean(2, 0)
    c.call("smooth_boxes", hi, 1); orc.o.smooth_boxes(hi, 1)
    _assert_same(dev, orc)
