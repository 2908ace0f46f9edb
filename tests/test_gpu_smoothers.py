"""The round-3 smoother paths, bit for bit against the C oracle on every
stored cell:

- lexicographic GS over compacted hyperplanes (k_gs_lex_plane), which reads
  rhs from a plane-order copy: the copy must follow every change of rhs,
  between cycles through the API and inside a cycle (update_coarse rewrites
  the rhs of the levels below);
- the resident red-black smoother (k_gsrb_resident) on small levels: all
  substeps of one smooth_boxes call in one launch with a grid barrier between
  them, with physical and refinement-boundary faces, Laplacian and Helmholtz,
  boxes of 16 and 8, several cycle counts.

The environment switches OMG_NO_GS_PLANE / OMG_NO_RESIDENT (read when a
context is created) give the old paths; both must agree with the oracle."""
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


GS_CASES = ["16 64 64 64 2 v gs lpl 0 d0 sol 1 lb 0",
            "16 64 64 64 2 v gs helm 2.5 n0 sol 1 lb 0",
            "8 32 32 32 2 v gs lpl 0 sol sol 2 lb 0",
            "16 128 128 128 1 v gs lpl 0 sol sol 2 lb 0"]


@pytest.mark.parametrize("env", [(), ("OMG_NO_GS_PLANE",)], ids=["plane", "lines"])
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


RES_CASES = ["16 128 128 128 2 v gsrb lpl 0 sol sol 2 lb 0",    # C4's tree: refinement boundaries
             "16 128 128 128 2 v gsrb helm 3 d0 sol 1 lb 0",
             "16 64 64 64 2 v gsrb lpl 0 per sol 1 lb 0",
             "8 64 64 64 2 v gsrb lpl 0 n0 sol 2 lb 0",
             "16 128 128 128 2 f gsrb lpl 0 c0 sol 1 lb 0"]


@pytest.mark.parametrize("env", [(), ("OMG_NO_RESIDENT",)], ids=["resident", "per-substep"])
@pytest.mark.parametrize("args", RES_CASES)
def test_resident_smoother_matches_oracle(args, env, monkeypatch):
    dev, orc = _pair(args, monkeypatch, env)
    cfg = parse(args)
    for _ in range(2):
        if cfg["cycle"] == "f":
            assert dev.fmg(True, True) == orc.fmg(True, True)
        else:
            assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc, ivs=(1, 2, 3, 4))


@pytest.mark.parametrize("down,up", [(1, 1), (3, 2), (2, 4)])
def test_resident_smoother_cycle_counts(down, up, monkeypatch):
    """n_cycle_down / n_cycle_up other than 2: the resident launch covers
    substeps 1 .. 2 n (minus the one k_smooth_resid fuses), or 2 .. 2 n after
    the fused prolongation."""
    import pyoracle  # noqa: F401  (on sys.path once OracleBackend exists; checker only)
    cfg = parse("16 128 128 128 2 v gsrb lpl 0 sol sol 2 lb 0")
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    dev.mg.n_cycle_down, dev.mg.n_cycle_up = down, up
    dev.mg._push_methods()
    orc.o.configure(op=pyoracle.LAPLACIAN, lam=0.0, smoother=pyoracle.GSRB, n_cycle_down=down,
                    n_cycle_up=up, subtract_mean=False)
    for be in (dev, orc):
        setup_problem(be)
    for _ in range(2):
        assert dev.vcycle(True) == orc.vcycle(True)
        _assert_same(dev, orc, ivs=(1, 2, 3, 4))


@pytest.mark.parametrize("args", ["16 128 128 128 1 v gsrb lpl 0 sol sol 2 lb 0",
                                  "8 32 32 32 1 v gsrb helm 2 d0 sol 1 lb 0"])
def test_resident_smoother_stale_ghosts(args):
    """smooth_boxes right after random data (ghosts stale): the first substep
    reads the stale ghosts and is followed by a full fill, then the resident
    launch runs the rest."""
    cfg = parse(args)
    dev, orc = DeviceBackend(cfg), OracleBackend(cfg)
    for be in (dev, orc):
        _random_fill(be, np.random.default_rng(13))
    for lvl in list(dev.levels())[::-1]:
        for n_cycle in (1, 3):
            dev.mg.ctx.call("smooth_boxes", lvl, n_cycle)
            orc.o.smooth_boxes(lvl, n_cycle)
            _assert_same(dev, orc)
