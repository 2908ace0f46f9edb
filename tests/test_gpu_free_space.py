"""Free-space boundary conditions on the GPU (omg_poisson_free_3d: the
Green's function, the hipFFT solve, the boundary table and the multigrid
cycle in libomg.so) against the reference's own results
(tests/golden/free_golden.json, PSolver's output in tests/golden/*_phi.npy)
and against the CPU oracle, within the round-off tolerance of
tests/freedriver.py (the transforms sum in another order than PSolver)."""
import ctypes
import json
import os

import numpy as np
import pytest

from tests import freedriver as FD

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "free_golden.json")))["configs"]

pytestmark = pytest.mark.gpu


def _highest_xyz(mg, phi):
    """[box, k, j, i] of the highest level (my_ids order) -> [x, y, z]."""
    lvl = mg.highest_lvl
    nc = mg.box_size_lvl[lvl]
    dom = np.max(mg.ix[mg.lvls[lvl].ids], axis=0) * nc
    out = np.zeros(dom)
    for n, id_ in enumerate(mg.lvls[lvl].my_ids):
        p = (mg.ix[id_] - 1) * nc
        out[p[0]:p[0] + nc, p[1]:p[1] + nc, p[2]:p[2] + nc] = phi[n, 1:-1, 1:-1, 1:-1].transpose(2, 1, 0)
    return out


@pytest.mark.parametrize("name", ["free16_fftonly", "free24x16_fftonly"])
def test_fft_solve_matches_reference_psolver(name):
    """The FFT level is the highest: phi is the device's Green's-function
    solve itself, against PSolver's output."""
    e = GOLDEN[name]
    cfg = FD.parse(e["args"])
    out = FD.run_device(e["args"])
    ref = np.load(os.path.join(ROOT, "tests", "golden", e["phi_npy"]))
    got = _highest_xyz(out["mg"], out["phi"])
    d = float(np.max(np.abs(got - ref)))
    assert d <= FD.tolerances(cfg)["phi_abs"], d
    FD.compare_history(out["history"], FD.golden_history(e), cfg, name)


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_free_space_matches_reference_history(name):
    """Every iteration of the reference's test_free_space set-up (max error,
    rms error, max_res) within the stated tolerance, one GPU."""
    e = GOLDEN[name]
    out = FD.run_device(e["args"])
    FD.compare_history(out["history"], FD.golden_history(e), FD.parse(e["args"]), name)


@pytest.mark.parametrize("name", ["free64_box8_f", "free48x32_f", "free64_lowest_f"])
def test_free_space_final_phi_matches_oracle(name):
    """The final phi of the highest level, device against the CPU oracle."""
    e = GOLDEN[name]
    cfg = FD.parse(e["args"])
    dev = FD.run_device(e["args"])
    orc = FD.run_oracle(e["args"])
    d = float(np.max(np.abs(dev["phi"][:, 1:-1, 1:-1, 1:-1] - orc["phi"][:, 1:-1, 1:-1, 1:-1])))
    assert d <= FD.tolerances(cfg)["phi_abs"], d


@pytest.mark.parametrize("name,ranks", [("free64_box8_f", 2), ("free64_box8_f", 4), ("free64_box16_f", 2),
                                        ("free128_box16_f", 4), ("free32_fftonly", 2)])
def test_free_space_multirank_matches_reference(name, ranks):
    """Several ranks through the loopback transport: the FFT level's rhs is
    gathered on every rank, each solves the same grid, the boundary table
    covers its own boxes; the reference's run at that rank count."""
    e = GOLDEN[name]
    out = FD.run_device_loopback(e["args"], ranks)
    for h in out["all"]:
        assert h == out["all"][0]
    FD.compare_history(out["history"], FD.golden_history(e, ranks), FD.parse(e["args"]), name)


def test_free_space_replicated_fft_level():
    """The FFT level replicated on every rank (omg_set_coarse_replication):
    the rhs is gathered locally, no exchange."""
    e = GOLDEN["free64_box8_f"]
    out = FD.run_device_loopback(e["args"], 2, rep_cells=40000)
    FD.compare_history(out["history"], FD.golden_history(e, 2), FD.parse(e["args"]), "replicated")


def test_first_call_needs_new_rhs():
    cfg = FD.parse("8 32 32 32 1 0.15 f")
    d = FD._Device(cfg)
    with pytest.raises(RuntimeError, match="first call requires new_rhs"):
        FD.omg.mg_poisson_free_3d(d.mg, False, 0.15, True)


def test_laplacian_required():
    cfg = FD.parse("8 32 32 32 1 0.15 f")
    d = FD._Device(cfg)
    d.mg.operator_type = FD.T.MG_HELMHOLTZ
    with pytest.raises(RuntimeError, match="laplacian operator required"):
        FD.omg.mg_poisson_free_3d(d.mg, True, 0.15, True)
    # the C-ABI refuses it too (the device's operator, not the host's flag)
    FD.omg.helmholtz_set_lambda(d.mg, 1.0)
    FD.omg.mg_set_methods(d.mg)
    m = ctypes.c_double(0.0)
    with pytest.raises(FD.omg.device.OmgError, match="laplacian operator required"):
        d.mg.ctx.call("poisson_free_3d", 1, 0.15, 1, 1, ctypes.byref(m), np.zeros(3), None)


def test_boundary_callback_reproduces_device_table():
    """After the solve, the host callback installed in mg.bc (the planes
    copied back) tabulates exactly the values the device stored: pushing it
    again and re-running the cycle changes nothing."""
    e = GOLDEN["free64_box8_f"]
    cfg = FD.parse(e["args"])
    d = FD._Device(cfg)
    d.step(cfg, 1)
    a = d.step(cfg, 2)
    phi_a = d.mg.get_level(d.mg.highest_lvl, 1)
    d2 = FD._Device(cfg)
    d2.step(cfg, 1)
    d2.mg.push_bc([1])
    FD.omg.mg_phi_bc_store(d2.mg)
    b = d2.step(cfg, 2)
    phi_b = d2.mg.get_level(d2.mg.highest_lvl, 1)
    assert a == b
    assert np.array_equal(phi_a, phi_b)
