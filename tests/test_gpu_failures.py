"""Failure detection and recovery on the GPU.

* A NaN or Inf anywhere in phi / rhs makes the requested max residual an
  error ("non-finite residual") instead of a number; the reference's max()
  drops NaN operands (src/m_multigrid.f90:226-234, 296-311).
* OMG_DEBUG=1 (the reference's DEBUG=1 build, makerules.make:13-17:
  -finit-real=snan): ghost faces start as signalling NaN, so a step that reads
  a ghost nothing has defined poisons the result, while every golden run still
  matches bit for bit (no defined run reads one); unstored edge / corner cells
  download as NaN.
* A HIP-graph cycle (OMG_GRAPH=1) that fails after its host logic ran leaves
  the context usable: the next cycles reproduce the golden history.
"""
import json
import os

import numpy as np
import pytest

from tests.mgdriver import (DeviceBackend, T, _cycles, omg, parse, phi_digest, run_loopback, run_problem,
                            setup_problem)

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))["configs"]

pytestmark = pytest.mark.gpu


def _poke(be, lvl, iv, value, box=0, cell=(3, 4, 5)):
    a = be.get_level(lvl, iv)
    a[(box,) + cell] = value
    be.set_level(lvl, iv, a)


@pytest.mark.parametrize("args", ["8 32 32 32 1 v gsrb lpl 0 d0 sol 1 lb 1",
                                  "16 64 64 64 1 v gsrb lpl 0 per sol 1 lb 1",
                                  "8 32 32 32 1 v gs helm 2 n0 sol 1 lb 1",
                                  "8 32 32 32 1 f gsrb lpl 0 sol sol 2 lb 1"])
@pytest.mark.parametrize("bad", [np.nan, np.inf])
def test_non_finite_rhs_is_an_error(args, bad):
    cfg = parse(args)
    be = DeviceBackend(cfg)
    setup_problem(be)
    _poke(be, be.tree.highest_lvl, T.MG_IRHS, bad)
    with pytest.raises(omg.device.OmgError, match="non-finite residual"):
        if cfg["cycle"] == "f":
            be.fmg(False, True)
        else:
            be.vcycle(True)


@pytest.mark.parametrize("bad", [np.nan, np.inf])
def test_non_finite_on_another_rank_is_an_error(bad):
    """Two loopback ranks, the bad value in a box rank 1 owns: the max over
    ranks propagates it like the device max does (round 3 combined the ranks
    with std::max_element, which skips a NaN after the first rank)."""
    args = "16 64 64 64 1 v gsrb lpl 0 d0 sol 1 lb 0"

    def body(be, rank, reduce):
        if rank == 1:   # (an rhs upload on one rank: allowed, only phi uploads are collective)
            _poke(be, be.tree.highest_lvl, T.MG_IRHS, bad, box=len(be.my_ids(be.tree.highest_lvl)) - 1)
        try:
            be.vcycle(True)
        except omg.device.OmgError as ex:
            return str(ex)
        return "no error"

    for msg in run_loopback(args, 2, body):
        assert "non-finite residual" in msg


def test_max_residual_lvl_reports_nan():
    be = DeviceBackend(parse("8 32 32 32 1 v gsrb lpl 0 d0 sol 1 lb 0"))
    setup_problem(be)
    hi = be.tree.highest_lvl
    assert np.isfinite(be.mg.ctx.scalar("max_residual_lvl", hi))
    _poke(be, hi, T.MG_IPHI, np.nan, box=5)
    with pytest.raises(omg.device.OmgError, match="max_residual_lvl: non-finite residual"):
        be.mg.ctx.scalar("max_residual_lvl", hi)


def test_diffusion_non_finite_is_an_error():
    be = DeviceBackend(parse("8 32 32 32 1 d1 gsrb helm 0.001 n0 phi 1 lb 0"))
    setup_problem(be)
    _poke(be, be.tree.highest_lvl, T.MG_IPHI, np.nan)
    with pytest.raises(omg.device.OmgError, match="diffusion_solve: non-finite residual"):
        be.diffusion(1, 0.001)


DEBUG_CASES = ["c1_gsrb_v", "u32_gs_d0_one", "per32_gsrb_v", "helm32_gsrb_n0", "ref3_gsrb_v", "vlpl32_gsrb_v",
               "u64_box16_gsrb_d0_one", "c1_gsrb_f_maxres"]


@pytest.mark.parametrize("name", DEBUG_CASES)
def test_debug_poison_keeps_golden_runs_exact(name, monkeypatch):
    monkeypatch.setenv("OMG_DEBUG", "1")
    e = GOLDEN[name]
    run = e["runs"]["1"]
    out = run_problem(e["args"], backend="device")
    assert out["history"] == run["history"]
    if "phi_sha256" in run:
        assert out["phi_sha256"] == run["phi_sha256"]


def test_debug_unstored_cells_download_as_nan(monkeypatch):
    monkeypatch.setenv("OMG_DEBUG", "1")
    be = DeviceBackend(parse("8 16 16 16 1 v gsrb lpl 0 d0 sol 1 lb 0"))
    setup_problem(be)
    a = be.get_level(be.tree.highest_lvl, T.MG_IPHI)
    s = a.shape[-1]
    ix = np.arange(s)
    bnd = ((ix == 0) | (ix == s - 1)).astype(int)
    n_bnd = bnd[:, None, None] + bnd[None, :, None] + bnd[None, None, :]
    assert np.all(np.isnan(a[:, n_bnd >= 2]))
    assert np.all(np.isfinite(a[:, n_bnd < 2]))


def test_debug_poison_catches_an_unfilled_ghost(monkeypatch):
    """Smoothing a level whose phi ghosts nothing ever defined: the reference
    reads its zero initialisation there, the debug context reads NaN and the
    residual says so.  Without OMG_DEBUG the same steps stay finite."""
    results = {}
    for dbg in ("0", "1"):
        monkeypatch.setenv("OMG_DEBUG", dbg)
        be = DeviceBackend(parse("8 32 32 32 1 v gsrb lpl 0 d0 one 1 lb 0"))
        setup_problem(be)   # rhs = 1 on the interior only: phi is never uploaded
        hi = be.tree.highest_lvl
        be.mg.ctx.call("smooth_boxes", hi, 1)
        try:
            results[dbg] = be.mg.ctx.scalar("max_residual_lvl", hi)
        except omg.device.OmgError as ex:
            results[dbg] = str(ex)
    assert isinstance(results["0"], float) and np.isfinite(results["0"])
    assert "non-finite residual" in results["1"]


@pytest.mark.parametrize("fail_at", [1, 2])
@pytest.mark.parametrize("name", ["c1_gsrb_v", "u64_box16_gsrb_d0_one", "c2_256_box16_gs_d0"])
def test_graph_failure_rolls_back(name, fail_at, monkeypatch):
    """OMG_GRAPH_FAIL injects one failure into the first captured cycle: 1 before
    the cycle's host logic runs, 2 after it ran (host state changed, graph
    never launched).  The call fails, nothing on the device changed, and the
    cycles after it reproduce the reference's history and final phi.  The
    256^3 GS case runs the register-ring sweep, whose ring-order rhs copy the
    failed capture had marked built without running it."""
    monkeypatch.setenv("OMG_GRAPH", "1")
    monkeypatch.setenv("OMG_GRAPH_FAIL", str(fail_at))
    e = GOLDEN[name]
    run = e["runs"]["1"]
    cfg = parse(e["args"])
    be = DeviceBackend(cfg)
    setup_problem(be)
    before = phi_digest(be)
    with pytest.raises(omg.device.OmgError, match="injected failure"):
        be.vcycle(cfg["maxres"])
    assert phi_digest(be) == before
    hist = _cycles(be, cfg)
    assert hist == run["history"]
    if "phi_sha256" in run:
        assert phi_digest(be) == run["phi_sha256"]
