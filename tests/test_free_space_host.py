"""Free-space boundary conditions (m_free_space) on the CPU: the oracle's
restatement of PSolver pinned against the reference's own output, the oracle's
whole mg_poisson_free_3d against the reference's histories, and the host logic
of the product (FFT level choice, transform lengths, the boundary callback,
the Gaussian table) — no GPU."""
import json
import os
import re
import sys

import numpy as np
import pytest

from tests import freedriver as FD

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import free_space_oracle as F  # noqa: E402  (checker)

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "free_golden.json")))["configs"]
fs = FD.omg.free_space


@pytest.mark.parametrize("name", ["free16_fftonly", "free24x16_fftonly"])
def test_green_solve_matches_reference_psolver(name):
    """The direct-convolution restatement against PSolver's own result (the
    FFT level is the highest, so the reference's phi is PSolver's output):
    the cube branch and the anisotropic (hx != hy) branch of Free_Kernel."""
    e = GOLDEN[name]
    cfg = FD.parse(e["args"])
    ref = np.load(os.path.join(ROOT, "tests", "golden", e["phi_npy"]))
    dom = cfg["domain"]
    nx = [d + 2 for d in dom]
    dr = [1.0 / d for d in dom]
    tree = FD.build_tree(cfg, FD.T.MGTree())
    lvl = tree.highest_lvl
    rhs, _ = FD.level_fields(tree, lvl, tree.lvls[lvl].ids)
    nc = tree.box_size_lvl[lvl]
    rho = np.zeros(nx)
    for n, id_ in enumerate(tree.lvls[lvl].ids):
        p = (tree.ix[id_] - 1) * nc + 1
        rho[p[0]:p[0] + nc, p[1]:p[1] + nc, p[2]:p[2] + nc] = \
            F.RHS_FAC * rhs[n, 1:-1, 1:-1, 1:-1].transpose(2, 1, 0)
    pot = F.free_solve(rho, dr, (nx[0], nx[2], nx[2]))[1:-1, 1:-1, 1:-1]
    tol = FD.tolerances(cfg)["phi_abs"]
    assert np.max(np.abs(pot - ref)) <= tol, np.max(np.abs(pot - ref))


@pytest.mark.parametrize("name", ["free16_fftonly", "free32_fftonly", "free64_box8_f", "free64_box8_v",
                                  "free48x32_f", "free64_lowest_f"])
def test_oracle_free_space_matches_reference_history(name):
    """mg_poisson_free_3d restated over the C oracle: every iteration's max
    error, rms error and max_res as the reference printed them, within the
    stated round-off tolerance."""
    e = GOLDEN[name]
    out = FD.run_oracle(e["args"])
    FD.compare_history(out["history"], FD.golden_history(e), FD.parse(e["args"]), name)


def test_reference_histories_do_not_depend_on_rank_count():
    """The reference's own multi-rank runs agree with its one-rank runs (max
    error and max_res bit for bit; the rms error only up to MPI_SUM order),
    so the multi-rank device runs are held to the same goldens."""
    for name, e in GOLDEN.items():
        r1 = e["runs"]["1"]["history"]
        for r, run in e["runs"].items():
            assert [h["err"] for h in run["history"]] == [h["err"] for h in r1], (name, r)
            assert [h["max_res"] for h in run["history"]] == [h["max_res"] for h in r1], (name, r)


@pytest.mark.parametrize("args,frac,lvl", [("8 64 64 64", 0.15, 0), ("8 64 64 64", 1.0, 1),
                                           ("8 64 64 64", 0.001, -4), ("16 128 128 128", 0.15, 0),
                                           ("8 48 32 32", 0.15, 0), ("8 16 16 16", 0.15, 0),
                                           ("8 16 16 16", 0.01, -2)])
def test_fft_level_choice(args, frac, lvl):
    """m_free_space.f90:80-93: the product's host choice equals the oracle's
    restatement and the expected level."""
    cfg = FD.parse(args + " 1 %g f" % frac)
    tree = FD.build_tree(cfg, FD.T.MGTree())
    assert fs.fft_level(tree, frac) == F.fft_level(tree, frac) == lvl


def test_fft_lengths():
    for m in range(2, 600):
        n = fs.fft_length(m)
        assert n >= m and n % 2 == 0
        r = n
        for f in (2, 3, 5, 7):
            while r % f == 0:
                r //= f
        assert r == 1
        assert all(fs.fft_length(k) == n for k in range(m, n + 1))


def test_gequad_table_matches_oracle():
    """The product's Gaussian expansion (csrc/omg_free_gequad.h) is the one
    the oracle restates (both from gequad, build_kernel.f90:1549-1740)."""
    src = open(os.path.join(ROOT, "octree-mg_amd", "csrc", "omg_free_gequad.h")).read()
    tabs = {}
    for name in ("kGequadP", "kGequadW"):
        body = src[src.index(name):]
        body = body[body.index("{") + 1:body.index("}")]
        tabs[name] = [float.fromhex(v) for v in re.findall(r"0x[0-9a-fA-F.]+p[+-]\d+", body)]
    assert tabs["kGequadP"] == F.GEQUAD_P
    assert tabs["kGequadW"] == F.GEQUAD_W
    assert len(F.GEQUAD_P) == len(F.GEQUAD_W) == 89


def test_boundary_callback_matches_oracle_interpolation():
    """The host boundary callback the Python mirror installs
    (FreeBoundary, ghost_cells_free_bc) equals the oracle's interp_bc on the
    same planes, bit for bit, on every physical face of every level."""
    cfg = FD.parse("8 32 32 32 1 0.15 f")
    tree = FD.build_tree(cfg, FD.T.MGTree())
    lvl = 0
    nx = [18, 18, 18]
    rng = np.random.default_rng(5)
    sizes = [nx[1] * nx[2]] * 2 + [nx[0] * nx[2]] * 2 + [nx[0] * nx[1]] * 2
    flat = rng.standard_normal(sum(sizes))
    cb = fs.FreeBoundary(tree, lvl, nx, flat)
    planes, pos = [], 0
    shapes = [(nx[2], nx[1])] * 2 + [(nx[2], nx[0])] * 2 + [(nx[1], nx[0])] * 2
    for s, sh in zip(sizes, shapes):
        planes.append(flat[pos:pos + s].reshape(sh))
        pos += s
    dr = tree.dr[lvl]
    n_faces = 0
    for l in range(tree.lowest_lvl, tree.highest_lvl + 1):
        nc = tree.box_size_lvl[l]
        for id_ in tree.lvls[l].ids:
            for nb in range(1, 7):
                if tree.neighbors[id_, nb - 1] >= 0:
                    continue
                d = (nb - 1) // 2
                ixs = [q for q in range(3) if q != d]
                rr = tree.get_face_coords(int(id_), nb, nc)
                ref = F._interp(planes, nb, rr[:, :, ixs[0]], rr[:, :, ixs[1]],
                                [tree.r_min[q] - 0.5 * dr[q] for q in ixs], [1.0 / dr[q] for q in ixs])
                t, vals = cb(tree, int(id_), nc, 1, nb)
                assert t == FD.T.MG_BC_DIRICHLET
                assert np.array_equal(vals, np.ascontiguousarray(ref.T).reshape(-1))
                n_faces += 1
    assert n_faces > 6
