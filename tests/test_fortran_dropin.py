"""The Fortran drop-in (octree-mg_amd/fortran/): the reference's own golden
driver, compiled against the GPU-backed m_multigrid instead of the
reference's, must print the reference's histories bit for bit.

oracle/omg_golden.f90 is the program whose output under the reference
(amdflang -O2, MPICH) is tests/golden/golden.json; `make -C
octree-mg_amd/fortran drivers` links it against m_multigrid.f90 + libomg.so
as _build/omg_golden_gpu.  The binaries are built in the container (they need
the reference's host modules from /root/reference/src) and travel to the GPU
box with the tree.
"""
import hashlib
import json
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "octree-mg_amd", "fortran", "_build")
DRIVER = os.path.join(BUILD, "omg_golden_gpu")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["configs"]

needs_driver = pytest.mark.skipif(not os.path.exists(DRIVER),
                                  reason="Fortran drop-in not built (make -C octree-mg_amd/fortran drivers)")


def run_driver(args, dump=None, timeout=300):
    cmd = [DRIVER] + args.split() + [dump or "x"]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)


def parse(out):
    its = []
    for line in out.splitlines():
        f = line.split()
        if f and f[0] == "IT":
            its.append({"it": int(f[1]), "err": f[2], "res": f[3], "max_res": f[4]})
    return its


@needs_driver
def test_dropin_fails_loudly_without_gpu():
    """No GPU visible: the drop-in must stop with the backend's error, never
    fall back to the host loops."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = run_driver("8 16 16 16 1 v gs lpl 0 sol sol 1 lb 0", timeout=120)
    assert p.returncode != 0
    assert "GPU backend" in (p.stdout + p.stderr)
    assert len(parse(p.stdout)) == 1      # only the it-0 line before the first cycle


@pytest.mark.gpu
@needs_driver
@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_dropin_golden(name):
    cfg = GOLDEN[name]
    ref = cfg["runs"]["1"]
    key = "phi_sha256" if "phi_sha256" in ref else "rhs_sha256" if "rhs_sha256" in ref else None
    with tempfile.TemporaryDirectory() as td:
        dump = os.path.join(td, "dump.bin") if key else None   # phi, or rhs for ahelm
        p = run_driver(cfg["args"], dump)
        if "error" in ref:   # the reference's error stop, after the same printed lines
            assert p.returncode != 0
            assert "ERROR STOP: " + ref["error"] in p.stdout + p.stderr
            assert parse(p.stdout) == ref["history"]
            return
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        assert parse(p.stdout) == ref["history"]
        if dump:
            with open(dump, "rb") as f:
                assert hashlib.sha256(f.read()).hexdigest() == ref[key]


MPIEXEC = "/opt/conda/bin/mpiexec"
# every configuration the reference ran at 2-4 ranks, at the largest such
# count (5, 6 and 8 ranks stay with the loopback replay,
# tests/test_gpu_multirank.py)
MULTI = sorted({n: max(int(r) for r in e["runs"] if 1 < int(r) <= 4)
                for n, e in GOLDEN.items()
                if not e.get("big") and any(1 < int(r) <= 4 for r in e["runs"])}.items())


def _rank_dumps(fn):
    """The golden driver's per-rank dumps (<fn>.r<rank>) in the one-rank
    order (tests/golden/make_golden.py read_rank_dumps)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(ROOT, "tests", "golden",
                                                                              "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg.read_rank_dumps(fn)


@pytest.mark.gpu
@needs_driver
@pytest.mark.parametrize("name,ranks", MULTI)
def test_dropin_golden_multirank(name, ranks):
    """`mpiexec -n R` of the golden driver linked against the drop-in: R MPI
    ranks on one GPU, which RCCL refuses, so the drop-in takes the host
    transport over MPI (include/omg.h omg_set_host_transport; same plans,
    packing kernels and reduction orders as RCCL).  The printed history and
    every rank's final phi must be the reference's R-rank run, bit for bit:
    the Fortran drop-in's multi-rank bookkeeping (ranks, my_ids uploads and
    downloads, collective calls) end to end."""
    run = GOLDEN[name]["runs"][str(ranks)]
    key = "phi_sha256" if "phi_sha256" in run else "rhs_sha256" if "rhs_sha256" in run else None
    with tempfile.TemporaryDirectory() as td:
        dump = os.path.join(td, "dump.bin") if key else None
        cmd = [MPIEXEC, "-n", str(ranks), DRIVER] + GOLDEN[name]["args"].split() + [dump or "x"]
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        if "error" in run:
            assert p.returncode != 0
            assert "ERROR STOP: " + run["error"] in p.stdout + p.stderr
            assert parse(p.stdout) == run["history"]
            return
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        assert parse(p.stdout) == run["history"]
        if dump:
            assert hashlib.sha256(_rank_dumps(dump)).hexdigest() == run[key]


REF_PROGRAMS = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_programs.json")))["runs"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(REF_PROGRAMS))
def test_reference_programs_unchanged(name):
    """The reference's tests/test_uniform_grid.f90 and test_refinement.f90,
    unmodified, linked against the drop-in: same printed error histories as
    the reference build (tests/golden/make_ref_programs.py)."""
    run = REF_PROGRAMS[name]
    exe = os.path.join(BUILD, run["program"])
    if not os.path.exists(exe):
        pytest.skip("Fortran drop-in not built")
    ranks = run.get("ranks", 1)   # `mpiexec -n 4 test_refinement`: 4 ranks on one GPU, host transport
    cmd = ([MPIEXEC, "-n", str(ranks)] if ranks > 1 else []) + [exe] + run["args"].split()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = [ln.rstrip() for ln in p.stdout.splitlines()
             if "max solution error" in ln or "max err" in ln]
    assert lines == run["lines"]


RESIDENT = os.path.join(BUILD, "omg_golden_gpu_resident")
RESIDENT_CASES = ["c1_gsrb_f_maxres", "per32_gsrb_v", "helm32_gs_c0", "ref3_gsrb_v", "vlpl32_gsrb_v",
                  "u32_gs_d0_one", "diff_helm_d2_d0", "diff_helm_d1_ref2", "diff_vhelm_d1_per",
                  "c4_ref2_box16_gsrb", "regrid_ref2_gs", "regrid_c4_box16_gsrb"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", RESIDENT_CASES)
def test_dropin_resident_mode(name):
    """mg_gpu_set_resident(.true.): the cycles run back to back on GPU data and
    the host copy is only refreshed (mg_gpu_to_host) for printing; the
    histories are still the reference's."""
    if not os.path.exists(RESIDENT):
        pytest.skip("Fortran drop-in drivers not built")
    cfg = GOLDEN[name]
    p = subprocess.run([RESIDENT] + cfg["args"].split() + ["x"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert parse(p.stdout) == cfg["runs"]["1"]["history"]


# -- m_free_space ------------------------------------------------------------
FREE_DRIVER = os.path.join(BUILD, "omg_free_golden_gpu")
FREE_GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "free_golden.json")))["configs"]


def _free_history(its):
    import struct
    f = lambda h: struct.unpack(">d", bytes.fromhex(h))[0]
    return [{"it": h["it"], "err": f(h["err"]), "err2": f(h["err2"]), "max_res": f(h["max_res"])} for h in its]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FREE_GOLDEN))
def test_dropin_free_space_golden(name):
    """oracle/omg_free_golden.f90 (the reference's test_free_space set-up)
    against the drop-in m_free_space: the reference's histories within the
    round-off tolerance of the Green's-function solve (tests/freedriver.py)."""
    from tests import freedriver as FD
    if not os.path.exists(FREE_DRIVER):
        pytest.skip("Fortran drop-in drivers not built")
    cfg = FREE_GOLDEN[name]
    p = subprocess.run([FREE_DRIVER] + cfg["args"].split() + ["x"], capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    its = []
    for line in p.stdout.splitlines():
        f = line.split()
        if f and f[0] == "IT":
            its.append({"it": int(f[1]), "err": f[2], "err2": f[3], "max_res": f[4]})
    FD.compare_history(_free_history(its), FD.golden_history(cfg), FD.parse(cfg["args"]), name)


@pytest.mark.gpu
def test_reference_free_space_program():
    """The reference's tests/test_free_space.f90, unmodified, linked against
    the drop-in (8 64 64 64, its default fft_frac 0.15, 5 FMG iterations):
    the printed max err / err2 / residual match the reference's run of the
    same program (free64_box8_f) within the stated tolerance."""
    from tests import freedriver as FD
    exe = os.path.join(BUILD, "test_free_space_3d")
    if not os.path.exists(exe):
        pytest.skip("Fortran drop-in not built")
    p = subprocess.run([exe, "8", "64", "64", "64"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    toks = p.stdout.replace("\n", " ").split("max err/err2/res")[1:]
    got = []
    for n, t in enumerate(toks, 1):
        v = [float(x) for x in t.split()[:3]]
        got.append({"it": n, "err": v[0], "err2": v[1], "max_res": v[2]})
    cfg = FREE_GOLDEN["free64_box8_f"]
    FD.compare_history(got, FD.golden_history(cfg), FD.parse(cfg["args"]), "test_free_space")
