#!/usr/bin/env python3
"""Record the error lines the reference's own test programs print.

Runs tests/test_uniform_grid.f90 and tests/test_refinement.f90 of the
reference, compiled unmodified by `make -C oracle ref` (amdflang -O2, MPICH),
and stores the lines that carry numbers the solver produced ("max solution
error ... max residual ..." / "max err ...") in ref_programs.json.
tests/test_fortran_dropin.py runs the same programs built against the
GPU-backed m_multigrid (octree-mg_amd/fortran) and compares these lines
verbatim.
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "..", "..", "oracle", "_ref")

RUNS = {
    "uniform_v": ("test_uniform_grid_3d", "8 64 64 64 10 f"),
    "uniform_fmg": ("test_uniform_grid_3d", "8 64 64 64 10 t"),
    "uniform_box16_v": ("test_uniform_grid_3d", "16 64 64 64 6 f"),
    "refinement2_v": ("test_refinement_3d", "2 16 64 64 64 5 f"),
    "refinement3_fmg": ("test_refinement_3d", "3 8 32 32 32 5 t"),
    # BASELINE C4 as the reference runs it: `mpiexec -n 4 test_refinement`
    # on the one-level-refined 128^3 tree, box 16; and a 3-level tree at 3
    # ranks (refinement boundaries across ranks)
    "refinement2_c4_4ranks": ("test_refinement_3d", "2 16 128 128 128 5 f", 4),
    "refinement3_fmg_3ranks": ("test_refinement_3d", "3 8 32 32 32 5 t", 3),
}
MPIEXEC = "/opt/conda/bin/mpiexec"


def error_lines(out):
    return [ln.rstrip() for ln in out.splitlines() if "max solution error" in ln or "max err" in ln]


def main():
    rec = {}
    for name, spec in RUNS.items():
        prog, args = spec[:2]
        ranks = spec[2] if len(spec) > 2 else 1
        cmd = ([MPIEXEC, "-n", str(ranks)] if ranks > 1 else []) + [os.path.join(REF, prog)] + args.split()
        out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
        rec[name] = {"program": prog, "args": args, "lines": error_lines(out)}
        if ranks > 1:
            rec[name]["ranks"] = ranks
    with open(os.path.join(HERE, "ref_programs.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_ref_programs.py",
                   "reference": "FermiQ/octree-mg @ 2025-06-14 tests/*.f90, amdflang -O2, MPICH 3.3.2",
                   "runs": rec}, f, indent=1)


if __name__ == "__main__":
    main()
