#!/usr/bin/env python3
"""Free-space boundary conditions (m_free_space) on one GPU, next to the
reference's own CPU path on the host cores.

For each configuration (oracle/omg_free_golden arguments: box nx ny nz n_its
fft_frac cycle) the test_free_space set-up runs through
octree_mg_amd.mg_poisson_free_3d:
  * first call (new_rhs): rhs restriction, Green's function of the FFT grid,
    FFT solve, boundary table of every level, guess, one FMG;
  * later calls (no new rhs): one FMG each (what the reference's test times
    after its first iteration);
  * a new rhs on the same grid: FFT solve + boundary table + guess + FMG;
with the device phases from HIP events (omg_set_profiling: free_fft_solve is
the gather + D2Z + spectrum product + Z2D + planes).  The CPU column is the
reference itself (oracle/_ref/omg_free_golden: m_free_space + its bundled
PSolver, amdflang -O2, MPICH, mpiexec -n P), mpi_wtime per call averaged over
its n_its calls (the first included, as its test_free_space reports).

usage: free_bench.py [--cpu-ranks P] [--no-cpu] [--only NAME ...]"""
import argparse
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

omg = __graft_entry__.load_package()
from tests import freedriver as FD  # noqa: E402  (the set-up shared with the parity tests)

CONFIGS = {
    "free64": ("8 64 64 64 5 0.15 f", "tests/test_free_space as shipped (64^3, box 8)"),
    "free256": ("16 256 256 256 5 0.15 f", "256^3, box 16, FFT level 128^3"),
    "free512": ("16 512 512 512 3 0.15 f", "512^3, box 16, FFT level 256^3 (512^3 transforms)"),
}


def sync(mg):
    mg.ctx.call("synchronize")


def gpu_run(args, reps=3):
    cfg = FD.parse(args)
    d = FD._Device(cfg)
    mg = d.mg
    mg.ctx.call("set_profiling", 1)
    sync(mg)
    t0 = time.perf_counter()
    d.step(cfg, 1)
    sync(mg)
    first = time.perf_counter() - t0
    fft_first = mg.ctx.kernel_stats("free_fft_solve")[1]
    mg.ctx.call("reset_stats")
    d.step(cfg, 2)      # warm
    sync(mg)
    t0 = time.perf_counter()
    for _ in range(reps):
        d.step(cfg, 2)
    sync(mg)
    later = (time.perf_counter() - t0) / reps
    mg.ctx.call("reset_stats")
    t0 = time.perf_counter()
    for _ in range(reps):
        omg.mg_poisson_free_3d(mg, True, cfg["frac"], cfg["cycle"] == "f", max_res=True)
    sync(mg)
    new_rhs = (time.perf_counter() - t0) / reps
    n, ms, _ = mg.ctx.kernel_stats("free_fft_solve")
    lvl = omg.free_space.fft_level(mg, cfg["frac"])
    nx = [int(v) * mg.box_size_lvl[lvl] + 2 for v in mg.ix[mg.lvls[lvl].ids].max(axis=0)]
    N = [omg.free_space.fft_length(max(2 * (v - 2), v)) for v in nx]
    cells = mg.number_of_unknowns()
    omg.mg_deallocate_storage(mg)
    return {"first_call_ms": 1e3 * first, "fmg_call_ms": 1e3 * later, "new_rhs_call_ms": 1e3 * new_rhs,
            "fft_solve_ms": ms / max(n, 1), "fft_solve_first_ms": fft_first, "fft_lvl": lvl, "nx": nx,
            "fft_grid": N, "cells": cells, "fmg_cell_updates_per_s": cells / later}


def cpu_run(args, ranks):
    ref = os.path.join(ROOT, "oracle", "_ref", "omg_free_golden")
    if not os.path.exists(ref):
        return None
    cmd = (["/opt/conda/bin/mpiexec", "-n", str(ranks)] if ranks > 1 else []) + [ref] + args.split() + ["x"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=1200).stdout
    m = re.search(r"TIME\s+(\S+)", out)
    return float(m.group(1)) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-ranks", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    rows = []
    for name, (args, desc) in CONFIGS.items():
        if a.only and name not in a.only:
            continue
        g = gpu_run(args)
        c = None if a.no_cpu else cpu_run(args, a.cpu_ranks)
        rec = {"config": name, "args": args, "desc": desc, "gpu": g,
               "cpu_s_per_call": c, "cpu_ranks": a.cpu_ranks if c else None}
        print(json.dumps(rec), flush=True)
        rows.append(rec)
    print("config     first ms   FMG call ms   new-rhs ms   FFT solve ms   FFT grid        CPU s/call")
    for r in rows:
        g = r["gpu"]
        print("%-9s %9.2f %12.2f %12.2f %13.3f   %-14s %s" % (
            r["config"], g["first_call_ms"], g["fmg_call_ms"], g["new_rhs_call_ms"], g["fft_solve_ms"],
            "x".join(map(str, g["fft_grid"])), "%.3f" % r["cpu_s_per_call"] if r["cpu_s_per_call"] else "-"))


if __name__ == "__main__":
    main()
