#!/usr/bin/env python3
"""Throughput of every BASELINE.json configuration on one GPU, next to the
reference's own CPU path on the host cores.

For each configuration (omg_golden argument strings, tests/mgdriver.py):
  * GPU: the problem set up as omg_golden does, W warm-up cycles, then K timed
    V-cycles (FMG for 'f'), everything resident in HBM; cells = leaf cells of
    the tree, value = cells x cycles / s; the finest-level smoother launch time
    from HIP events (omg_set_profiling) gives its HBM roofline fraction at the
    algorithmic 24 B per cell update (+16 B per eps variable of the
    variable-coefficient operators);
  * CPU: the reference itself (oracle/_ref/omg_golden, amdflang -O2, MPICH,
    mpiexec -n P) on the same configuration, its own mpi_wtime per cycle.

usage: configs_bench.py [--cpu-ranks P] [--no-cpu] [--only NAME ...]
prints one JSON line per configuration and a table."""
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
from tests import mgdriver as D  # noqa: E402  (problem set-up shared with the parity tests)

T = omg.tree

# name: (omg_golden args with n_its = GPU timed cycles, CPU cycles, description)
CONFIGS = {
    "C1": ("8 64 64 64 20 v gs lpl 0 sol sol 1 lb 0", 5,
           "test_uniform_grid 3D Laplacian 64^3, box 8, lexicographic GS, Dirichlet u"),
    "C1-gsrb": ("8 64 64 64 20 v gsrb lpl 0 sol sol 1 lb 0", 5, "C1 with GSRB"),
    "C2": ("16 256 256 256 10 v gsrb lpl 0 d0 sol 1 lb 0", 3,
           "3D Poisson 256^3, box 16, Dirichlet 0, GSRB"),
    "C3": ("16 512 512 512 10 v gsrb lpl 0 per sol 1 lb 0", 1,
           "3D Poisson 512^3, box 16, periodic, GSRB (bench.py's workload)"),
    "C2-gs": ("16 256 256 256 10 v gs lpl 0 d0 sol 1 lb 0", 3,
              "C2 with the tests' default lexicographic GS"),
    "perf-gs": ("16 512 512 512 5 v gs lpl 0 d0 one 1 lbp 0", 1,
                "tests/test_performance as shipped at 512^3: lexicographic GS, rhs = 1, Dirichlet 0, "
                "mg_load_balance_parents"),
    "C4": ("16 128 128 128 10 v gsrb lpl 0 sol sol 2 lb 0", 3,
           "one-level-refined octree, 128^3 base, box 16, Dirichlet u, GSRB"),
    "C5-helm": ("16 256 256 256 10 v gsrb helm 10 d0 sol 1 lb 0", 3,
                "3D Helmholtz lambda=10, 256^3, box 16, Dirichlet 0, GSRB"),
    "C5-vlpl": ("16 256 256 256 10 v gsrb vlpl 0 d0 sol 1 lb 0", 3,
                "variable-coefficient Laplacian (m_vlaplacian), 256^3, box 16"),
    "C5-ahelm": ("16 256 256 256 10 v gsrb ahelm 10 d0 sol 1 lb 0", 0,
                 "anisotropic Helmholtz (m_ahelmholtz, smoother index fixed), 256^3, box 16; "
                 "the reference's 3D smoother is broken (SURVEY §8 a6): no CPU time"),
}
HBM = 8000.0


def leaf_cells(tree):
    n = 0
    for lvl in range(1, tree.highest_lvl + 1):
        n += len(tree.lvls[lvl].leaves) * tree.box_size_lvl[lvl] ** 3
    return n


def gpu_run(args, warmup=2):
    cfg = D.parse(args)
    be = D.DeviceBackend(cfg)
    D.setup_problem(be)
    mg = be.mg

    def cycle():
        if cfg["cycle"] == "f":
            omg.mg_fas_fmg(mg, True)
        else:
            omg.mg_fas_vcycle(mg)
    for _ in range(warmup):
        cycle()
    mg.ctx.call("synchronize")
    t0 = time.perf_counter()
    for _ in range(cfg["n_its"]):
        cycle()
    mg.ctx.call("synchronize")
    dt = (time.perf_counter() - t0) / cfg["n_its"]
    # one profiled cycle: the finest-level smoother's launches
    mg.ctx.call("reset_stats")
    mg.ctx.call("set_profiling", 1)
    cycle()
    mg.ctx.call("set_profiling", 0)
    hi = mg.highest_lvl
    roof = None
    # algorithmic bytes per cell update: phi read + write and rhs (24 B), plus
    # every eps variable in full (both colours) per red-black substep, i.e.
    # 16 B per variable per update (vlaplacian / vhelmholtz 1, ahelmholtz 3)
    n_eps = {"vlpl": 1, "vhelm": 1, "ahelm": 3}.get(cfg["op"], 0)
    for fam, bpu in (("smoother_gsrb", 24.0 + 16.0 * n_eps), ("smoother_gs", 24.0 + 8.0 * n_eps)):
        n, ms, upd = mg.ctx.kernel_stats(f"{fam}@{hi}")
        if n and ms > 0:
            # cells counts the updates of the launch (half a level per RB substep)
            gbs = bpu * upd / (ms * 1e-3) / 1e9
            roof = {"kernel": fam, "launches": n, "avg_launch_us": ms * 1e3 / n, "achieved_GBs": gbs,
                    "frac": gbs / HBM}
    cells = leaf_cells(mg)
    out = {"ms_per_cycle": dt * 1e3, "cells": cells, "value": cells / dt, "roofline": roof}
    omg.mg_deallocate_storage(mg)
    return out


def cpu_run(args, n_its, ranks):
    ref = os.path.join(ROOT, "oracle", "_ref", "omg_golden")
    if not os.path.exists(ref) or n_its == 0:
        return None
    f = args.split()
    f[4] = str(n_its)
    cmd = (["/opt/conda/bin/mpiexec", "-n", str(ranks)] if ranks > 1 else []) + [ref] + f + ["x"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600).stdout
    m = re.search(r"TIME\s+(\S+)", out)
    return float(m.group(1)) if m else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-ranks", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    rows = []
    for name, (args, cpu_its, desc) in CONFIGS.items():
        if a.only and name not in a.only:
            continue
        g = gpu_run(args)
        c = None if a.no_cpu else cpu_run(args, cpu_its, a.cpu_ranks)
        line = {"config": name, "args": args, "desc": desc, "gpu": g,
                "cpu": None if c is None else {"s_per_cycle": c, "value": g["cells"] / c,
                                               "ranks": a.cpu_ranks, "kind": "reference"}}
        print(json.dumps(line), flush=True)
        rows.append(line)
    print(f"{'config':10s} {'ms/cycle':>9s} {'G cell/s':>9s} {'smoother %HBM':>14s} {'CPU s/cycle':>12s} {'GPU/CPU':>8s}")
    for r in rows:
        g, c = r["gpu"], r["cpu"]
        fr = f"{100 * g['roofline']['frac']:.1f}" if g["roofline"] else "-"
        cs = f"{c['s_per_cycle']:.4f}" if c else "-"
        sp = f"{c['s_per_cycle'] * 1e3 / g['ms_per_cycle']:.0f}x" if c else "-"
        print(f"{r['config']:10s} {g['ms_per_cycle']:9.3f} {g['value'] / 1e9:9.2f} {fr:>14s} {cs:>12s} {sp:>8s}")


if __name__ == "__main__":
    main()
