#!/usr/bin/env python3
"""Micro-benchmark of the level-1 smoother at 512^3 (box 16, periodic, GSRB):
times smooth_boxes(highest_lvl, n_cycle) (or another level op, or a
whole V-cycle) in isolation, for rocprofv3 PMC
passes and kernel A/B work.  Usage: tools/sweep_bench.py [reps] [domain]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

omg = __graft_entry__.load_package()
T = omg.tree


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    which = sys.argv[3] if len(sys.argv) > 3 else "smooth"
    if which == "vcycle_nofuse":
        os.environ["OMG_NO_FUSE_UP"] = "1"
    mg = omg.MG()
    # *_gs: the lexicographic Gauss-Seidel smoother (the reference tests' default)
    mg.smoother_type = T.MG_SMOOTHER_GS if which.endswith("_gs") else T.MG_SMOOTHER_GSRB
    omg.mg_set_methods(mg)
    omg.mg_comm_init(mg)
    d = np.array([n, n, n])
    omg.mg_build_rectangle(mg, d, 16, 1.0 / d, [0.0] * 3, [True] * 3, 0)
    omg.mg_load_balance(mg)
    omg.mg_allocate_storage(mg)
    for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
        mg.set_level(lvl, T.MG_IPHI, omg.problems.level_solution(mg, lvl))
    omg.mg_apply_op(mg, T.MG_IRHS)
    omg.mg_fill_ghost_cells(mg, T.MG_IPHI)
    c = mg.ctx
    hi = mg.highest_lvl
    ops = {
        "smooth": lambda: c.call("smooth_boxes", hi, 1),
        "smooth_gs": lambda: c.call("smooth_boxes", hi, 1),
        "vcycle_gs": lambda: omg.mg_fas_vcycle(mg),
        "residual": lambda: c.call("residual_lvl", hi),
        "fill": lambda: c.call("fill_ghost_cells_lvl", hi, 1),
        "update_coarse": lambda: c.call("update_coarse", hi),
        "correct": lambda: c.call("correct_children", hi - 1),
        "vcycle": lambda: omg.mg_fas_vcycle(mg),
        "vcycle_nofuse": lambda: omg.mg_fas_vcycle(mg),
    }
    f = ops[which]
    for _ in range(3):
        f()
    c.call("synchronize")
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    c.call("synchronize")
    dt = (time.perf_counter() - t0) / reps
    cells = float(n) ** 3
    print(f"{which}: {dt*1e3:.3f} ms per call, {cells/dt/1e9:.2f} G cell/s, "
          f"{24*cells/dt/1e9:.0f} GB/s at 24 B/cell")


if __name__ == "__main__":
    main()
