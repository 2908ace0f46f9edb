#!/usr/bin/env python3
"""Benchmark: FAS V-cycles of the 3D Poisson problem, 512^3 per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N ...     (one rank per GPU)

A "step" is one mg_fas_vcycle over the whole tree: box 16, fully periodic
(so subtract_mean runs twice per cycle), red-black Gauss-Seidel, n_cycle_down =
n_cycle_up = 2.  Weak scaling: every GPU owns a 512^3 octant (Morton chunks of
mg_load_balance); the global domain is 512^3 x (1,1,1)/(2,1,1)/(2,2,1)/(2,2,2).
Input is synthetic: u = prod(sin(2 pi 5 x)), rhs = L_h u on every level, phi0 = 0.

value = finest-level cells x V-cycles / s over all ranks (the BASELINE metric).
roofline: the red-black smoother kernel, algorithmic 12 B per level cell per
substep (24 B per cell update), timed with HIP events on the
library's stream in a separate pass, against 8 TB/s HBM3E.
cpu_baseline: the reference itself (oracle/_ref, amdflang -O2 + MPICH) on the
host cores, one V-cycle of the same 512^3 problem.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

HBM_PEAK_GBS = 8000.0
PER_GPU = 512
BOX = 16
REPLICATE_CELLS = int(os.environ.get("OMG_REPLICATE_CELLS", 64 * 16 ** 3))
# V-cycles of the reference's CPU path in the cpu_baseline sample (~0.7-0.9 s
# each at 512^3 on 8 host cores: ~10 s of CPU work)
CPU_CYCLES = 12


# every Prof name the library records (omg_api.cpp); the per-cycle breakdown
# also reports what these do not account for
KERNEL_FAMILIES = ("smoother_gsrb", "smoother_gs", "smooth_resid", "prolong_smooth", "coarse_tail",
                   "fill_gc", "resid_restrict", "residual", "restrict", "prolong_fill", "prolong",
                   "sub_parents", "coarse_rhs", "box_sums", "seq_sum", "subtract", "subtract_rhs")


def pmc_traffic():
    """HBM bytes per launch of the finest-level smoother from the newest
    committed PMC summary (tools/pmc.sh + tools/pmc_summary.py: FETCH_SIZE x2
    + WRITE_SIZE, the MI355X guide's gfx950 correction), or None."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_smoother.json")), reverse=True):
        try:
            d = json.load(open(f))
            for k, e in d["kernels"].items():
                if re.match(r"void omg::k_gsrb_tile<16, 1[,>]", k) and "hbm_bytes_per_launch" in e:
                    if e["workgroups"] == (PER_GPU // BOX) ** 3:
                        return e["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def rank_grid(n):
    return {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}.get(n, (n, 1, 1))


def setup_dist(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        return dist, dist.get_rank(), world, int(os.environ.get("LOCAL_RANK", "0"))
    return None, 0, 1, 0


def build(omg, n_ranks, dev):
    T = omg.tree
    mg = omg.MG()
    mg.operator_type = T.MG_LAPLACIAN
    mg.smoother_type = T.MG_SMOOTHER_GSRB
    omg.mg_set_methods(mg)
    omg.mg_comm_init(mg)
    domain = np.array(rank_grid(n_ranks)) * PER_GPU
    t0 = time.time()
    omg.mg_build_rectangle(mg, domain, BOX, 1.0 / domain.astype(np.float64), [0.0] * 3,
                           [True] * 3, 0)
    omg.mg_load_balance(mg)
    omg.mg_set_methods(mg)
    # coarse levels of at most 64 boxes of 16^3 live on every GPU: no
    # latency-bound exchanges below them (omg_set_coarse_replication)
    mg.coarse_replication_cells = REPLICATE_CELLS
    t1 = time.time()
    omg.mg_allocate_storage(mg, device_index=dev)
    # u on every level, rhs = L_h u, phi = 0 (tests/test_uniform_grid.f90:137-170);
    # every rank uploads every level (collective on replicated levels)
    for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
        ids = mg.lvls[lvl].my_ids
        mg.set_level(lvl, T.MG_IPHI, omg.problems.level_solution(mg, lvl, ids))
    omg.mg_apply_op(mg, T.MG_IRHS)
    for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
        n, nc = mg.ctx.level_size(lvl)
        mg.set_level(lvl, T.MG_IPHI, np.zeros((n, nc + 2, nc + 2, nc + 2)))
    mg.ctx.call("synchronize")
    return mg, domain, t1 - t0, time.time() - t1


def cpu_baseline(domain):
    """The reference's own CPU path on this host, bounded to CPU_CYCLES V-cycles."""
    ref = os.path.join(ROOT, "oracle", "_ref", "omg_golden")
    cores = min(8, os.cpu_count() or 1)
    args = [str(BOX)] + [str(int(d)) for d in domain] + \
        f"{CPU_CYCLES} v gsrb lpl 0 per sol 1 lb 0 x".split()
    if not os.path.exists(ref):
        return {"value": None, "unit": "cell-updates/s", "cores": 0, "kind": "reference",
                "sample": "unavailable: oracle/_ref not built"}
    mpiexec = "/opt/conda/bin/mpiexec"
    cmd = ([mpiexec, "-n", str(cores)] if cores > 1 and os.path.exists(mpiexec) else []) + [ref] + args
    if not cmd[0].endswith("mpiexec"):
        cores = 1
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=240).stdout
        t = float(re.search(r"TIME\s+(\S+)", out).group(1))
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "cell-updates/s", "cores": cores, "kind": "reference",
                "sample": f"failed: {e}"}
    cells = float(np.prod(domain))
    return {"value": cells / t, "unit": "cell-updates/s", "cores": cores, "kind": "reference",
            "seconds_per_vcycle": t,
            "sample": f"reference octree-mg (amdflang -O2, MPICH, {cores} ranks): {CPU_CYCLES} FAS V-cycles "
                      f"({CPU_CYCLES * t:.1f} s), "
                      f"{'x'.join(str(int(d)) for d in domain)} periodic GSRB box 16"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile-pass", action="store_true")
    a = ap.parse_args()

    dist, rank, world, local_rank = setup_dist(a.gpus)
    omg = __graft_entry__.load_package()
    import torch
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    mg, domain, t_tree, t_alloc = build(omg, world, local_rank)

    def barrier():
        mg.ctx.call("synchronize")
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist:
            dist.barrier()

    for _ in range(a.warmup):
        omg.mg_fas_vcycle(mg)
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        omg.mg_fas_vcycle(mg)
    barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])

    cells = float(np.prod(domain))
    value = cells * a.steps / dt

    roof = None
    kern = {}
    if not a.no_profile_pass:
        mg.ctx.call("reset_stats")
        mg.ctx.call("set_profiling", 1)
        barrier()
        tp = time.perf_counter()
        omg.mg_fas_vcycle(mg)
        barrier()
        tp = time.perf_counter() - tp
        mg.ctx.call("set_profiling", 0)
        hi = mg.highest_lvl
        total = 0.0
        for name in KERNEL_FAMILIES:
            n, ms, c = mg.ctx.kernel_stats(name)
            if n:
                total += ms
                n1, ms1, _ = mg.ctx.kernel_stats(f"{name}@{hi}")
                kern[name] = {"launches": n, "ms": round(ms, 4), f"launches_lvl{hi}": n1,
                              f"ms_lvl{hi}": round(ms1, 4)}
        # wall time of the profiled cycle (event pairs add a little) and what
        # the families above do not account for (launch gaps, RCCL, host
        # waits; side-stream work overlaps and can make it negative)
        kern["profiled_cycle_ms"] = round(tp * 1e3, 4)
        kern["unaccounted_ms"] = round(tp * 1e3 - total, 4)
        # dominant kernel: the red-black substep on the finest level
        n, ms, upd = mg.ctx.kernel_stats(f"smoother_gsrb@{hi}")
        if n and ms > 0:
            alg_bytes = 24.0 * upd / n          # 24 B per cell update, per launch
            dur = ms * 1e-3 / n
            achieved = alg_bytes / dur / 1e9
            traffic, tsrc = pmc_traffic()
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "kernel": f"k_gsrb_tile<16,OP_LPL> on level {hi} ({len(mg.lvls[hi].my_ids)} boxes)",
                    "launches": n, "avg_launch_us": dur * 1e6,
                    "alg_bytes_per_launch": alg_bytes,
                    "alg_bytes_rule": "24 B per cell update x (level cells / 2) per substep",
                    "traffic_source": tsrc}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(domain)

    if rank == 0:
        line = {
            "metric": "V-cycle cell-updates/s + smoother HBM GB/s vs roofline, 3D Poisson 512^3",
            "value": value,
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: u=prod(sin(10 pi x)), rhs=L_h u on every level, phi0=0",
            "config": {"workload": "C3: 3D Poisson, 512^3 per GPU, box 16, periodic, GSRB "
                                   "FAS V-cycle (n_cycle_down=up=2)",
                       "domain": [int(d) for d in domain], "box_size": BOX,
                       "levels": [mg.lowest_lvl, mg.highest_lvl],
                       "parallelism": f"domain-decomposition x{world} (RCCL halos)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "ref_unknowns_per_us": mg.n_boxes * BOX ** 3 * a.steps / dt * 1e-6,
            "kernels_one_cycle": kern,
            "setup_s": {"tree": t_tree, "alloc_and_rhs": t_alloc},
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
