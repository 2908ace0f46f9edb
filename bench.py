#!/usr/bin/env python3
"""Benchmark: FAS V-cycles of the 3D Poisson problem.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode weak|strong|weak256]
    torchrun --nproc-per-node N ... bench.py --gpus N ...      (one rank per GPU)

With --gpus N > 1 and no torchrun environment (WORLD_SIZE unset) the script
launches its N ranks itself: N child processes (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, one GPU each) started before this process touches
the GPU; rank 0 prints the line.

A "step" is one mg_fas_vcycle over the whole tree: box 16, fully periodic
(so subtract_mean runs twice per cycle), red-black Gauss-Seidel, n_cycle_down
= n_cycle_up = 2.  Input is synthetic: u = prod(sin(2 pi 5 x)), rhs = L_h u on
every level, phi0 = 0.  Partition: mg_load_balance's Morton chunks, one rank
per GPU, halos over RCCL (ncclSend/ncclRecv).

Modes (the domain for N ranks):
  weak     (default) 512^3 per GPU: 512^3 x (1,1,1)/(2,1,1)/(2,2,1)/(2,2,2);
           N = 1 is BASELINE's C3 workload on one GPU
  strong   512^3 in total over the N GPUs (C3 exactly, "512^3, 8xMI355X")
  weak256  SURVEY §8(d)'s weak curve: 256^3 per GPU, 512^3 at N = 8
With N > 1 in weak mode the line also carries "c3_strong": the 512^3 problem
split over the same N GPUs, timed the same way.  Every line carries
"c4_refined": the one-level-refined octree of BASELINE's C4 (test_refinement,
128^3 base, box 16, n_levels 2) split over the N ranks.  On one GPU it also
carries "gs_lex": C2 (256^3) with the reference tests' default smoother,
lexicographic GS, and that sweep's fraction of 8 TB/s.

value = finest-level cells x V-cycles / s over all ranks (the BASELINE metric).
roofline: the red-black smoother kernel on the finest level, algorithmic 12 B
per level cell per substep (24 B per cell update), timed with
HIP events on the library's stream in a separate profiled cycle, against
8 TB/s HBM3E; traffic from the committed rocprofv3 PMC summary.  On C3's
periodic finest level the kernel is k_gsrb3 in its correct_children form
(omg_block.hip: the up-smoothing's correction + three substeps per pass, one
per cycle, the level's longest kernel; the down-smoothing is one k_gsrb4 pass
of four substeps): the same rule over its 1.5 cell updates per level cell, and
beside it the pass's own minimum HBM bytes (phi of one colour and rhs in,
phi and the ghost faces out, the coarse res in: 21 B per cell + 12 KiB per box).
cpu_baseline: the reference itself (oracle/_ref, amdflang -O2 + MPICH) on the
host cores of this box at P = 1, 8 and the job's CPU share (rank 0, N = 1).
parity: before anything is timed, the N ranks run C3 itself (512^3 in total,
the strong tree, with the timed run's coarse replication) for the 3 V-cycles
the reference ran at the same rank count (tests/golden/golden.json
c3_per512_box16, runs 1/2/4/8) and compare the printed history (max |phi - u|,
max |res| over the leaves, reduced over ranks) bit for bit; a mismatch prints
the line with "parity": {"ok": false} and no value, and exits 3.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import signal
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

HBM_PEAK_GBS = 8000.0
BOX = 16
REPLICATE_CELLS = int(os.environ.get("OMG_REPLICATE_CELLS", 64 * 16 ** 3))
C4_ARGS = "16 128 128 128 10 v gsrb lpl 0 sol sol 2 lb 0"   # omg_golden / tests.mgdriver form
GS_ARGS = "16 256 256 256 10 v gs lpl 0 d0 sol 1 lb 0"      # C2 with lexicographic GS
METRIC = "V-cycle cell-updates/s + smoother HBM GB/s vs roofline, 3D Poisson 512^3"

# every Prof name the library records (omg_api.cpp); the per-cycle breakdown
# also reports what these do not account for
KERNEL_FAMILIES = ("smoother_gsrb", "smoother_gsrb3", "smoother_gsrb3p", "smoother_gsrb3r", "smoother_gsrb4",
                   "smoother_gsrb4p", "smoother_gs", "smooth_resid", "prolong_smooth", "coarse_tail",
                   "fill_gc", "resid_restrict", "residual", "restrict", "prolong_fill", "prolong",
                   "sub_parents", "coarse_rhs", "box_sums", "seq_sum", "subtract", "subtract_rhs")
COMM_FAMILIES = ("comm", "comm_overlap")
# the deep-halo rounds of split levels (pack + exchange + unpack, omg_api.cpp
# deep_before / deep_after): reported beside the exchanges, not summed
DEEP_FAMILIES = ("deep_phi", "deep_rhs", "deep_faces")


# the multi-substep passes (omg_block.hip) by Prof name: kernel, cell updates
# per level cell, PMC row, the pass's own minimum bytes per level cell (phi of
# one colour and rhs in, phi out; + the coarse res for the correction form),
# beside 12 KiB of ghost faces per box
PASSES = {
    "smoother_gsrb4": ("k_gsrb4<OP_LPL, 0> (the down-smoothing: four red-black substeps per pass)", 2.0,
                       r"void omg::k_gsrb4<1(, 0)?(, false)?>", 20.0),
    "smoother_gsrb4p": ("k_gsrb4<OP_LPL, 2> (the up-smoothing: correction + four substeps per pass)", 2.0,
                        r"void omg::k_gsrb4<1, 2(, false)?>", 21.0),
    "smoother_gsrb3p": ("k_gsrb3<OP_LPL, 2, false> (the up-smoothing: correction + three substeps per pass)", 1.5,
                        r"void omg::k_gsrb3<1, 2, false(, false)?>", 21.0),
    "smoother_gsrb3": ("k_gsrb3<OP_LPL, 0, false> (three red-black substeps per pass)", 1.5,
                       r"void omg::k_gsrb3<1, 0, false(, false)?>", 20.0),
}


PARITY_CONFIG = "c3_per512_box16"
PARITY_EXIT = 3


def parity_verdict(history, golden_history):
    """Bitwise comparison of a run's history with the reference's: ok, and the
    first differing iteration (or None)."""
    first = next((i for i, (a, b) in enumerate(zip(history, golden_history)) if a != b), None)
    if first is None and len(history) != len(golden_history):
        first = min(len(history), len(golden_history))
    return {"ok": first is None, "first_mismatch": first}


def c3_parity(dist, world):
    """C3 (512^3 in total over the N ranks, the strong tree) for the reference's
    3 V-cycles on this rank's GPU, its history against the reference's own run
    at N MPI ranks (golden c3_per512_box16).  The history is omg_golden's
    print_state (tests/mgdriver.py measure: max |phi - u| and max |res| over the
    leaves, each reduced by max over ranks, m_multigrid.f90:150-243's cycle in
    between).  No golden at this N: ok None."""
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["configs"][PARITY_CONFIG]
    run = golden["runs"].get(str(world))
    if run is None:
        return {"ok": None, "config": PARITY_CONFIG, "reason": f"no reference run at {world} ranks"}
    from tests import mgdriver as D   # the golden driver's problem set-up and print_state (device backend)
    import torch

    def reduce(e, r):
        if not dist:
            return e, r
        t = torch.tensor([e, r], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0]), float(t[1])

    t0 = time.time()
    cfg = D.parse(golden["args"])
    be = D.DeviceBackend(cfg, None, REPLICATE_CELLS)
    D.setup_problem(be)
    hist = D._cycles(be, cfg, reduce)
    be.mg.ctx.call("synchronize")
    omg_pkg = __graft_entry__.load_package()
    omg_pkg.mg_deallocate_storage(be.mg)
    if os.environ.get("OMG_BENCH_PARITY_CORRUPT"):   # (tests: the mismatch path)
        hist[-1] = dict(hist[-1], res="%016X" % (int(hist[-1]["res"], 16) ^ 1))
    out = parity_verdict(hist, run["history"])
    out.update({"config": PARITY_CONFIG, "ranks": world, "vcycles": cfg["n_its"], "seconds": round(time.time() - t0, 1),
                "checked": "history (max |phi-u|, max |res|, per V-cycle) bit for bit vs the reference's run at "
                           f"{world} MPI ranks"})
    return out


def pmc_traffic(per_gpu_cells, block3_pat=None):
    """HBM bytes per launch of the finest-level smoother from the newest
    committed PMC summary (tools/pmc.sh + tools/pmc_summary.py: FETCH_SIZE x2
    + WRITE_SIZE, the MI355X guide's gfx950 correction), or None.  block3:
    k_gsrb3 / k_gsrb4 (one workgroup per column of 2 x 16 boxes on C3's level
    1; their loads are 8 B per lane, for which the x2 holds exactly as for the
    guide's 16-B loads: profiles/r06/fetch_calib.txt)."""
    import glob
    block3 = block3_pat is not None
    name, pat = ("pmc_block3.json", block3_pat) if block3 else \
        ("pmc_smoother.json", r"void omg::k_gsrb_tile<16, 1[,>]")
    # (k_gsrb3: the finest level's launch is the one with the most workgroups,
    # one per column of boxes, whatever the column length)
    wgs = per_gpu_cells // BOX ** 3
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)), reverse=True):
        try:
            d = json.load(open(f))
            hits = [e for k, e in d["kernels"].items() if re.match(pat, k) and "hbm_bytes_per_launch" in e]
            if block3 and hits:
                e = max(hits, key=lambda e: e["workgroups"])
                return e["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
            for e in hits:
                if e["workgroups"] == wgs:
                    return e["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def rank_grid(n):
    return {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}.get(n, (n, 1, 1))


def domain_for(mode, world):
    if mode == "strong":
        return np.array([512, 512, 512])
    per = 256 if mode == "weak256" else 512
    return np.array(rank_grid(world)) * per


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(n):
    """N ranks of this script, one per GPU, started before any GPU call in
    this process (nothing here initialises HIP); returns the worst exit code."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                r = p.poll()
                if r is None:
                    continue
                procs.remove(p)
                if r != 0:
                    rc = rc or r
                    for q in procs:   # one rank failed: the others would wait for it forever
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            p.kill()
    return rc


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        return dist, dist.get_rank(), world, int(os.environ.get("LOCAL_RANK", "0"))
    return None, 0, 1, 0


def build(omg, domain, dev):
    """C3's tree over `domain` on this rank's GPU, u / rhs = L_h u on every
    level, phi = 0 (tests/test_uniform_grid.f90:137-170)."""
    T = omg.tree
    mg = omg.MG()
    mg.operator_type = T.MG_LAPLACIAN
    mg.smoother_type = T.MG_SMOOTHER_GSRB
    omg.mg_set_methods(mg)
    omg.mg_comm_init(mg)
    t0 = time.time()
    omg.mg_build_rectangle(mg, domain, BOX, 1.0 / domain.astype(np.float64), [0.0] * 3, [True] * 3, 0)
    omg.mg_load_balance(mg)
    omg.mg_set_methods(mg)
    # coarse levels of at most 64 boxes of 16^3 live on every GPU: no
    # latency-bound exchanges below them (omg_set_coarse_replication)
    mg.coarse_replication_cells = REPLICATE_CELLS
    t1 = time.time()
    omg.mg_allocate_storage(mg, device_index=dev)
    # every rank uploads every level (collective on replicated levels)
    for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
        ids = mg.lvls[lvl].my_ids
        mg.set_level(lvl, T.MG_IPHI, omg.problems.level_solution(mg, lvl, ids))
    omg.mg_apply_op(mg, T.MG_IRHS)
    for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
        n, nc = mg.ctx.level_size(lvl)
        mg.set_level(lvl, T.MG_IPHI, np.zeros((n, nc + 2, nc + 2, nc + 2)))
    mg.ctx.call("synchronize")
    return mg, t1 - t0, time.time() - t1


class Timer:
    """Barrier + device synchronisation on both sides, max over ranks."""

    def __init__(self, dist, ctx):
        import torch
        self.torch, self.dist, self.ctx = torch, dist, ctx

    def barrier(self):
        self.ctx.call("synchronize")
        if self.torch.cuda.is_available():
            self.torch.cuda.synchronize()
        if self.dist:
            self.dist.barrier()

    def max_over_ranks(self, dt):
        if not self.dist:
            return dt
        t = self.torch.tensor([dt], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def time(self, fn, steps, warmup):
        for _ in range(warmup):
            fn()
        self.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        self.barrier()
        return self.max_over_ranks(time.perf_counter() - t0)


def gather(dist, obj):
    if not dist:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def profile_cycle(omg, mg, timer, cycle):
    """One cycle with HIP events around every kernel family and comm round:
    per-family totals (and on the finest level), the finest-level smoother's
    launches, and this rank's exchange time."""
    mg.ctx.call("reset_stats")
    mg.ctx.call("set_profiling", 1)
    timer.barrier()
    tp = time.perf_counter()
    cycle()
    timer.barrier()
    tp = time.perf_counter() - tp
    mg.ctx.call("set_profiling", 0)
    hi = mg.highest_lvl
    total = 0.0
    kern = {}
    for name in KERNEL_FAMILIES:
        n, ms, c = mg.ctx.kernel_stats(name)
        if n:
            total += ms
            n1, ms1, _ = mg.ctx.kernel_stats(f"{name}@{hi}")
            kern[name] = {"launches": n, "ms": round(ms, 4), f"launches_lvl{hi}": n1, f"ms_lvl{hi}": round(ms1, 4)}
    comm = {}
    for name in COMM_FAMILIES + DEEP_FAMILIES:
        n, ms, doubles = mg.ctx.kernel_stats(name)
        if n:
            comm[name] = {"rounds": n, "ms": round(ms, 4), "MB_received": round(8e-6 * doubles, 3)}
    # wall time of the profiled cycle (event pairs add a little) and what
    # the families above do not account for (launch gaps, RCCL, host waits;
    # side-stream work overlaps and can make it negative)
    kern["profiled_cycle_ms"] = round(tp * 1e3, 4)
    kern["unaccounted_ms"] = round(tp * 1e3 - total - comm.get("comm", {}).get("ms", 0.0), 4)
    # the finest level's red-black smoother: its longest multi-substep pass
    # where they run (C3: the down-smoothing's k_gsrb4 and the up-smoothing's
    # k_gsrb3 in its correct_children form, within a few percent of each
    # other), else the one-substep kernel
    best = None
    for fam in PASSES:
        st = mg.ctx.kernel_stats(f"{fam}@{hi}")
        if st[0] and (best is None or st[1] / st[0] > best[2] / best[1]):
            best = (fam,) + tuple(st)
    smoother = best or ("smoother_gsrb",) + tuple(mg.ctx.kernel_stats(f"smoother_gsrb@{hi}"))
    return kern, comm, smoother


def roofline(smoother, per_gpu_cells, boxes_hi, hi):
    fam, n, ms, upd = smoother
    if not (n and ms > 0):
        return None
    kname, ups, pmc_pat, min_b = PASSES.get(fam, (None, None, None, None))
    block3 = kname is not None
    alg_bytes = 24.0 * upd / n          # 24 B per cell update, per launch
    dur = ms * 1e-3 / n
    achieved = alg_bytes / dur / 1e9
    traffic, tsrc = pmc_traffic(per_gpu_cells, pmc_pat)
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
           "kernel": (f"{kname} on level {hi} ({boxes_hi} boxes)" if block3
                      else f"k_gsrb_tile<16,OP_LPL> on level {hi} ({boxes_hi} boxes)"),
           "launches": n, "avg_launch_us": dur * 1e6,
           "alg_bytes_per_launch": alg_bytes,
           "alg_bytes_rule": "24 B per cell update x (level cells / 2) per substep" +
                             (f", {int(round(2 * ups))} substeps per launch" if block3 else ""),
           "traffic_source": tsrc}
    if block3:
        cells = upd / n / ups
        own = min_b * cells + 6 * BOX * BOX * 8 * boxes_hi
        out["pass_min_bytes_per_launch"] = own
        out["pass_min_frac"] = own / dur / 1e9 / HBM_PEAK_GBS
    return out


def run_c3(omg, domain, dist, rank, world, dev, steps, warmup, profile=True):
    mg, t_tree, t_alloc = build(omg, domain, dev)
    timer = Timer(dist, mg.ctx)
    dt = timer.time(lambda: omg.mg_fas_vcycle(mg), steps, warmup)
    cells = float(np.prod(domain))
    out = {"value": cells * steps / dt, "ms_per_step": dt * 1e3 / steps, "domain": [int(d) for d in domain],
           "levels": [mg.lowest_lvl, mg.highest_lvl], "setup_s": {"tree": t_tree, "alloc_and_rhs": t_alloc},
           "ref_unknowns_per_us": mg.n_boxes * BOX ** 3 * steps / dt * 1e-6}
    n_comm, transport = mg.ctx.comm_info()
    out["comm"] = {"transport": transport, "comm_ranks": n_comm}
    if profile:
        kern, comm, smoother = profile_cycle(omg, mg, timer, lambda: omg.mg_fas_vcycle(mg))
        hi = mg.highest_lvl
        out["kernels_one_cycle"] = kern
        per_rank = gather(dist, {"rank": rank, "comm": comm, "boxes_lvl_hi": len(mg.lvls[hi].my_ids),
                                 "profiled_cycle_ms": kern["profiled_cycle_ms"]})
        out["comm"]["per_rank"] = per_rank
        out["roofline"] = roofline(smoother, int(np.prod(domain)) // world, len(mg.lvls[hi].my_ids), hi)
    omg.mg_deallocate_storage(mg)
    return out


def run_c4(omg, dist, world, steps=10, warmup=3):
    """BASELINE's C4: the one-level-refined octree (test_refinement's tree,
    128^3 base, box 16, n_levels 2), GSRB V-cycles, over the N ranks.
    Cells = leaf cells of the tree (448 x 16^3 on level 1 + 512 x 16^3 on
    level 2)."""
    from tests import mgdriver as D   # problem set-up shared with the parity tests (device backend)
    cfg = D.parse(C4_ARGS)
    be = D.DeviceBackend(cfg)
    D.setup_problem(be)
    mg = be.mg
    timer = Timer(dist, mg.ctx)
    dt = timer.time(lambda: omg.mg_fas_vcycle(mg), steps, warmup)
    cells = sum(len(mg.lvls[l].leaves) * mg.box_size_lvl[l] ** 3 for l in range(1, mg.highest_lvl + 1))
    kern, comm, _ = profile_cycle(omg, mg, timer, lambda: omg.mg_fas_vcycle(mg))
    hi = mg.highest_lvl
    n, ms, upd = mg.ctx.kernel_stats(f"smoother_gsrb@{hi}")
    fr = None
    if world == 1 and n and ms > 0:
        fr = {"avg_launch_us": ms * 1e3 / n, "achieved_GBs": 24.0 * upd / (ms * 1e-3) / 1e9,
              "frac": 24.0 * upd / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    if world == 1 and n:
        # the same launches back to back: smooth_boxes on the finest level,
        # 10 cycles = 20 substeps (one launch each, the fill fused), timed as
        # one block; a 12-us kernel timed by its own event pair reads several
        # us long (compare the kernel trace, profiles/r03/v14_trace_C4_by_grid.txt)
        k = 10
        mg.ctx.call("smooth_boxes", hi, 1)
        mg.ctx.call("synchronize")
        t0 = time.perf_counter()
        mg.ctx.call("smooth_boxes", hi, k)
        mg.ctx.call("synchronize")
        tb = (time.perf_counter() - t0) / (2 * k)
        upd1 = upd / n
        fr["back_to_back"] = {"launches": 2 * k, "avg_launch_us": tb * 1e6,
                              "achieved_GBs": 24.0 * upd1 / tb / 1e9,
                              "frac": 24.0 * upd1 / tb / 1e9 / HBM_PEAK_GBS}
    out = {"workload": "C4: test_refinement 2 16 128 128 128 (one refined level, box 16), GSRB, "
                       "callback Dirichlet u",
           "value": cells * steps / dt, "unit": "cell-updates/s (leaf cells)", "ms_per_step": dt * 1e3 / steps,
           "leaf_cells": cells, "steps": steps, "warmup": warmup, "smoother_lvl2": fr,
           "kernels_one_cycle": {k: v for k, v in kern.items() if k in ("profiled_cycle_ms", "smoother_gsrb")}}
    omg.mg_deallocate_storage(mg)
    return out


def run_gs(omg, dist, world, steps=10, warmup=3):
    """C2 with the reference tests' default smoother, lexicographic GS
    ("C2-gs": 256^3, box 16, Dirichlet, n_cycle 2+2), one GPU:
    its cell-updates/s and the finest-level sweep against 8 TB/s (24 B per
    cell per sweep: phi in, phi out, rhs)."""
    from tests import mgdriver as D
    cfg = D.parse(GS_ARGS)
    be = D.DeviceBackend(cfg)
    D.setup_problem(be)
    mg = be.mg
    timer = Timer(dist, mg.ctx)
    dt = timer.time(lambda: omg.mg_fas_vcycle(mg), steps, warmup)
    hi = mg.highest_lvl
    cells = float(len(mg.lvls[hi].leaves)) * mg.box_size_lvl[hi] ** 3
    profile_cycle(omg, mg, timer, lambda: omg.mg_fas_vcycle(mg))
    n, ms, upd = mg.ctx.kernel_stats(f"smoother_gs@{hi}")
    fr = None
    if n and ms > 0:
        fr = {"kernel": "k_gs_lex_reg (register-ring lexicographic GS)", "launches": n,
              "avg_launch_us": ms * 1e3 / n, "achieved_GBs": 24.0 * upd / (ms * 1e-3) / 1e9,
              "frac": 24.0 * upd / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    out = {"workload": "C2-gs: 256^3, box 16, Dirichlet, lexicographic GS V-cycle (n_cycle_down=up=2)",
           "value": cells * steps / dt, "unit": "cell-updates/s", "ms_per_step": dt * 1e3 / steps,
           "steps": steps, "warmup": warmup, "smoother_lvl_hi": fr}
    omg.mg_deallocate_storage(mg)
    return out


def host_cores():
    """Physical cores of the host (lscpu), and the CPUs this job may use."""
    phys = None
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
        phys = len({ln for ln in out.splitlines() if ln and not ln.startswith("#")})
    except Exception:  # noqa: BLE001
        pass
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    # the GPU box gives one GPU's job a share of 16 CPUs (OMP_NUM_THREADS)
    share = min(share, int(os.environ.get("OMP_NUM_THREADS", share) or share))
    return phys, os.cpu_count(), share


def run_group(cmd, timeout):
    """Run cmd in a session of its own and return its stdout; on exit or
    timeout every process left in that session's group is killed, so nothing
    (MPICH's hydra proxies, ranks) outlives the call.  Raises
    subprocess.TimeoutExpired / CalledProcessError like subprocess.run."""
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        _kill_group(p.pid)
        p.communicate()
        raise
    finally:
        _kill_group(p.pid)
    if p.returncode != 0:
        raise subprocess.CalledProcessError(p.returncode, cmd, out, err)
    return out


def _kill_group(pgid):
    try:
        os.killpg(pgid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError):
        pass


def cpu_baseline(domain, ref=None, timeout=180, plan=None):
    """The reference's own CPU path (oracle/_ref/omg_golden, amdflang -O2 +
    MPICH, mpiexec -n P, its mpi_wtime around the cycles) on this host:
    P = 1 (one run of 1 V-cycle), P = 8 and P = the job's CPU share (min of 3
    runs of 2 V-cycles each).  value = the best P measured (normally the job's
    CPU share), with every P kept in by_ranks."""
    ref = ref or os.path.join(ROOT, "oracle", "_ref", "omg_golden")
    phys, logical, share = host_cores()
    if not os.path.exists(ref):
        return {"value": None, "unit": "cell-updates/s", "cores": 0, "kind": "reference",
                "sample": "unavailable: oracle/_ref not built"}
    mpiexec = "/opt/conda/bin/mpiexec"
    cells = float(np.prod(domain))
    runs = {}
    plan = plan or [(1, 1, 1), (8, 2, 3)] + ([(share, 2, 3)] if share not in (1, 8) else [])
    for p, cycles, repeat in plan:
        args = [str(BOX)] + [str(int(d)) for d in domain] + f"{cycles} v gsrb lpl 0 per sol 1 lb 0 x".split()
        cmd = ([mpiexec, "-n", str(p)] if p > 1 else []) + [ref] + args
        ts = []
        for _ in range(repeat):
            try:
                out = run_group(cmd, timeout)
                ts.append(float(re.search(r"TIME\s+(\S+)", out).group(1)))
            except Exception as e:  # noqa: BLE001
                runs[str(p)] = {"error": f"{type(e).__name__}: {e}"[:200]}
                break
        if ts:
            t = min(ts)
            runs[str(p)] = {"seconds_per_vcycle": t, "value": cells / t, "runs": len(ts),
                            "vcycles_per_run": cycles}
    done = [(int(p), r) for p, r in runs.items() if r.get("value")]
    best_p, head = max(done, key=lambda x: x[1]["value"]) if done else (0, {})
    return {"value": head.get("value"), "unit": "cell-updates/s", "cores": best_p, "kind": "reference",
            "ranks": best_p, "seconds_per_vcycle": head.get("seconds_per_vcycle"),
            "host_physical_cores": phys, "host_logical_cpus": logical, "job_cpu_share": share,
            "by_ranks": runs,
            "sample": f"reference octree-mg (amdflang -O2, MPICH), mpiexec -n P, P in "
                      f"{[p for p, _, _ in plan]} (one rank per CPU of the job's share of {share}): "
                      f"{'x'.join(str(int(d)) for d in domain)} periodic GSRB box 16, its own mpi_wtime "
                      f"per V-cycle; value = the best P (P = {best_p}), min of 3 runs of 2 V-cycles"}


def plan_check(omg, domain, dist, rank, world):
    """--plan-only (CPU, no GPU): this rank's plan-only context
    (OMG_DEVICE_NONE) of the bench's tree, and the check that every transfer
    pairs up with its peer's, key for key in wire order (the contract
    sort_and_transfer_buffers relies on, src/m_communication.f90:37-66)."""
    T = omg.tree
    tree = T.MGTree()
    tree.n_cpu, tree.my_rank = world, rank
    tree.build_rectangle(domain, BOX, 1.0 / domain.astype(np.float64), [0.0] * 3, [True] * 3, 0)
    tree.load_balance()
    ctx = omg.device.Context(-2, rank, world)
    ctx.call("set_coarse_replication", REPLICATE_CELLS)
    arrs = omg.mg._tree_arrays(tree)
    ctx.call("tree_setup", tree.n_boxes, *arrs[:6], tree.lowest_lvl, tree.highest_lvl,
             tree.first_normal_lvl, tree.box_size, arrs[6], arrs[7], arrs[8], arrs[9], 4)
    mine = {(lvl, w, d): ctx.plan_transfer(lvl, w, d)
            for lvl in range(tree.lowest_lvl, tree.highest_lvl + 1) for w in range(5) for d in (0, 1)}
    ctx.close()
    allp = gather(dist, mine)
    problems = []
    for (lvl, w, d), (items, _) in mine.items():
        if d:
            continue
        for b in range(world):
            sent = [k for p, k in items if p == b]
            expected = [k for p, k in allp[b][(lvl, w, 1)][0] if p == rank]
            if b == rank and sent:
                problems.append(f"lvl {lvl} transfer {w}: sends to itself")
            elif sent != expected:
                problems.append(f"lvl {lvl} transfer {w}: {rank}->{b} sends {len(sent)}, {b} expects {len(expected)}")
    hi = tree.highest_lvl
    return {"rank": rank, "problems": problems, "boxes_lvl_hi": len(tree.lvls[hi].my_ids),
            "halo_faces_recv_lvl_hi": len(mine[(hi, 0, 1)][0]),
            "peers_lvl_hi": sorted({p for p, _ in mine[(hi, 0, 1)][0]})}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", choices=("weak", "strong", "weak256"), default="weak")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile-pass", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the c3_strong / c4_refined sub-benchmarks")
    ap.add_argument("--no-parity", action="store_true", help="skip the C3 parity check before the timed runs")
    ap.add_argument("--plan-only", action="store_true",
                    help="CPU only: launch the ranks, build each rank's communication plan, check they pair up")
    a = ap.parse_args()

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(a.gpus))

    dist, rank, world, local_rank = setup_dist()
    omg = __graft_entry__.load_package()
    if a.plan_only:
        per_rank = gather(dist, plan_check(omg, domain_for(a.mode, world), dist, rank, world))
        if rank == 0:
            print(json.dumps({"plan_only": True, "n_ranks": world, "mode": a.mode,
                              "domain": [int(d) for d in domain_for(a.mode, world)],
                              "ok": not any(r["problems"] for r in per_rank), "ranks": per_rank}), flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    import torch
    if torch.cuda.is_available():
        # (more ranks than GPUs: they share, and the library takes its host
        # transport, octree-mg_amd/mg.py _use_host_transport)
        torch.cuda.set_device(local_rank % torch.cuda.device_count())

    parity = None if a.no_parity else c3_parity(dist, world)
    if parity and parity["ok"] is False:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "cell-updates/s", "n_gpus": world,
                              "parity": parity, "error": "C3 history differs from the reference's"}), flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        sys.exit(PARITY_EXIT)
    domain = domain_for(a.mode, world)
    main_run = run_c3(omg, domain, dist, rank, world, local_rank, a.steps, a.warmup,
                      profile=not a.no_profile_pass)
    extra = {}
    if not a.no_extra:
        if world > 1 and a.mode != "strong":
            s = run_c3(omg, domain_for("strong", world), dist, rank, world, local_rank, a.steps, a.warmup,
                       profile=not a.no_profile_pass)
            extra["c3_strong"] = {"workload": "C3: 512^3 in total over the N GPUs (strong scaling)",
                                  "value": s["value"], "ms_per_step": s["ms_per_step"], "domain": s["domain"],
                                  "steps": a.steps, "warmup": a.warmup, "roofline": s.get("roofline"),
                                  "comm": s["comm"]}
        extra["c4_refined"] = run_c4(omg, dist, world)
        if world == 1:
            extra["gs_lex"] = run_gs(omg, dist, world)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(domain)

    if rank == 0:
        desc = {"weak": "512^3 per GPU", "strong": "512^3 over the N GPUs", "weak256": "256^3 per GPU"}[a.mode]
        line = {
            "metric": METRIC,
            "value": main_run["value"],
            "unit": "cell-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": main_run["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong" if a.mode == "strong" else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: u=prod(sin(10 pi x)), rhs=L_h u on every level, phi0=0",
            "config": {"workload": f"C3: 3D Poisson, {desc}, box 16, periodic, GSRB "
                                   "FAS V-cycle (n_cycle_down=up=2)",
                       "mode": a.mode, "domain": main_run["domain"], "box_size": BOX,
                       "levels": main_run["levels"],
                       "parallelism": f"domain-decomposition x{world} (RCCL halos)"},
            "roofline": main_run.get("roofline"),
            "cpu_baseline": cpu,
            "parity": parity,
            "comm": main_run["comm"],
            "ref_unknowns_per_us": main_run["ref_unknowns_per_us"],
            "kernels_one_cycle": main_run.get("kernels_one_cycle"),
            "setup_s": main_run["setup_s"],
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
