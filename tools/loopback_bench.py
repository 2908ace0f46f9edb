#!/usr/bin/env python3
"""bench.py's multi-GPU set-up (weak scaling, periodic, GSRB, box 16, rank
grids of bench.rank_grid) replayed with N ranks as threads of ONE process on
GPU 0, exchanging through the loopback transport.  A rehearsal of the
orchestration the driver's multi-GPU run exercises (plans, comm stream,
collective decisions, reductions) at bench scale; timings share one GPU and
say nothing about scaling.

usage: loopback_bench.py N [per_rank_n] [cycles] [replicate_cells]"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402
import bench  # noqa: E402

omg = __graft_entry__.load_package()
T = omg.tree


def main():
    n = int(sys.argv[1])
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    cycles = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rep = int(sys.argv[4]) if len(sys.argv) > 4 else bench.REPLICATE_CELLS
    tag = int.from_bytes(os.urandom(6), "little")
    bar = threading.Barrier(n)
    res = [None] * n
    errs = []

    def worker(rank):
        try:
            mg = omg.MG()
            mg.operator_type = T.MG_LAPLACIAN
            mg.smoother_type = T.MG_SMOOTHER_GSRB
            omg.mg_set_methods(mg)
            omg.mg_comm_init(mg, omg.Loopback(tag, rank, n))
            domain = np.array(bench.rank_grid(n)) * per
            omg.mg_build_rectangle(mg, domain, 16, 1.0 / domain.astype(np.float64), [0.0] * 3, [True] * 3, 0)
            omg.mg_load_balance(mg)
            omg.mg_set_methods(mg)
            mg.coarse_replication_cells = rep
            omg.mg_allocate_storage(mg)
            for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
                ids = mg.lvls[lvl].my_ids
                mg.set_level(lvl, T.MG_IPHI, omg.problems.level_solution(mg, lvl, ids))
            omg.mg_apply_op(mg, T.MG_IRHS)
            for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
                k, nc = mg.ctx.level_size(lvl)
                mg.set_level(lvl, T.MG_IPHI, np.zeros((k, nc + 2, nc + 2, nc + 2)))
            r = omg.mg_fas_vcycle(mg, max_res=True)
            mg.ctx.call("synchronize")
            bar.wait()
            t0 = time.perf_counter()
            for _ in range(cycles):
                r = omg.mg_fas_vcycle(mg, max_res=True)
            mg.ctx.call("synchronize")
            bar.wait()
            res[rank] = (time.perf_counter() - t0, r)
            omg.mg_deallocate_storage(mg)
        except BaseException as e:  # noqa: BLE001
            errs.append((rank, e))
            bar.abort()

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(900)
    if errs:
        raise RuntimeError(errs)
    dt = max(x[0] for x in res)
    print(f"loopback ranks={n} per_rank={per}^3 grid={bench.rank_grid(n)} replicate<={rep} cells: "
          f"{dt / cycles * 1e3:.2f} ms/cycle "
          f"(all ranks on one GPU), max_res={res[0][1]:.6e}, same on all ranks: "
          f"{len(set(x[1] for x in res)) == 1}")


if __name__ == "__main__":
    main()
