"""Diagnose the reverted one-wave coarse tail (round 4, commit 4aa12c0,
OMG_TAIL_WAVE=1), which failed
test_free_space_multirank_matches_reference[free128_box16_f-4].

Runs a configuration through the library named by OMG_LIB (a build of that
commit) with R loopback ranks, one free-space FMG step (or a V-cycle for an
omg_golden argument string) and writes every level's phi, rhs, old and res
of rank 0 to an .npz, so that a run with OMG_TAIL_WAVE=1 and one without can
be compared level by level (tools/tailwave_cmp.py).

    python tools/tailwave_diag.py <out.npz> <ranks> [free|golden] [args...]
"""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, ranks = sys.argv[1], int(sys.argv[2])
    kind = sys.argv[3] if len(sys.argv) > 3 else "free"
    args = " ".join(sys.argv[4:]) if len(sys.argv) > 4 else "16 128 128 128 3 0.15 f"
    if kind == "free":
        from tests import freedriver as FD
        omg, T = FD.omg, FD.T
        cfg = FD.parse(args)
    else:
        from tests import mgdriver as D
        omg, T = D.omg, D.T
        cfg = D.parse(args)
    tag = int.from_bytes(os.urandom(6), "little")
    res = [None] * ranks
    errs = []

    def worker(rank):
        try:
            comm = omg.Loopback(tag, rank, ranks) if ranks > 1 else None
            if kind == "free":
                d = FD._Device(cfg, comm)
                mg = d.mg
                m = d.step(cfg, 1)
            else:
                be = D.DeviceBackend(cfg, comm)
                D.setup_problem(be)
                mg = be.mg
                m = omg.mg_fas_vcycle(mg, max_res=True)
            mg.ctx.call("synchronize")
            data = {"max_res": np.array([m])}
            for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
                n, nc = mg.ctx.level_size(lvl)
                if not n:
                    continue
                for iv, nm in ((1, "phi"), (2, "rhs"), (3, "old"), (4, "res")):
                    data[f"{nm}@{lvl}"] = mg.get_level(lvl, iv)
            res[rank] = data
            omg.mg_deallocate_storage(mg)
        except BaseException as ex:  # noqa: BLE001
            errs.append((rank, ex))

    th = [threading.Thread(target=worker, args=(r,)) for r in range(ranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    if errs:
        raise RuntimeError(errs)
    np.savez(out, **res[0])
    print(out, "max_res", float(res[0]["max_res"][0]))


if __name__ == "__main__":
    main()
