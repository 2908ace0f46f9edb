#!/usr/bin/env python3
"""RCCL transport rehearsal on ONE GPU: N processes (gloo for the host-side
collectives), every rank's context on device 0, halos over a real RCCL
communicator (omg_get_unique_id / ncclCommInitRank), replaying golden runs
the reference made at N MPI ranks.  RCCL may refuse two ranks on one device
("Duplicate GPU detected"); the probe reports that as its result.

usage: rccl_probe.py N name [name ...]      (prints one JSON line per config)"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(n, names):
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), str(n)] + names, env=env))
    rc = 0
    for p in procs:
        try:
            r = p.wait(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            r = 124
        rc = rc or r
    return rc


def rank_main(names):
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import torch
    from tests import mgdriver as D
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["configs"]

    def reduce(e, r):
        t = torch.tensor([e, r], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0]), float(t[1])

    for name in names:
        e = golden[name]
        out = {"config": name, "ranks": world}
        try:
            res = D.run_problem(e["args"], backend="device", reduce=reduce)
            be = res["backend"]
            out["transport"] = be.mg.ctx.comm_info()
            out["history_match"] = res["history"] == e["runs"][str(world)]["history"]
            D.omg.mg_deallocate_storage(be.mg)
        except Exception as ex:  # noqa: BLE001
            out["error"] = f"{type(ex).__name__}: {ex}"[:400]
        if rank == 0:
            print(json.dumps(out), flush=True)
        if "error" in out:
            break
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1])
    names = sys.argv[2:]
    if "WORLD_SIZE" not in os.environ:
        sys.exit(launch(n, names))
    rank_main(names)
