#!/usr/bin/env python3
"""Where two builds / switches of the GS smoothing differ: the same problem on
two device contexts (default and OMG_NO_GS_DBL=1), smooth_boxes(hi, n) on
both, then the first differing stored cells of phi with their (box, i, j, k)
and the box's face kinds.   usage: diag_gsdbl.py "<omg_golden args>" n_cycle"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.mgdriver import DeviceBackend, OracleBackend, parse, setup_problem  # noqa: E402
from tests.test_gpu_parity import _stored_mask  # noqa: E402

SWITCHES = ("OMG_NO_GS_DBL", "OMG_NO_FILL_XL", "OMG_GS_LEX_PLANE", "OMG_NO_GS_PLANE")


def run(args, n_cycle, env, oracle=False):
    for k in SWITCHES:
        os.environ.pop(k, None)
    os.environ.update(env)
    be = (OracleBackend if oracle else DeviceBackend)(parse(args))
    setup_problem(be)
    hi = be.tree.highest_lvl
    if oracle:
        be.o.smooth_boxes(hi, n_cycle)
    else:
        be.mg.ctx.call("smooth_boxes", hi, n_cycle)
    return be, be.get_level(hi, 1)


def report(be, a, b, what):
    m = _stored_mask(be.tree.box_size_lvl[be.tree.highest_lvl])
    d = (a != b) & m[None]
    print(what, "differing stored cells:", int(d.sum()), "of", int(m.sum()) * a.shape[0])
    ids = be.my_ids(be.tree.highest_lvl)
    for q in np.argwhere(d)[:12]:
        bx, k, j, i = (int(x) for x in q)
        nbs = be.tree.neighbors[ids[bx], :]
        print(f"  box {bx} id {ids[bx]} (i,j,k)=({i},{j},{k}) {a[bx,k,j,i]!r} vs {b[bx,k,j,i]!r} nbrs {list(nbs)}")


def main():
    args, n = sys.argv[1], int(sys.argv[2])
    ob, o = run(args, n, {}, oracle=True)
    for env in ({}, {"OMG_NO_GS_DBL": "1"}, {"OMG_NO_FILL_XL": "1"}, {"OMG_GS_LEX_PLANE": "1"},
                {"OMG_NO_GS_PLANE": "1"}):
        be, a = run(args, n, env)
        report(be, a, o, f"device {env or 'default'} vs oracle:")


if __name__ == "__main__":
    main()
