#!/usr/bin/env python3
"""Generate the free-space golden vectors: tests/golden/free_golden.json and
the phi fixtures tests/golden/free_*_phi.npy.

Runs the REFERENCE m_free_space itself (src/m_free_space.f90 with its bundled
BigDFT PSolver, poisson_3d_fft/, compiled from /root/reference by
`make -C oracle ref`, amdflang -O2 + MPICH) through oracle/omg_free_golden,
the set-up of the reference's tests/test_free_space.f90, and records per
iteration max |phi - sol|, sqrt(mean (phi - sol)^2) and max_res as IEEE-754
bit patterns.  For the FFT-only runs (max_fft_frac >= 1: the FFT level is the
highest, no multigrid cycle) the highest level's phi, which is PSolver's
output itself, is kept as a float64 array [x, y, z].

Only numbers are committed; the reference's sources and binaries never enter
the repository.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")
MPIEXEC = "/opt/conda/bin/mpiexec"
sys.path.insert(0, os.path.join(ROOT, "octree-mg_amd"))

# name: (box nx ny nz n_its fft_frac cycle), ranks, keep phi
CONFIGS = {
    # tests/test_free_space as shipped (8 64 64 64, fft_frac 0.15, FMG)
    "free64_box8_f": ("8 64 64 64 5 0.15 f", [1, 2, 4], False),
    "free64_box8_v": ("8 64 64 64 5 0.15 v", [1], False),
    "free64_box16_f": ("16 64 64 64 4 0.15 f", [1, 2], False),
    "free128_box16_f": ("16 128 128 128 3 0.15 f", [1, 4], False),
    # anisotropic spacing (48 x 32 x 32 cells on the unit cube: the
    # kernel's general branch), ny == nz as the reference needs
    "free48x32_f": ("8 48 32 32 4 0.15 f", [1], False),
    # fft_frac so small that no level qualifies: the FFT runs on the lowest
    # level (2^3 cells)
    "free64_lowest_f": ("8 64 64 64 3 0.001 f", [1], False),
    # the FFT level is the highest: phi is PSolver's output, no cycle
    "free16_fftonly": ("8 16 16 16 1 1.0 f", [1], True),
    "free24x16_fftonly": ("8 24 16 16 1 1.0 f", [1], True),
    "free32_fftonly": ("8 32 32 32 1 1.0 f", [1, 2], False),
}


def run(args, ranks, dump):
    cmd = [os.path.join(REF, "omg_free_golden")] + args.split() + [dump or "x"]
    if ranks > 1:
        cmd = [MPIEXEC, "-n", str(ranks)] + cmd
    out = subprocess.run(cmd, capture_output=True, text=True, check=True).stdout
    its, t = [], None
    for line in out.splitlines():
        f = line.split()
        if f and f[0] == "IT":
            its.append({"it": int(f[1]), "err": f[2], "err2": f[3], "max_res": f[4]})
        elif f and f[0] == "TIME":
            t = float(f[1])
    return its, t


def highest_phi(args, raw):
    """The highest level of omg_free_golden's dump as [x, y, z]."""
    from tree import MG_SMOOTHER_GSRB, MGTree   # the host tree restatement (same ids order)
    f = args.split()
    box, dom = int(f[0]), [int(v) for v in f[1:4]]
    t = MGTree()
    t.smoother_type = MG_SMOOTHER_GSRB   # as omg_free_golden (it decides the coarsest levels)
    t.build_rectangle(dom, box, [1.0 / v for v in dom], [0, 0, 0], [False] * 3)
    off = sum(len(t.lvls[l].ids) * t.box_size_lvl[l] ** 3 for l in range(t.lowest_lvl, t.highest_lvl))
    nc = t.box_size_lvl[t.highest_lvl]
    phi = np.zeros(dom)
    for id_ in t.lvls[t.highest_lvl].ids:
        b = raw[off:off + nc ** 3].reshape(nc, nc, nc).transpose(2, 1, 0)
        off += nc ** 3
        p = (t.ix[id_] - 1) * nc
        phi[p[0]:p[0] + nc, p[1]:p[1] + nc, p[2]:p[2] + nc] = b
    return phi


def main():
    if not os.path.exists(os.path.join(REF, "omg_free_golden")):
        sys.exit("build the reference first: make -C oracle ref")
    golden = {}
    for name, (args, ranks, keep) in CONFIGS.items():
        entry = {"args": args, "runs": {}}
        for r in ranks:
            with tempfile.TemporaryDirectory() as td:
                fn = os.path.join(td, "phi.bin") if keep and r == 1 else None
                its, t = run(args, r, fn)
                entry["runs"][str(r)] = {"history": its, "ref_seconds_per_call": t}
                if fn:
                    phi = highest_phi(args, np.fromfile(fn))
                    npy = "%s_phi.npy" % name
                    np.save(os.path.join(HERE, npy), phi)
                    entry["phi_npy"] = npy
            print(name, r, its[-1], file=sys.stderr)
        golden[name] = entry
    with open(os.path.join(HERE, "free_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_free_golden.py",
                   "reference": "FermiQ/octree-mg @ 2025-06-14 m_free_space + poisson_3d_fft, "
                                "amdflang -O2, MPICH 3.3.2",
                   "configs": golden}, f, indent=1)


if __name__ == "__main__":
    main()
