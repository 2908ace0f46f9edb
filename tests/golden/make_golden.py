#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/golden.json.

Runs the REFERENCE octree-mg itself (compiled from /root/reference/src by
`make -C oracle ref`, amdflang -O2 + MPICH) through oracle/omg_golden for
every configuration below, and records per-iteration max error / max residual
/ max_res as exact IEEE-754 bit patterns, plus the sha256 of the final phi of
every box (ids order per level, lowest..highest, i fastest) where dumped.

Only the numbers are committed (tests/golden/golden.json); the reference's
sources and binaries never enter the repository.
"""
import glob
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "..", "..", "oracle", "_ref")
MPIEXEC = "/opt/conda/bin/mpiexec"

# name: (box nx ny nz n_its cycle smoother op lambda bc rhs n_levels lb maxres), dump?, ranks
# BIG: too large for the CPU oracle in the quick CPU suite (the device is
# compared with the reference's numbers directly; tests/test_gpu_parity.py)
BIG = {"c3_per512_box16", "c2_256_box16_gsrb_d0", "c2_256_box16_gs_d0", "c5_helm256_box16_gsrb_d0",
       "per256_box16_helm_v", "per256_box16_gsrb_f", "mx1_256_box16"}
CONFIGS = {
    # tests/test_uniform_grid 8 64 64 64 10 f, as shipped (GS)
    "c1_gs_v": ("8 64 64 64 10 v gs lpl 0 sol sol 1 lb 0", False, [1, 4]),
    "c1_gsrb_v": ("8 64 64 64 10 v gsrb lpl 0 sol sol 1 lb 0", False, [1]),
    "c1_gs_f": ("8 64 64 64 10 f gs lpl 0 sol sol 1 lb 0", False, [1]),
    "c1_gsrb_f_maxres": ("8 64 64 64 5 f gsrb lpl 0 sol sol 1 lb 1", False, [1, 4, 8]),
    "u32_gsrb_v": ("8 32 32 32 6 v gsrb lpl 0 sol sol 1 lb 1", True, [1]),
    "u32_gs_d0_one": ("8 32 32 32 4 v gs lpl 0 d0 one 1 lbp 1", True, [1]),
    "u64_box16_gsrb_d0_one": ("16 64 64 64 3 v gsrb lpl 0 d0 one 1 lbp 1", True, [1, 2, 8]),
    "nonsquare_gsrb": ("8 64 32 32 6 v gsrb lpl 0 sol sol 1 lb 1", True, [1]),
    "odd48_gsrb": ("8 48 48 48 4 v gsrb lpl 0 d0 sol 1 lb 0", True, [1]),
    "odd48_gs": ("8 48 48 48 4 v gs lpl 0 d0 sol 1 lb 0", True, [1]),
    # C3-like periodic GSRB (subtract_mean), rank counts pin the allreduce order
    "per32_gsrb_v": ("8 32 32 32 10 v gsrb lpl 0 per sol 1 lb 0", True, [1, 2, 3, 4, 5, 6, 8]),
    "per32_gs_f": ("8 32 32 32 5 f gs lpl 0 per sol 1 lb 1", True, [1, 4]),
    # multi-rank levels that also have boxes without a face on another rank
    # (the fused prolongation + substep runs on those, the unfused pair on the
    # others)
    "per64_gsrb_v": ("8 64 64 64 4 v gsrb lpl 0 per sol 1 lb 0", True, [1, 2, 4, 8]),
    "helm128_box16_d0": ("16 128 128 128 3 v gsrb helm 10 d0 sol 1 lb 1", True, [1, 2, 4]),
    # box-16 periodic levels with boxes both with and without a face on
    # another rank (the multi-GPU bench's level kind): the fused down-step
    # (k_smooth_resid over a box list) next to the unfused substep + residual;
    # at 6 ranks the 128x128x64 tree leaves ranks 1 and 4 with no box free of
    # remote faces, so they stay unfused while their peers fuse
    "per128_box16_gsrb_v": ("16 128 128 128 3 v gsrb lpl 0 per sol 1 lb 0", True, [1, 2, 8]),
    "per128x64_box16_mixed": ("16 128 128 64 3 v gsrb lpl 0 per sol 1 lb 0", True, [1, 6]),
    # SURVEY §8(d) C3 at the bench's own size: 512^3 per GPU, box 16,
    # periodic, GSRB (the reference takes ~40 s on one core)
    # (2, 4 and 8 ranks: the BASELINE C3 configuration on 8 GPUs, and the
    # MPICH allreduce order of get_sum at the bench's size)
    "c3_per512_box16": ("16 512 512 512 3 v gsrb lpl 0 per sol 1 lb 0", True, [1, 2, 4, 8]),
    # periodic 256^3 at box 16: the 4096-box level runs k_gsrb3 (three
    # red-black substeps per pass) at its default size bound, Helmholtz (no
    # subtract_mean) and FMG with the max residual
    "per256_box16_helm_v": ("16 256 256 256 3 v gsrb helm 10 per sol 1 lb 0", True, [1]),
    "per256_box16_gsrb_f": ("16 256 256 256 2 f gsrb lpl 0 per sol 1 lb 1", True, [1]),
    # SURVEY §8(d) C2 at its own size: 256^3, box 16, Dirichlet 0, GSRB and
    # the reference tests' lexicographic GS
    "c2_256_box16_gsrb_d0": ("16 256 256 256 3 v gsrb lpl 0 d0 sol 1 lb 0", True, [1]),
    "c2_256_box16_gs_d0": ("16 256 256 256 3 v gs lpl 0 d0 sol 1 lb 0", True, [1]),
    # C5 at its own size: Helmholtz lambda = 10, 256^3, box 16
    "c5_helm256_box16_gsrb_d0": ("16 256 256 256 3 v gsrb helm 10 d0 sol 1 lb 1", True, [1]),
    # per-face boundary types with nonzero constant values (omg_golden.f90 mx1 /
    # mx2); at box 16 on non-cubic domains the finest level takes the block
    # passes with physical faces (k_gsrb3) once their level bound is lowered
    # (tests/test_gpu_block3.py), at 256^3 at the default bound
    "mx1_box16_96x128x64": ("16 96 128 64 3 v gsrb lpl 0 mx1 sol 1 lb 0", True, [1, 2]),
    "mx2_helm_box16_128x64x96": ("16 128 64 96 3 v gsrb helm 2 mx2 sol 1 lb 0", True, [1]),
    "mx1_box8_gs": ("8 32 32 32 4 v gs lpl 0 mx1 sol 1 lb 0", True, [1]),
    "mx2_box8_gsrb_f": ("8 32 32 32 3 f gsrb lpl 0 mx2 sol 1 lb 1", True, [1]),
    "mx1_256_box16": ("16 256 256 256 3 v gsrb lpl 0 mx1 sol 1 lb 0", True, [1]),
    # C5: Helmholtz, lambda = 10
    "helm32_gsrb_v": ("8 32 32 32 8 v gsrb helm 10 sol sol 1 lb 1", True, [1]),
    "helm32_gsrb_n0": ("8 32 32 32 5 v gsrb helm 10 n0 sol 1 lb 0", True, [1, 2, 6]),
    "helm32_gs_c0": ("8 32 32 32 5 v gs helm 10 c0 sol 1 lb 0", True, [1]),
    # §8(f) row 1: variable-coefficient Laplacian / Helmholtz (m_vlaplacian,
    # m_vhelmholtz), eps = (1.5+sin 2pi x)(1.5+sin 2pi y)(1.5+sin 2pi z)
    "vlpl32_gsrb_v": ("8 32 32 32 6 v gsrb vlpl 0 sol sol 1 lb 1", True, [1, 4]),
    "vlpl32_gs_f": ("8 32 32 32 4 f gs vlpl 0 d0 sol 1 lb 0", True, [1]),
    "vhelm32_gsrb_v": ("8 32 32 32 6 v gsrb vhelm 10 sol sol 1 lb 0", True, [1]),
    "vhelm32_gs_n0": ("8 32 32 32 4 v gs vhelm 10 n0 sol 1 lb 0", True, [1]),
    "vlpl_ref2_gs_v": ("8 32 32 32 4 v gs vlpl 0 sol sol 2 lb 0", True, [1, 3]),
    # aniso-Helmholtz (m_ahelmholtz): the reference's 3D smoother is broken
    # (NaN), so only the operator box_ahelmh is pinned: no cycle,
    # the sha256 is that of rhs = L(u) on every box
    "ahelm32_op": ("8 32 32 32 0 v gsrb ahelm 10 sol sol 1 lb 0", True, [1]),
    "ahelm_ref2_op": ("8 32 32 32 0 v gs ahelm 5 sol sol 2 lb 0", True, [1]),
    # C4-like: tests/test_refinement (centre-refined AMR tree)
    # ranks 3 put refinement boundaries across ranks (power-of-two rank counts
    # cut these trees along the octree and never do)
    "ref2_gs_v": ("8 32 32 32 6 v gs lpl 0 sol sol 2 lb 0", True, [1, 3, 4]),
    "ref3_gs_f": ("8 32 32 32 5 f gs lpl 0 sol sol 3 lb 1", True, [1, 3]),
    "ref3_gsrb_v": ("8 32 32 32 5 v gsrb lpl 0 d0 sol 3 lb 0", True, [1, 2, 3, 4]),
    "c4_ref2_box16": ("16 128 128 128 4 v gs lpl 0 sol sol 2 lb 0", True, [1, 3, 4]),
    # the bench's c4_refined configuration itself (bench.py: GSRB, box 16,
    # callback Dirichlet, one refined level): k_gsrb_tile<16> with refinement
    # boundaries and the fused correction + fill on a refined level
    "c4_ref2_box16_gsrb": ("16 128 128 128 4 v gsrb lpl 0 sol sol 2 lb 0", True, [1, 2, 3, 4, 8]),
    # a custom refinement_bnd callback (lb "lbrb": omg_golden.f90's custom_rb,
    # sides_rb's form with other coefficients) on the refined trees: the
    # drop-in runs it on the host after each device fill; at 3 ranks the
    # coarse faces of some refinement boundaries arrive from another rank
    "c4_ref2_box16_gsrb_rb": ("16 128 128 128 4 v gsrb lpl 0 sol sol 2 lbrb 0", True, [1, 3]),
    "ref3_gs_rb": ("8 32 32 32 4 v gs lpl 0 sol sol 3 lbrb 0", True, [1, 3]),
    # a rebuilt tree (lb suffix "mv", omg_golden.f90): n_its iterations, then
    # mg_deallocate_storage, the AMR tree with its refined region moved (same
    # box count, other neighbours / children / ranks / ids order),
    # mg_load_balance (+ _parents), mg_allocate_storage, the problem set up
    # again and n_its more iterations: AMRVAC's regrid
    # (coupling_amrvac/mod_multigrid_coupling.t:116-130,272-351)
    "regrid_ref2_gs": ("8 32 32 32 2 v gs lpl 0 sol sol 2 lbpmv 1", True, [1, 3]),
    "regrid_ref3_gsrb_d0": ("8 32 32 32 2 v gsrb lpl 0 d0 sol 3 lbmv 1", True, [1, 3]),
    "regrid_c4_box16_gsrb": ("16 128 128 128 2 v gsrb lpl 0 sol sol 2 lbpmv 0", True, [1, 3]),
    # §8(f) row 1: m_diffusion — one implicit time step per iteration from
    # phi = u (cycle d1 = backward Euler, d2 = Crank-Nicolson; the lambda
    # field is dt; helm: diffusion_solve with D = 0.5, vhelm: _vcoeff)
    "diff_helm_d1_n0": ("8 32 32 32 4 d1 gsrb helm 0.001 n0 phi 1 lb 0", True, [1, 2]),
    "diff_helm_d2_d0": ("8 32 32 32 4 d2 gsrb helm 0.001 d0 phi 1 lb 0", True, [1]),
    "diff_helm_d2_box16": ("16 64 64 64 2 d2 gsrb helm 0.0001 d0 phi 1 lb 0", True, [1]),
    "diff_helm_d1_ref2": ("8 32 32 32 3 d1 gsrb helm 0.001 n0 phi 2 lb 0", True, [1, 3]),
    "diff_vhelm_d1_per": ("8 32 32 32 3 d1 gsrb vhelm 0.01 per phi 1 lb 0", True, [1, 4]),
    # the reference's error stop "diffusion_solve: no convergence" (10 V-cycles
    # after the FMG without reaching max_res)
    "diff_nonconv_helm_per_ref2": ("8 32 32 32 3 d2 gs helm 0.01 per phi 2 lb 0", False, [1], True),
    "diff_nonconv_vhelm_sol": ("8 32 32 32 3 d2 gs vhelm 0.001 sol phi 1 lb 0", False, [1], True),
}


def read_rank_dumps(fn):
    """The multi-rank dump (omg_golden.f90 dump_phi_rank: <fn>.r<rank>, per
    owned box int32 lvl, int32 position in lvls(lvl)%ids, int32 nc, nc^3
    doubles) in the one-rank file's order: levels lowest first, ids order."""
    boxes = []
    for f in glob.glob(fn + ".r*"):
        b = open(f, "rb").read()
        o = 0
        while o < len(b):
            lvl, n, nc = struct.unpack_from("<3i", b, o)
            o += 12
            boxes.append(((lvl, n), b[o:o + 8 * nc ** 3]))
            o += 8 * nc ** 3
    boxes.sort(key=lambda x: x[0])
    if len(set(k for k, _ in boxes)) != len(boxes):
        raise RuntimeError("a box was dumped by two ranks")
    return b"".join(v for _, v in boxes)


def run(args, ranks, dump, expect_error=False):
    cmd = [os.path.join(REF, "omg_golden")] + args.split() + [dump or "x"]
    if ranks > 1:
        cmd = [MPIEXEC, "-n", str(ranks)] + cmd
    p = subprocess.run(cmd, capture_output=True, text=True)
    out, err = p.stdout, None
    if expect_error:
        assert p.returncode != 0, "expected an error stop"
        for line in (p.stdout + p.stderr).splitlines():
            if "ERROR STOP:" in line:
                err = line.split("ERROR STOP:", 1)[1].strip()
        assert err, p.stderr
    elif p.returncode != 0:
        raise subprocess.CalledProcessError(p.returncode, cmd, p.stdout, p.stderr)
    its, t = [], None
    for line in out.splitlines():
        f = line.split()
        if f and f[0] == "IT":
            its.append({"it": int(f[1]), "err": f[2], "res": f[3], "max_res": f[4]})
        elif f and f[0] == "TIME":
            t = float(f[1])
    return (its, t, err) if expect_error else (its, t)


def main():
    """make_golden.py [name ...]: all configurations, or only the named ones
    (merged into the existing golden.json)."""
    if not os.path.exists(os.path.join(REF, "omg_golden")):
        sys.exit("build the reference first: make -C oracle ref")
    path = os.path.join(HERE, "golden.json")
    only = sys.argv[1:]
    golden = json.load(open(path))["configs"] if only else {}
    for name, spec in CONFIGS.items():
        if only and name not in only:
            continue
        args, dump, ranks = spec[:3]
        expect_error = len(spec) > 3 and spec[3]
        entry = {"args": args, "runs": {}}
        if name in BIG:
            entry["big"] = True
        if args.split()[12].endswith("rb"):
            entry["custom_rb"] = True   # not in the C oracle (tests/test_oracle_golden.py)
        for r in ranks:
            with tempfile.TemporaryDirectory() as td:
                fn = os.path.join(td, "phi.bin") if dump else None
                if expect_error:
                    its, t, err = run(args, r, fn, True)
                    entry["runs"][str(r)] = {"history": its, "error": err}
                    print(name, r, err, file=sys.stderr)
                    continue
                its, t = run(args, r, fn)
                run_entry = {"history": its, "ref_seconds_per_cycle": t}
                if fn:
                    if r == 1:
                        with open(fn, "rb") as f:
                            b = f.read()
                    else:
                        b = read_rank_dumps(fn)
                    key = "rhs_sha256" if " ahelm " in args else "phi_sha256"
                    run_entry[key] = hashlib.sha256(b).hexdigest()
                    run_entry["phi_bytes"] = len(b)
            entry["runs"][str(r)] = run_entry
            print(name, r, its[-1]["err"], its[-1]["res"], file=sys.stderr)
        golden[name] = entry
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "FermiQ/octree-mg @ 2025-06-14, amdflang -O2, MPICH 3.3.2",
                   "configs": golden}, f, indent=1)


if __name__ == "__main__":
    main()
