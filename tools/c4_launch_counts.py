"""Per-rank launch counts of one C4 V-cycle (bench.py's c4_refined tree:
test_refinement's 128^3 base, box 16, one refined level, GSRB, callback
Dirichlet) on N loopback ranks of one GPU, by kernel family and level
(omg_set_profiling / omg_kernel_stats).  Shows which fused kernels run on
split levels: smooth_resid (the last down-substep + residual + restriction),
prolong_smooth (correction + fill + first up-substep), fill_crhs.

    python tools/c4_launch_counts.py [ranks]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.mgdriver import run_loopback  # noqa: E402

C4_ARGS = "16 128 128 128 1 v gsrb lpl 0 sol sol 2 lb 0"
FAMILIES = ["smoother_gsrb", "smooth_resid", "resid_restrict", "prolong_smooth", "prolong_fill", "fill_gc",
            "fill_crhs", "coarse_rhs", "coarse_tail", "face_gc", "residual", "restrict", "prolong"]


def main():
    ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 4

    def body(be, rank, reduce):
        mg = be.mg
        c = mg.ctx
        from tests.mgdriver import omg
        omg.mg_fas_vcycle(mg)            # warm: the stand-alone fill state settles
        c.call("synchronize")
        c.call("reset_stats")
        c.call("set_profiling", 1)
        omg.mg_fas_vcycle(mg)
        c.call("synchronize")
        c.call("set_profiling", 0)
        out = {}
        for lvl in range(mg.lowest_lvl, mg.highest_lvl + 1):
            for f in FAMILIES:
                n = c.kernel_stats(f"{f}@{lvl}")[0]
                if n:
                    out[(f, lvl)] = n
        return out

    res = run_loopback(C4_ARGS, ranks, body)
    keys = sorted(set(k for r in res for k in r), key=lambda k: (-k[1], k[0]))
    print(f"C4 (one V-cycle after one warm-up), {ranks} loopback ranks: launches per rank")
    print("%-16s %5s " % ("family", "level") + " ".join("r%-3d" % r for r in range(ranks)))
    for k in keys:
        print("%-16s %5d " % k + " ".join("%-4d" % res[r].get(k, 0) for r in range(ranks)))
    tot = [sum(r.values()) for r in res]
    print("%-16s %5s " % ("total", "") + " ".join("%-4d" % t for t in tot))


if __name__ == "__main__":
    main()
