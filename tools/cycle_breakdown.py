#!/usr/bin/env python3
"""Kernel time of one V-cycle from a rocprofv3 kernel trace: the window
between two consecutive launches of a marker kernel (default: the fused rhs
subtract that opens every stand-alone cycle), summed per (kernel, grid).
usage: cycle_breakdown.py run_kernel_trace.csv [marker] [which-from-end]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_box_sums3<16, true"
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[-back], idx[-back + 1]
    seg = rows[a:b]
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    d = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        k = (r["Kernel_Name"].split("(")[0].replace("void omg::", "").replace("omg::", ""), wg)
        d[k][0] += 1
        d[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"cycle span {(t1 - t0) / 1e3:.1f} us, {len(seg)} kernels, busy {sum(v[1] for v in d.values()) / 1e3:.1f} us")
    for (k, wg), (n, t) in sorted(d.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k[:44]:44s} wg={wg:6d} x{n:3d} {t / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
