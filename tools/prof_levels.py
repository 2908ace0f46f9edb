#!/usr/bin/env python3
"""Per-(kernel, grid size) summary of a rocprofv3 --kernel-trace CSV.

rocprofv3's own --stats table averages a kernel over every level it ran on;
the grid size separates the levels (one workgroup per box for the tiled
kernels), so this table is the one the bench's per-level figures compare to.
usage: prof_levels.py run_kernel_trace.csv [min_total_us]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        d[(r["Kernel_Name"].split("(")[0], wg)].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'kernel':58s} {'workgroups':>10s} {'calls':>6s} {'avg_us':>9s} {'total_us':>10s}")
    for (k, wg), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        if sum(v) / 1e3 < min_us:
            continue
        print(f"{k[:58]:58s} {wg:10d} {len(v):6d} {sum(v) / len(v) / 1e3:9.1f} {sum(v) / 1e3:10.1f}")


if __name__ == "__main__":
    main()
