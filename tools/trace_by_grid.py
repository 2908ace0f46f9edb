#!/usr/bin/env python3
"""Average duration per (kernel, workgroup count) over a whole rocprofv3
kernel trace.  rocprofv3 --stats averages every launch of a kernel name,
which mixes the levels of the V-cycle (the same smoother runs at 32,768,
4,096, 512, ... workgroups); this splits them, so the finest-level launches
can be compared with bench.py's HIP-event roofline.
usage: trace_by_grid.py run_kernel_trace.csv [regex]"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void omg::", "").replace("omg::", "")
        if not pat.search(k):
            continue
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        acc[(k, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':48s} {'workgroups':>10s} {'launches':>8s} {'avg us':>9s} {'min us':>9s} {'max us':>9s}")
    for (k, wg), v in sorted(acc.items(), key=lambda x: -sum(x[1])):
        print(f"{k[:48]:48s} {wg:10d} {len(v):8d} {sum(v) / len(v):9.1f} {min(v):9.1f} {max(v):9.1f}")


if __name__ == "__main__":
    main()
