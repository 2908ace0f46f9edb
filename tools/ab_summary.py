#!/usr/bin/env python3
"""Average duration per (kernel, grid) over the traces of tools/ab_run.sh.
usage: ab_summary.py [regex]"""
import collections
import csv
import glob
import os
import re
import sys

pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
for d in sorted(glob.glob("gpurun_out/ab/*")):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if not pat.search(k):
                continue
            wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
            acc[(k, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(os.path.basename(d))
    for (k, wg), v in sorted(acc.items(), key=lambda x: -sum(x[1])):
        print(f"  {k[:50]:50s} wg={wg:6d} n={len(v):3d} avg {sum(v)/len(v):8.1f} us")
