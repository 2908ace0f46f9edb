#!/usr/bin/env python3
"""HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, the gfx950 correction) and kernel-
trace duration of the level-1 red-black substep (32768 workgroups, 512^3)
for the builds of tools/archive/r04_pmc_yz.sh: base, yz1 (no y/z ghost pushes), yz3
(no y/z pushes and no y/z ghost loads).  usage: pmc_yz_summary.py <dir>"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    for v in ("base", "yz1", "yz3"):
        tot = {}
        for g in ("FETCH_SIZE", "WRITE_SIZE"):
            vals = [float(r["Counter_Value"])
                    for f in glob.glob(os.path.join(d, f"{v}_{g}", "**", "*counter_collection.csv"), recursive=True)
                    for r in csv.DictReader(open(f))
                    if int(r["Grid_Size"]) // int(r["Workgroup_Size"]) == 32768]
            tot[g] = sum(vals) / len(vals) if vals else 0.0
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
               for f in glob.glob(os.path.join(d, f"{v}_trace", "**", "*kernel_trace.csv"), recursive=True)
               for r in csv.DictReader(open(f))
               if "gsrb_tile" in r["Kernel_Name"] and int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) == 32768]
        rd, wr = tot["FETCH_SIZE"] * 1024 * 2, tot["WRITE_SIZE"] * 1024
        print(f"{v:5s} read {rd / 1e9:.3f} GB, write {wr / 1e9:.3f} GB, total {(rd + wr) / 1e9:.3f} GB per launch; "
              f"{sum(dur) / max(len(dur), 1):.1f} us mean over {len(dur)} launches")


if __name__ == "__main__":
    main()
