#!/usr/bin/env python3
"""Summarise the PMC passes of tools/pmc.sh into one JSON per kernel.

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts
exactly half the bytes of a 16-B-per-lane streaming read, so it is doubled;
the same holds for 8-B-per-lane loads (the block passes', calibrated in
profiles/r06/fetch_calib.txt).  WRITE_SIZE is taken as is (exact for 8-B and
16-B stores, temporal or nt).
usage: pmc_summary.py gpurun_out/pmc_<op> > profiles/<round>/pmc_<op>.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            key = (k, int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
            per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid[key] = r
    out = {}
    for (k, wg), cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"kernel": k, "workgroups": wg, "dispatches": max(len(v) for v in cs.values()),
             "counters_avg": avg}
        if "FETCH_SIZE" in avg:
            e["hbm_read_bytes"] = avg["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in avg:
            e["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        out[f"{k}@{wg}"] = e
    tl = os.path.join(d, "time.log")
    json.dump({"source": d, "time_log": open(tl).read().strip().splitlines()[-1] if os.path.exists(tl) else None,
               "correction": "FETCH_SIZE x2 (gfx950 streaming reads, 16-B and 8-B per lane: profiles/r06/fetch_calib.txt), KiB -> bytes",
               "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
