#!/usr/bin/env python3
"""Per kernel and grid size, from the PMC passes of tools/archive/r04_c4_pmc.sh:
waves, the GPU-busy clock (GRBM_GUI_ACTIVE, summed over the 8 XCDs),
SQ_BUSY_CYCLES, the mean resident waves (SQ_WAVE_CYCLES, quad-cycles, x4
/ GRBM_GUI_ACTIVE per XCD), the share of wave time waiting (SQ_WAIT_ANY /
SQ_WAVE_CYCLES), HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, the gfx950
correction of tools/pmc_summary.py), and the kernel's share of all busy
clocks.  usage: pmc_occupancy.py <dir with p*/ passes>"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("omg::", "")
            key = (k, int(r["Grid_Size"]) // int(r["Workgroup_Size"]), int(r["Workgroup_Size"]))
            per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    tot = 0.0
    for key, cs in per.items():
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        g = a.get("GRBM_GUI_ACTIVE", 0.0)
        tot += g * n
        rows.append((key, n, a))
    rows.sort(key=lambda x: -x[2].get("GRBM_GUI_ACTIVE", 0.0) * x[1])
    print(f"{'kernel':44s} {'WGs':>6s} {'thr':>4s} {'calls':>5s} {'waves':>7s} {'GUI_ACT/XCD':>11s} "
          f"{'SQ_BUSY':>9s} {'mean waves/XCD':>14s} {'wait %':>6s} {'HBM KB':>8s} {'% busy':>6s}")
    for (k, wg, th), n, a in rows:
        g = a.get("GRBM_GUI_ACTIVE", 0.0)
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        occ = 4 * wc / g if g else 0.0   # g sums 8 XCDs, so this is per XCD
        wait = 100 * a.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0
        hbm = (2 * a.get("FETCH_SIZE", 0.0) + a.get("WRITE_SIZE", 0.0))
        print(f"{k[:44]:44s} {wg:6d} {th:4d} {n:5d} {a.get('SQ_WAVES', 0):7.0f} {g / 8:11.0f} "
              f"{a.get('SQ_BUSY_CYCLES', 0):9.0f} {occ:14.1f} {wait:6.1f} {hbm:8.0f} {100 * g * n / tot:6.1f}")


if __name__ == "__main__":
    main()
