#!/usr/bin/env python3
"""The launches of the last V-cycle(s) of a rocprofv3 kernel trace in start
order: kernel, workgroups, duration, gap to the previous launch's end.
usage: cycle_seq.py run_kernel_trace.csv [n_last]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    prev_end = None
    for r in rows[-n:]:
        k = r["Kernel_Name"].split("(")[0].replace("void omg::", "").replace("omg::", "")
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e if prev_end is None else max(prev_end, e)
        print(f"{k[:60]:60s} {wg:7d} {(e - s) / 1e3:9.1f} us  gap {gap:7.1f}")


if __name__ == "__main__":
    main()
