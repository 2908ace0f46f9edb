#!/usr/bin/env python3
"""Overlap of a rocprofv3 kernel + memory-copy trace, per stream.

For every stream: its kernels' and copies' busy time (union of intervals),
and how much of that time some other stream was busy too.  For the copies
(the loopback halo exchange) and for the comm stream's kernels (unpacks):
the share of their time that ran under another stream's kernels.
usage: overlap_summary.py <rocprofv3 -d dir>"""
import collections
import csv
import glob
import os
import sys


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter(a, b):
    """total length of the intersection of two unions"""
    i = j = 0
    t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            t += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


def length(u):
    return sum(e - s for s, e in u)


def main():
    d = sys.argv[1]
    kern = collections.defaultdict(list)
    names = collections.defaultdict(collections.Counter)
    copies = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            st = r.get("Stream_Id") or r.get("Queue_Id")
            kern[st].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            names[st][r["Kernel_Name"].split("(")[0].split("<")[0]] += 1
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            st = r.get("Stream_Id") or "copy"
            copies[st].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    ku = {s: union(v) for s, v in kern.items()}
    print(f"{'stream':>8s} {'kernels':>8s} {'busy us':>10s} {'under other streams %':>22s}  top kernels")
    for s in sorted(ku, key=lambda x: -length(ku[x])):
        others = union([iv for t, u in ku.items() if t != s for iv in u])
        b = length(ku[s])
        ov = inter(ku[s], others)
        top = ", ".join(f"{k} x{n}" for k, n in names[s].most_common(4))
        print(f"{s:>8s} {len(kern[s]):8d} {b / 1e3:10.1f} {100 * ov / max(b, 1):21.1f}%  {top}")
    allk = union([iv for u in ku.values() for iv in u])
    for s, v in sorted(copies.items()):
        cu = union(v)
        b = length(cu)
        print(f"copies on stream {s}: {len(v)} copies, {b / 1e3:.1f} us busy, "
              f"{100 * inter(cu, allk) / max(b, 1):.1f}% of it under kernels")
    if not copies:
        print("no memory-copy records (same-device copies may run as blit kernels: see the kernel rows)")


if __name__ == "__main__":
    main()
