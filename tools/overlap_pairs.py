#!/usr/bin/env python3
"""Per-stream-pair overlap of a rocprofv3 kernel trace (tools/overlap_summary
helpers): the share of each row stream's busy time during which the column
stream was busy too, and for each halo stream (the one carrying
k_unpack_faces) how much of its unpacks / blit copies ran under each main
stream's red-black substeps.  usage: overlap_pairs.py <rocprofv3 -d dir>"""
import collections
import csv
import glob
import importlib.util
import os
import sys

spec = importlib.util.spec_from_file_location("ov", os.path.join(os.path.dirname(__file__), "overlap_summary.py"))
ov = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ov)


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    kn = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        kn[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    U = {s: ov.union([(a, b) for a, b, _ in v]) for s, v in kn.items()}
    ss = sorted(U, key=int)
    print("share of the row stream's busy time with the column stream busy (%)")
    print("stream " + " ".join(f"{s:>6s}" for s in ss))
    for a in ss:
        print(f"{a:>6s} " + " ".join(f"{100 * ov.inter(U[a], U[b]) / max(ov.length(U[a]), 1):6.1f}" for b in ss))
    mains = [s for s in ss if any("gsrb_tile" in n for _, _, n in kn[s])]
    for cs in [s for s in ss if any("unpack_faces" in n for _, _, n in kn[s])]:
        unp = ov.union([(a, b) for a, b, n in kn[cs] if "unpack" in n])
        cp = ov.union([(a, b) for a, b, n in kn[cs] if "copyBuffer" in n])
        for ms in mains:
            g = ov.union([(a, b) for a, b, n in kn[ms] if "gsrb_tile" in n])
            print(f"halo stream {cs}: unpacks {ov.length(unp) / 1e3:.0f} us, {100 * ov.inter(unp, g) / max(ov.length(unp), 1):.0f}% "
                  f"under stream {ms}'s substeps; blit copies {ov.length(cp) / 1e3:.0f} us, "
                  f"{100 * ov.inter(cp, g) / max(ov.length(cp), 1):.0f}%")


if __name__ == "__main__":
    main()
