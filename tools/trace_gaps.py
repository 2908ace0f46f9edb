#!/usr/bin/env python3
"""Launch gaps of a rocprofv3 kernel trace: for the windows between
consecutive launches of a marker kernel (one per V-cycle, e.g. the coarse
tail), the window span, the time the GPU had at least one kernel running
(union of kernel intervals), the number of kernels and the idle time between
them.  A span far above the busy time means the cycle is bound by launch
latency / host submission, not by the kernels.
usage: trace_gaps.py run_kernel_trace.csv [marker] [n_windows]"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_coarse_tail"
    nwin = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    print(f"{len(idx)} marker launches; last {nwin} windows")
    for w in range(max(0, len(idx) - nwin - 1), len(idx) - 1):
        a, b = idx[w], idx[w + 1]
        seg = rows[a:b]
        t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
        busy, end = 0, t0
        for r in seg:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if e <= end:
                continue
            busy += e - max(s, end)
            end = e
        print(f"  span {(t1 - t0) / 1e3:8.1f} us  busy {busy / 1e3:8.1f} us  idle {(t1 - t0 - busy) / 1e3:8.1f} us"
              f"  kernels {len(seg):4d}  idle/kernel {(t1 - t0 - busy) / 1e3 / max(1, len(seg)):6.2f} us")


if __name__ == "__main__":
    main()
