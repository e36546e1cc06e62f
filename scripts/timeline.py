#!/usr/bin/env python3
"""One run's kernels from a rocprofv3 kernel-trace csv: start (us from the run's first
kernel), duration, the idle gap before it, queue, name.  The run = the kernels from the
second-to-last K1 launch's preceding fill up to the last K1 launch.
    python3 scripts/timeline.py <kernel_trace.csv> [k1 name substring]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    sub = sys.argv[2] if len(sys.argv) > 2 else "k_tokcount"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    k1 = [i for i, r in enumerate(rows) if sub in r["Kernel_Name"]]
    i0, i1 = k1[-2], k1[-1]
    while i0 > 0 and "k_tokcount" not in rows[i0 - 1]["Kernel_Name"] and i0 > k1[-3 if len(k1) > 2 else 0] + 1:
        i0 -= 1
        if "fill" in rows[i0]["Kernel_Name"]:
            break
    seg = rows[i0:i1]
    t0 = int(seg[0]["Start_Timestamp"])
    prev_end, idle = None, 0.0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        if gap > 0:
            idle += gap
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:52]
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} gap {gap:7.1f} q{r['Queue_Id']} {name}")
        prev_end = max(prev_end or 0, e)
    print(f"run span {(prev_end - t0) / 1e3:.1f} us, idle gaps {idle:.1f} us")


if __name__ == "__main__":
    main()
