#!/usr/bin/env python3
"""Median per-dispatch value of every counter in a prof_k1.sh output directory.

    python3 scripts/pmc_summary.py gpurun_out/prof_<tag> [kernel-substring]
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    d, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        v2 = v[1:] if len(v) > 1 else v
        print("%-28s %12.4g  (n=%d)" % (k, statistics.median(v2), len(v)))


if __name__ == "__main__":
    main()
