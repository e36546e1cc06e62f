#!/usr/bin/env python3
"""HBM traffic per K1 launch from rocprofv3 PMC passes (scripts/prof_k1.sh output).

traffic = 2 x FETCH_SIZE + WRITE_SIZE per dispatch (KB -> bytes), the gfx950 correction
of MI355X_MICROARCH.md §HBM (FETCH_SIZE reads half the bytes of a wide streaming read;
applied to all reads, so for K1's 16-byte vocabulary gathers it is an upper bound).
Steady-state value = median over the dispatches after the first.

    python3 scripts/traffic_k1.py <prof_dir> <out.json> [<out2.json> ...]
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_launch(prof_dir, counter):
    vals = []
    for f in glob.glob(os.path.join(prof_dir, "p*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "k_tokcount_vs" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        return None
    return statistics.median(vals[1:] if len(vals) > 1 else vals)


def main():
    prof_dir, outs = sys.argv[1], sys.argv[2:]
    fetch = per_launch(prof_dir, "FETCH_SIZE")
    write = per_launch(prof_dir, "WRITE_SIZE")
    doc = {"kernel": "k_tokcount_vs", "fetch_size_kb": fetch, "write_size_kb": write,
           "hbm_bytes_per_launch": None,
           "formula": "2*FETCH_SIZE + WRITE_SIZE (KB*1024); x2 on reads per MI355X_MICROARCH.md §HBM "
                      "(exact for the 16-B streaming corpus reads, an upper bound for the vocabulary gathers)"}
    if fetch is not None and write is not None:
        doc["hbm_bytes_per_launch"] = int((2.0 * fetch + write) * 1024)
    for o in outs:
        os.makedirs(os.path.dirname(os.path.abspath(o)), exist_ok=True)
        with open(o, "w") as f:
            json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
