#!/usr/bin/env python3
"""HBM traffic per K1 launch from rocprofv3 PMC passes (scripts/prof_k1.sh output), stored
per config in profiles/k1_pmc_traffic.json, the table bench.py's roofline.traffic reads.

traffic = 2 x FETCH_SIZE + WRITE_SIZE per dispatch (KB -> bytes), the gfx950 correction
of MI355X_MICROARCH.md §HBM (FETCH_SIZE reads half the bytes of a wide streaming read;
applied to all reads, so for K1's 16-byte vocabulary gathers it is an upper bound).
Steady-state value = median over the dispatches after the first.  Each entry carries the
digest of the K1 source it was measured on (bench.py ignores an entry of another source).

    python3 scripts/traffic_k1.py <prof_dir> <key> <table.json> [<copy.json> ...]
      key: bench.py's key of the run (c2, c4, c5, c3_strong_g8 ...)
"""
import csv
import glob
import hashlib
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = {"k_tokcount_sl": "tokcount_sl.hip", "k_tokcount_vs": "tokcount_vs.hip", "k_tokcount": "tokcount.hip"}


def k1_source_sha(kernel) -> str:
    with open(os.path.join(REPO, "parallel-systems-mpi-tfidf_amd", "csrc", SOURCES[kernel]), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def kernel_of(name):
    """k_tokcount_sl / k_tokcount_vs / k_tokcount from a demangled kernel name"""
    for k in ("k_tokcount_sl", "k_tokcount_vs"):
        if k in name:
            return k
    return "k_tokcount" if "k_tokcount(" in name else None


def per_launch(prof_dir, counter):
    """median per-dispatch value of `counter` over the dispatches of the K1 kernel the run
    ended on (the steady state: a config whose first runs grow the vocabulary table may
    start on another K1 kernel), and that kernel"""
    recs = []
    for f in glob.glob(os.path.join(prof_dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kernel_of(r["Kernel_Name"])
            if k and r["Counter_Name"] == counter:
                recs.append((int(r.get("Dispatch_Id", 0) or 0), k, float(r["Counter_Value"])))
    if not recs:
        return None, None
    recs.sort()
    kern = recs[-1][1]
    vals = [v for _, k, v in recs if k == kern]
    return statistics.median(vals[1:] if len(vals) > 1 else vals), kern


def main():
    prof_dir, key, table, copies = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
    fetch, kern = per_launch(prof_dir, "FETCH_SIZE")
    write, _ = per_launch(prof_dir, "WRITE_SIZE")
    kern = kern or "k_tokcount_sl"
    e = {"kernel": kern, "k1_source_sha": k1_source_sha(kern), "fetch_size_kb": fetch, "write_size_kb": write,
         "hbm_bytes_per_launch": None, "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({key})",
         "formula": "2*FETCH_SIZE + WRITE_SIZE (KB*1024); x2 on reads per MI355X_MICROARCH.md §HBM "
                    "(exact for the 16-B streaming corpus reads, an upper bound for the vocabulary gathers)"}
    if fetch is not None and write is not None:
        e["hbm_bytes_per_launch"] = int((2.0 * fetch + write) * 1024)
    tab = {}
    if os.path.exists(table):
        with open(table) as f:
            old = json.load(f)
        if isinstance(old, dict) and "kernel" not in old:
            tab = old
    tab[key] = e
    for o in [table] + copies:
        os.makedirs(os.path.dirname(os.path.abspath(o)), exist_ok=True)
        with open(o, "w") as f:
            json.dump(tab, f, indent=1)
    print(key, json.dumps(e))


if __name__ == "__main__":
    main()
