#!/usr/bin/env python3
"""Device allocations inside bench.py's timed steps, from a rocprofv3 --hip-trace
--kernel-trace run (GPU box):  python3 scripts/alloc_trace.py DIR WARMUP STEPS

The timed region starts at the first K1 launch after the WARMUP untimed runs and ends
with the last kernel of the last timed step's K1 + its stages (the end of the last K1 of
the STEPS timed runs plus everything enqueued before the next hipMalloc-free host phase is
approximated by the last kernel before the emission kernels of the untimed emission
measurement).  Prints every hipMalloc/hipFree/hipMallocAsync/hipFreeAsync call with its
time relative to the timed region, and the count inside it."""
import csv
import glob
import sys

d, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
kern, api = [], []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    kern += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    api += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in csv.DictReader(open(f))]
kern.sort()
api.sort()
k1 = [k for k in kern if "k_tokcount" in k[2]]
runs = warm + steps
if len(k1) < runs:
    print(f"only {len(k1)} K1 launches, expected {runs}")
    sys.exit(1)
t_first = k1[warm][0]                   # first timed K1
# end of the timed region: the last kernel that starts before the first emission kernel
# after the last timed K1 (bench.py formats the last step's lines after timing)
t_last_k1 = k1[runs - 1][0]
after = [k for k in kern if k[0] > t_last_k1]
emit = [k for k in after if "emit" in k[2] or "term_meta" in k[2] or "format" in k[2]]
t_end = max(k[1] for k in after if not emit or k[0] < emit[0][0]) if after else k1[runs - 1][1]
alloc = [a for a in api if a[2] in ("hipMalloc", "hipFree", "hipMallocAsync", "hipFreeAsync", "hipExtMallocWithFlags",
                                    "hipHostMalloc", "hipHostFree", "hipMallocManaged")]
inside = [a for a in alloc if t_first <= a[0] <= t_end]
print(f"K1 launches {len(k1)}, timed region {t_first} .. {t_end} ({(t_end - t_first) / 1e6:.3f} ms)")
print(f"allocation calls: {len(alloc)} in the whole process, {len(inside)} inside the timed region")
by = {}
for a in alloc:
    where = "before" if a[0] < t_first else ("inside" if a[0] <= t_end else "after")
    by[(a[2], where)] = by.get((a[2], where), 0) + 1
for (fn, where), n in sorted(by.items()):
    print(f"  {fn:24s} {where:7s} {n}")
for a in inside:
    print("  INSIDE:", a[2], (a[0] - t_first) / 1e3, "us after the first timed K1")
