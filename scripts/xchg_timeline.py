#!/usr/bin/env python3
"""The DF exchange of the last step of a K-shard run from a rocprofv3 kernel-trace csv:
every kernel from the first k_keys_by_rank (round 5), k_ssb_keys or k_owner_count of the last step to the last k_owner_back, with
its start (us from the first), duration and queue (one queue per rank's stream), then the
summed duration per kernel name.
    python3 scripts/xchg_timeline.py <kernel_trace.csv>"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = next(f for f in ("k_keys_by_rank", "k_ssb_keys", "k_owner_count")
                 if any(f in r["Kernel_Name"] for r in rows))
    kb = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    ob = [i for i, r in enumerate(rows) if "k_owner_back" in r["Kernel_Name"]]
    nr = 8
    i0, i1 = kb[-nr], ob[-1]
    seg = rows[i0:i1 + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    tot = collections.defaultdict(float)
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
        tot[name] += (e - s) / 1e3
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r['Queue_Id']:>3} {name}")
    print(f"span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{v:9.1f} us  {k}")


if __name__ == "__main__":
    main()
