#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 rocpd database (run_results.db): calls, total ms,
average us, sorted by total time.   python3 scripts/rocpd_stats.py <db> [top] [> out.csv]"""
import sqlite3
import sys


def short(name):
    """the kernel's name without return type, namespace and parameter list"""
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):   # cut at the parameter list's '(' (outside template brackets)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i][:90]
    return n[:90]


def main():
    db, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                     "order by sum(duration) desc").fetchall()
    print("Name,Calls,TotalDurationNs,AverageNs")
    for name, n, tot, avg in rows[:top]:
        print(f"\"{short(name)}\",{n},{int(tot)},{avg:.1f}")


if __name__ == "__main__":
    main()
