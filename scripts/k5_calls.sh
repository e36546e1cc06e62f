#!/bin/bash
# Per-call durations of the K5 kernels over a 10-step c2 bench (GPU box): which kernel makes
# the occasional slow score stage.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/k5c -o k5c -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-emit --no-probe > $R/gpurun_out/k5c.log 2>&1 || { tail -5 $R/gpurun_out/k5c.log; exit 1; }
python3 - $(find $R/gpurun_out/k5c -name "*kernel_trace.csv" | head -1) <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    if any(k in n for k in ("k_score", "k_k5", "k_emit_split", "k_idf_of_rank", "k_tokcount_st", "k_df_hist")):
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in d.items():
    print("%-40s %s" % (n[-40:], " ".join("%.0f" % x for x in v)))
PY
