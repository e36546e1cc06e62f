#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (GPU box):
#   bash scripts/kstats.sh <tag> [bench args]   -> gpurun_out/ks_<tag>/..., table on stdout
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
T=${1:-ks}
shift
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks_$T -o ks -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/ks_$T.log 2>&1 || exit 1
f=$(find $R/gpurun_out/ks_$T -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%8.3f ms total %6d calls %9.1f us avg  %s" % (float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]),
                                                         float(r["AverageNs"]) / 1e3, r["Name"][:90]))
PY
