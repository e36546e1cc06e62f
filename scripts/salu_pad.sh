#!/bin/bash
# Is K1's scalar issue a co-bottleneck?  K1 time of timing builds with extra scalar adds
# per token round (GPU box; scripts/k1a_ablate.sh style, kernel-trace averages).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-sp0 sp64}; do
  TFIDF_LIB=$v TFIDF_K1_ABLATE=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sp_$v -o sp -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $R/gpurun_out/sp_$v.log 2>&1 || { echo "fail $v"; tail -5 $R/gpurun_out/sp_$v.log; exit 1; }
  f=$(find $R/gpurun_out/sp_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith("k_tokcount"):
        print(sys.argv[2], r["Name"][:14], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3), "min %.1f" % (float(r["MinNs"]) / 1e3))
PY
done
