#!/bin/bash
# Split-K1 ablation timing (GPU box; results invalid by design): kernel-trace averages of
# k_tok_resolve / k_count_slots per diagnostic build lib/libtfidf_hip_<V>.so.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  if [ "$v" = "base" ]; then L=""; else L="$v"; fi
  TFIDF_LIB=$L TFIDF_K1_ABLATE=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abl_$v -o abl -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe > $R/gpurun_out/abl_$v.log 2>&1 || { echo "fail $v"; tail -5 $R/gpurun_out/abl_$v.log; exit 1; }
  f=$(find $R/gpurun_out/abl_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("k_tok_resolve", "k_count_slots", "k_tokcount")):
        print(sys.argv[2], r["Name"][:14], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3), "min %.1f" % (float(r["MinNs"]) / 1e3))
PY
done
