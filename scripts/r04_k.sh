#!/bin/bash
# Round 4: counters + kernel trace of the default c2 path (r04_h.sh), the end-to-end CLI on
# c2 files (ingest_bench.py), and the single-GPU benches of the other configs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-r04k}
mkdir -p $OUT
cd $R
if [ -z "$SKIP_PMC" ]; then
  TAG=${TAG:-r04k}_pmc KRE="k_tokcount_sl|k_df_hist_lds|k_score_wave" CFG=c2 bash scripts/r04_h.sh > $OUT/pmc.txt 2>&1 || { echo "PMC FAILED"; tail -20 $OUT/pmc.txt; exit 1; }
  echo "pmc done"
fi
if [ -z "$SKIP_CLI" ]; then
  cd $R && timeout -k 10 600 python3 scripts/ingest_bench.py --config c2 > $OUT/cli_c2.json 2> $OUT/cli_c2.err || { echo "CLI FAILED"; tail -20 $OUT/cli_c2.err; exit 1; }
  echo "cli: $(cut -c1-900 $OUT/cli_c2.json)"
fi
cd $R
for c in ${CFGS:-c4 c5 c3}; do
  timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-probe --steps ${STEPS:-10} --warmup 3 --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "bench $c failed"; tail -20 $OUT/bench_$c.err; exit 1; }
  python3 - "$OUT/bench_$c.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"], "value", d["value"], "ms", d["ms_per_step"], "k1", d["roofline"]["k1_avg_ms"],
      "stages", d["stage_ms_mean"])
EOF
done
