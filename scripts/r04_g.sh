#!/bin/bash
# Round 4: bench runs with per-run environment, each "ENVSPEC|config|extra bench args"
# (ENVSPEC: comma-separated VAR=value, or "-"), printed one line each; optional GPU test
# selection first (TESTS="file::expr ..." or "file -k expr").
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04g
mkdir -p $OUT
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "PASS|FAIL|Error|error" $OUT/tests.log | tail -40; exit 1; }
  echo "tests: $(tail -1 $OUT/tests.log)"
fi
i=0
IFS=';' read -ra RS <<< "$RUNS"
for r in "${RS[@]}"; do
  i=$((i+1))
  envs=$(echo "$r" | cut -d'|' -f1); cfg=$(echo "$r" | cut -d'|' -f2); extra=$(echo "$r" | cut -d'|' -f3)
  ev=""; [ "$envs" != "-" ] && ev=$(echo "$envs" | tr ',' ' ')
  env $ev timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --steps ${STEPS:-10} --warmup 3 --config $cfg $extra > $OUT/b$i.json 2>> $OUT/bench.err || { echo "bench $r failed"; tail -20 $OUT/bench.err; exit 1; }
  python3 - "$OUT/b$i.json" "$r" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sm = d.get("stage_ms_mean") or d.get("stage_ms_max_over_ranks_mean") or {}
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "k1", (d.get("roofline") or {}).get("k1_avg_ms"),
      "stages", {k: round(v, 3) for k, v in sm.items()}, "emit", d.get("emit"),
      "xchg", d.get("exchange_ms"), "xchg_min", d.get("exchange_ms_min_over_ranks"), "vcap", (d.get("k1_work") or {}).get("vocab_capacity"))
EOF
done
