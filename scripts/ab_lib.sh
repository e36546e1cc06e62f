#!/bin/bash
# A/B of library builds on one box (GPU): alternating bench runs, K1 and total per run.
#   VARIANTS="base vflat" ROUNDS=3 CFG=c2 bash scripts/ab_lib.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = "base" ]; then L=""; else L="$v"; fi
    out=$(TFIDF_LIB=$L timeout -k 10 200 python3 -u bench.py --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline --no-emit --no-probe 2>/dev/null) || { echo "fail $v"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$v', d['value'], 'k1', s['tokcount'], 'score', s['score'], 'df', s['df'])"
  done
done
