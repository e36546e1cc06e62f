#!/bin/bash
# A/B of environment settings on one box (GPU): alternating bench runs.
#   ENVS="A=1 A=2,B=1" ROUNDS=2 CFG=c2 bash scripts/ab_env.sh   ("-" = no setting)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${ENVS:--}; do
    E=""; [ "$v" != "-" ] && E=$(echo "$v" | tr ',' ' ')
    out=$(env $E timeout -k 10 200 python3 -u bench.py --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline --no-emit --no-probe 2>/dev/null) || { echo "fail $v"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$v', d['value'], d['ms_per_step'], 'k1', s['tokcount'], 'score', s['score'])"
  done
done
