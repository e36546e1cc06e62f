#!/bin/bash
# c4 stage times vs the vocabulary table's load limit (GPU box): 45 % (default: 32M slots
# for 9.75M terms) against 70 % (16M slots).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do for l in 45 70; do export TFIDF_VLOAD_BIG=$l;
  out=$(timeout -k 10 200 python3 -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-emit --no-probe 2>/dev/null) || { echo "fail $l"; exit 1; }
  echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vload $l', d['value'], d['k1_work']['vocab_capacity'], d['stage_ms'])"
done; done
