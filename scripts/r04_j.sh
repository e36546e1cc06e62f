#!/bin/bash
# Round 4: full GPU test suite + smoke + default bench (c2) + 8-shard exchange benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${TAG:-r04j}
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error" $OUT/tests.log | tail -30; tail -5 $OUT/tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/tests.log)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
echo "smoke: $(tail -1 $OUT/smoke.log)"
timeout -k 10 600 python3 bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "bench failed"; tail -20 $OUT/bench_c2.err; exit 1; }
tail -1 $OUT/bench_c2.json | cut -c1-600
for c in ${SHARD_CFGS:-c5 c4 c3}; do
  timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
  python3 - "$OUT/shards8_$c.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["workload"], "value", d["value"], "ms", d["ms_per_step"], "xchg", d.get("exchange_ms"),
      "xchg_min", d.get("exchange_ms_min_over_ranks"), "frac", d.get("exchange_frac_of_step"), "mode", d.get("exchange_mode"))
EOF
done
