#!/bin/bash
# Round 4: the multi-rank GPU tests, then 8-shard exchange benches (CFGS, default c3 c5),
# EXTRA env per bench run (e.g. TFIDF_XCHG=dense_table for the table numbering).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04x
mkdir -p $OUT
cd $R
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > $OUT/mr.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/mr.log | tail -20; tail -3 $OUT/mr.log; exit 1; }
  echo "tests: $(tail -1 $OUT/mr.log)"
fi
for run in ${RUNS:-"-:c3" "-:c5" "TFIDF_XCHG=dense_table:c3" "TFIDF_XCHG=dense_table:c5"}; do
  e=${run%%:*}; c=${run##*:}; tag=$(echo "$e" | tr -c 'a-zA-Z0-9\n' '_')
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_${c}_$tag.json 2> $OUT/shards8_${c}_$tag.err || { echo "shards $c $e failed"; tail -20 $OUT/shards8_${c}_$tag.err; exit 1; }
  echo "$c [$e]: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['exchange_ms'], d['exchange_ms_min_over_ranks'], d['exchange_mode'])" $OUT/shards8_${c}_$tag.json)"
done
if [ -n "$KT_C4" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c4x8 -o kt -- python3 $R/bench.py --shards 8 --steps 2 --warmup 1 --config c4 --no-cpu-baseline --no-probe --no-emit > $OUT/kt_c4x8.log 2>&1 || { echo "trace failed"; exit 1; }
  echo "c4 x8 trace done"
fi
