#!/bin/bash
# Round 5: host overhead of the per-run idf table (c2 step vs device time; c5 / c3 8 shards),
# then the c4 A/B of tokcount_sl over the 32M-slot table (TFIDF_SL_MAXCAP) against tokcount_vs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05d
mkdir -p $OUT
cd $R
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --steps 20 --warmup 3 > $OUT/c2_$i.json 2> $OUT/c2_$i.err || { tail -20 $OUT/c2_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c2_$i.json')); print('c2', d['value'], d['ms_per_step'], d['device_ms_per_step'], d['roofline']['k1_avg_ms'], d['idf'])"
done
for c in c5 c3; do
  timeout -k 10 600 python3 bench.py --shards 8 --steps 3 --warmup 1 --no-cpu-baseline --no-probe --no-emit --config $c > $OUT/shards8_$c.json 2> $OUT/shards8_$c.err || { echo "shards $c failed"; tail -20 $OUT/shards8_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shards8_$c.json')); print('shards8 $c', d['value'], d['ms_per_step'], d.get('exchange_ms_min_over_ranks'))"
done
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config c3 --steps 5 --warmup 2 > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c3.json')); print('c3', d['value'], d['ms_per_step'], d['device_ms_per_step'], d['stage_ms_mean']['idf'], d['idf'])"
[ -n "$TESTK" ] && { timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTK" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error" $OUT/gpu_tests.log | tail -20; exit 1; }; echo "tests: $(tail -1 $OUT/gpu_tests.log)"; }
