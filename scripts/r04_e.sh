#!/bin/bash
# Round 4: quick K1 iteration — parity subset per library variant, then bench (c2 unless CFG)
# for each "variant:k1mode" pair of RUNS (variant "" = the product library), alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04e
mkdir -p $OUT
cd $R
RUNS=${RUNS:-":sl :st ent2:sl pers:sl pe2:sl :sl :st ent2:sl pers:sl pe2:sl"}
for v in $(echo $RUNS | tr ' ' '\n' | cut -d: -f1 | sort -u); do
  TFIDF_LIB=$v TFIDF_K1=sl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "golden or variants or long or window or tiny or nul or edge or split or overflow or grouped" > $OUT/tests_$v.log 2>&1 || { echo "variant '$v' FAILED"; tail -30 $OUT/tests_$v.log; exit 1; }
  echo "variant '$v': $(tail -1 $OUT/tests_$v.log)"
done
for r in $RUNS; do
  v=${r%%:*}; k=${r##*:}
  TFIDF_LIB=$v TFIDF_K1=$k timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --steps 20 --warmup 3 --config ${CFG:-c2} > $OUT/bench.json 2>> $OUT/bench.err || { cat $OUT/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('$v:$k', d['value'], d['ms_per_step'], d['roofline']['k1_avg_ms'], d['k1_work']['partial_records'], 'df', d['stage_ms_mean']['df'], 'score', d['stage_ms_mean']['score'])"
done
