#!/bin/bash
# Round 6 AA: the split DF's main pass counting by the vocabulary's dense index, started
# beside the vocabulary sort (default) against the main pass by term rank after the sort
# (TFIDF_DF_EARLY=0); GPU parity suite first
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06aa
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/tests.log | tail -20; tail -3 $OUT/tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/tests.log)"
run() {   # variant config steps warmup tag
  local E=""; [ $1 != default ] && E=0
  TFIDF_DF_EARLY=$E timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; print('$2 $1', d['value'], d['ms_per_step'], 'vocab', s['vocab'], 'merge', s['merge'], 'df', s['df'], 'order', s['order'], 'score', s['score'])"
}
for rnd in 1 2 3; do
  for v in default late; do run $v c2 20 3 $rnd || exit 1; done
done
for c in c5 c3 c4; do
  for v in default late; do run $v $c 3 1 1 || exit 1; done
done
