#!/bin/bash
# Round 5: df counted in K1's slot space (TFIDF_DF_K1=1: the DF pass counts only the merged
# records, K5 maps K1's records' slots to ranks).  GPU parity suite under the setting first
# (TESTK), then the c2 / c4 A/B against the default (CFGS, ROUNDS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05e
mkdir -p $OUT
cd $R
if [ -n "$TESTK" ]; then
  TFIDF_DF_K1=1 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTK" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error" $OUT/gpu_tests.log | tail -30; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
fi
for c in ${CFGS:-c2}; do
  for r in $(seq 1 ${ROUNDS:-2}); do
    for v in ${VARIANTS:-base env:TFIDF_DF_K1=1}; do
      EV=""; case $v in env:*) EV=${v#env:};; esac
      [ $c = c4 ] && EV="$EV TFIDF_SL_MAXCAP=${C4_MAXCAP:-33554432}"
      env $EV timeout -k 10 300 python3 -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-emit --no-probe > $OUT/ab.json 2>$OUT/ab.err || { echo "fail $c $v"; tail -5 $OUT/ab.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/ab.json')); s=d['stage_ms_mean']; print('$c', '$v', d['value'], 'k1', s['tokcount'], 'score', s['score'], 'df', s['df'], 'merge', s['merge'], 'vocab', s['vocab'])"
    done
  done
done
