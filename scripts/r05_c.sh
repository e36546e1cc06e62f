#!/bin/bash
# Round 5: A/B of K1 library variants on c2 (VARIANTS, ROUNDS), then optionally the GPU suite
# (TESTS=1) and the comm_init deadline diagnostic (DIAG=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r05c
mkdir -p $OUT
cd $R
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-not nothing}" > $OUT/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|error" $OUT/gpu_tests.log | tail -30; exit 1; }
  echo "tests: $(tail -1 $OUT/gpu_tests.log)"
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    L=$v; [ $v = base ] && L=""
    EV=""; case $v in env:*) L=""; EV=${v#env:}; EV=${EV//,/ };; esac   # env:NAME=VALUE[,NAME=VALUE] = the product library with those settings
    env TFIDF_LIB=$L $EV timeout -k 10 200 python3 -u bench.py --config ${CFG:-c2} --steps 10 --warmup 2 --no-cpu-baseline --no-emit --no-probe > $OUT/ab.json 2>$OUT/ab.err || { echo "fail $v"; tail -5 $OUT/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/ab.json')); s=d['stage_ms_mean']; print('$v', d['value'], 'k1', s['tokcount'], 'score', s['score'], 'df', s['df'], 'merge', s['merge'], 'vocab', s['vocab'])"
  done
done
if [ "${DIAG:-0}" = 1 ]; then
  TFIDF_DEBUG_COMM=1 TFIDF_COMM_TIMEOUT_S=3 timeout -k 5 40 python3 -u scripts/r05_diag_init.py > $OUT/diag_init.log 2>&1
  echo "diag_init rc=$?"; grep -E "^ *[0-9]+\.[0-9]+ |tfidf:" $OUT/diag_init.log | tail -8
fi
