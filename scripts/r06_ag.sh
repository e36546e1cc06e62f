#!/bin/bash
# c4 (V ~ 1e7): K5 idf by df (default past 2^21 ranks: 4-byte df gather + small idf table)
# against idf by rank (idfrank: one 8-byte gather from a 78 MB table); parity on idfrank first
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06ag
mkdir -p $OUT
cd $R
TFIDF_LIB=idfrank timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "c4 or full_config" > $OUT/tests_idfrank.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/tests_idfrank.log | tail -20; tail -3 $OUT/tests_idfrank.log; exit 1; }
echo "tests idfrank: $(tail -1 $OUT/tests_idfrank.log)"
run() {   # variant tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config c4 --steps 5 --warmup 2 > $OUT/c4_$1_$2.json 2> $OUT/c4_$1_$2.err || { echo "bench $1 failed"; tail -5 $OUT/c4_$1_$2.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/c4_$1_$2.json')); s=d['stage_ms_mean']; print('c4 $1', d['value'], d['ms_per_step'], 'score', s['score'], 'df', s['df'], 'merge', s['merge'])"
}
for rnd in 1 2 3; do
  for v in default idfrank; do run $v $rnd || exit 1; done
done
