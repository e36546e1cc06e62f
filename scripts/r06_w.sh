#!/bin/bash
# Round 6 W: K5 half-wave kernel (documents of 129..512 pairs, two per wave) against the
# committed kernels (k5prev); GPU parity suite first
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06w
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/tests.log | tail -20; tail -3 $OUT/tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/tests.log)"
run() {   # variant config steps warmup tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; print('$2 $1', d['value'], d['ms_per_step'], 'score', s['score'], 'df', s['df'], 'merge', s['merge'])"
}
for rnd in 1 2; do
  for v in default k5prev; do run $v c2 20 3 $rnd || exit 1; done
done
for c in c3 c5 c4; do
  for v in default k5prev; do run $v $c 3 1 1 || exit 1; done
done
