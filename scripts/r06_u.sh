#!/bin/bash
# Round 6 U: DF loop with the next iteration's record loads sent right after this
# iteration's rank gathers (two register sets): default = 16 records per lane (the wide
# instance spills 24 VGPRs), dfd14 / dfd12 = 14 / 12 (no spills), dfprev = the committed loop
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06u
mkdir -p $OUT
cd $R
run() {   # variant config steps warmup tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; print('$2 $1', d['value'], d['ms_per_step'], 'merge', s['merge'], 'df', s['df'], 'score', s['score'])"
}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bin_overflow or wide_form or df_split or vocabulary_boundary or full_config or golden" > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -5 $OUT/tests.log; exit 1; }
echo "tests: $(tail -1 $OUT/tests.log)"
for rnd in 1 2; do
  for v in default dfd14 dfd12 dfprev; do run $v c2 20 3 $rnd || exit 1; done
done
for v in default dfd14 dfd12 dfprev; do run $v c3 3 1 1 || exit 1; done
for v in dfd14 dfprev; do run $v c5 10 2 1 || exit 1; done
