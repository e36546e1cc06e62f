#!/bin/bash
# Round 6 Y: K1 LDS count table with 4-slot buckets (bw4: one ds_read_b128, four compares,
# 896 buckets) against 8-slot buckets (default); parity tests on bw4 first
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06y
mkdir -p $OUT
cd $R
TFIDF_LIB=bw4 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_bw4.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/tests_bw4.log | tail -20; tail -3 $OUT/tests_bw4.log; exit 1; }
echo "tests bw4: $(tail -1 $OUT/tests_bw4.log)"
run() {   # variant config steps warmup tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; w=d.get('k1_work',{}); print('$2 $1', d['value'], d['ms_per_step'], 'k1', d['roofline']['k1_avg_ms'], 'merge', s['merge'], 'partial', w.get('partial_records'))"
}
for rnd in 1 2 3; do
  for v in default bw4; do run $v c2 20 3 $rnd || exit 1; done
done
for c in c5 c3 c4; do
  for v in default bw4; do run $v $c 3 1 1 || exit 1; done
done
