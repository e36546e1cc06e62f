#!/bin/bash
# stream priorities: the main stream (merge chain, score) above stream2 (the DF main pass
# beside the merge chain), against equal priorities (default); parity on prio first
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r06ah
mkdir -p $OUT
cd $R
TFIDF_LIB=prio timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_prio.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAIL|Error|assert" $OUT/tests_prio.log | tail -20; tail -3 $OUT/tests_prio.log; exit 1; }
echo "tests prio: $(tail -1 $OUT/tests_prio.log)"
run() {   # variant config steps warmup tag
  local L=""; [ $1 != default ] && L=$1
  TFIDF_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --no-emit --config $2 --steps $3 --warmup $4 > $OUT/$2_$1_$5.json 2> $OUT/$2_$1_$5.err || { echo "bench $2 $1 failed"; tail -5 $OUT/$2_$1_$5.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$2_$1_$5.json')); s=d['stage_ms_mean']; print('$2 $1', d['value'], d['ms_per_step'], 'k1', d['roofline']['k1_avg_ms'], 'merge', s['merge'], 'df', s['df'], 'score', s['score'])"
}
for rnd in 1 2 3 4; do
  for v in default prio; do run $v c2 20 3 $rnd || exit 1; done
done
for rnd in 1 2; do
  for v in default prio; do run $v c5 5 2 $rnd || exit 1; done
done
for c in c4 c3; do
  for v in default prio; do run $v $c 3 1 1 || exit 1; done
done
grep -h "stream priorities" $OUT/*.err | head -1
cd /tmp && export TMPDIR=/tmp
TFIDF_LIB=prio timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-emit --no-probe --config c2 > $OUT/kt.log 2>&1 || { echo "trace failed"; tail -5 $OUT/kt.log; exit 1; }
F=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/timeline.py $F > $OUT/timeline_c2_prio.txt && grep -E "df_hist|rs_scatter|part_merge|score_wave|span" $OUT/timeline_c2_prio.txt
